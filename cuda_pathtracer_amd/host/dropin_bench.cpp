// The drop-in call sequence, timed: what a reference caller gets from the C++ mirror.
//
// The reference's render loop (path_tracer/src/main.cpp:114-168, runCuda) calls pathtrace() once
// per iteration; pathtrace() re-reads the GUI flags (pathtrace.cu:438-463), traces one sample per
// pixel and copies the accumulated image to the host (pathtrace.cu:524).  host/pathtrace.cpp mirrors
// exactly that (pt_set_flags + pt_render_pass with one iteration + pt_get_image), so this shim only
// loops over it.  bench.py loads it through ctypes (libpt_dropin.so) and reports the rate beside the
// batched-pass value; it is a bench harness, not part of the C ABI in include/.
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>

#include "pathtrace.h"

extern "C" int pt_dropin_bench(const char* scene_path, int warmup, int iters, double* ms, uint64_t* segments,
                               uint64_t* flag_syncs) {
    if (!scene_path || warmup < 0 || iters <= 0 || !ms || !segments) return PT_ERR_ARG;
    // the mirror prints like the reference ("Reading scene from ..."); keep stdout for the bench line
    std::fflush(stdout);
    const int saved = dup(1);
    dup2(2, 1);
    int rc = PT_OK;
    {
        Scene scene(scene_path);
        GuiDataContainer gui;
        InitDataContainer(&gui);
        pathtraceInit(&scene);
        int it = 0;
        for (int k = 0; k < warmup; ++k) pathtrace(nullptr, 0, ++it);
        pt_stats_t s0, s1;
        uint64_t syncs0 = 0, syncs1 = 0;
        if ((rc = pt_stats(pathtraceContext(), &s0)) == PT_OK &&
            (rc = pt_ctx_counters(pathtraceContext(), nullptr, &syncs0)) == PT_OK) {
            const auto t0 = std::chrono::steady_clock::now();
            for (int k = 0; k < iters; ++k) pathtrace(nullptr, 0, ++it);   // ends with a synchronous image copy
            const auto t1 = std::chrono::steady_clock::now();
            *ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
            if ((rc = pt_stats(pathtraceContext(), &s1)) == PT_OK)
                rc = pt_ctx_counters(pathtraceContext(), nullptr, &syncs1);
            *segments = s1.segments - s0.segments;
            if (flag_syncs) *flag_syncs = syncs1 - syncs0;
        }
        InitDataContainer(nullptr);
        pathtraceFree();
    }
    std::fflush(stdout);
    dup2(saved, 1);
    close(saved);
    return rc;
}
