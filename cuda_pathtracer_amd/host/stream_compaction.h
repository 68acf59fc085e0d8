// C++ host mirror of the reference's StreamCompaction interface, backed by the C ABI in
// include/sc_amd.h (libpt_amd.so).  Same names, argument meaning and error behaviour as
//   path_tracer/stream_compaction/efficient.h:5-13   (Efficient::timer / scan / compact)
//   path_tracer/stream_compaction/common.h:46-130    (Common::PerformanceTimer)
//   path_tracer/stream_compaction/cpu.h:7-14         (CPU::timer / scan / compactWithoutScan / compactWithScan)
//   path_tracer/stream_compaction/naive.h:7-10       (Naive::timer / scan)
//   path_tracer/stream_compaction/thrust.h:7-10      (Thrust::timer / scan)
//   path_tracer/stream_compaction/common.cu:3-15     (checkCUDAError: print and exit(1))
// Only Efficient is on the path tracer's hot path; the other three let the reference's self-test
// (stream_compaction/src/main.cpp) compare the four implementations.  CPU:: runs the library's
// own host loops (sc_cpu_*), not the test oracle.
//
// Pointers may be host or device memory, like the reference (pathtrace.cu:397 hands device
// pointers to Efficient::scan through UVA): device pointers run on the null stream without
// staging, host pointers are staged through the library's cached device buffers.
#pragma once

#include <chrono>
#include <stdexcept>

namespace StreamCompaction {
namespace Common {

// PerformanceTimer (common.h:46-130): CPU timing with std::chrono; the GPU time of the previous
// Efficient operation is measured by the library with hipEvents around the device work.
class PerformanceTimer {
public:
    PerformanceTimer() = default;
    void startCpuTimer() {
        if (cpu_timer_started) throw std::runtime_error("CPU timer already started");
        cpu_timer_started = true;
        time_start_cpu = std::chrono::high_resolution_clock::now();
    }
    void endCpuTimer() {
        const auto end = std::chrono::high_resolution_clock::now();
        if (!cpu_timer_started) throw std::runtime_error("CPU timer not started");
        prev_cpu_ms = std::chrono::duration<float, std::milli>(end - time_start_cpu).count();
        cpu_timer_started = false;
    }
    void setGpuElapsed(float ms) { prev_gpu_ms = ms; }
    float getCpuElapsedTimeForPreviousOperation() { return prev_cpu_ms; }
    float getGpuElapsedTimeForPreviousOperation() { return prev_gpu_ms; }
    PerformanceTimer(const PerformanceTimer&) = delete;
    PerformanceTimer(PerformanceTimer&&) = delete;
    PerformanceTimer& operator=(const PerformanceTimer&) = delete;
    PerformanceTimer& operator=(PerformanceTimer&&) = delete;

private:
    std::chrono::high_resolution_clock::time_point time_start_cpu;
    bool cpu_timer_started = false;
    float prev_cpu_ms = 0.f;
    float prev_gpu_ms = 0.f;
};

}  // namespace Common

namespace CPU {
StreamCompaction::Common::PerformanceTimer& timer();
// Exclusive scan on the host (wrapping int32); odata may equal idata.
void scan(int n, int* odata, const int* idata);
// The non-zero elements of idata in order; returns how many.
int compactWithoutScan(int n, int* odata, const int* idata);
// Map to 0/1, exclusive scan, scatter; returns how many were kept.
int compactWithScan(int n, int* odata, const int* idata);
}  // namespace CPU

namespace Naive {
StreamCompaction::Common::PerformanceTimer& timer();
// Hillis & Steele exclusive scan on the device (ceil(log2 n) launches, then the shift).
void scan(int n, int* odata, const int* idata);
}  // namespace Naive

namespace Thrust {
StreamCompaction::Common::PerformanceTimer& timer();
// rocThrust's exclusive_scan.
void scan(int n, int* odata, const int* idata);
}  // namespace Thrust

namespace Efficient {
StreamCompaction::Common::PerformanceTimer& timer();
// Exclusive scan (wrapping int32) of idata[0..n) into odata.  Any n >= 0.
void scan(int n, int* odata, const int* idata);
// Keeps the non-zero elements of idata in order; returns how many were kept.
int compact(int n, int* odata, const int* idata);
}  // namespace Efficient

}  // namespace StreamCompaction
