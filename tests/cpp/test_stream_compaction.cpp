// C++ restatement of the reference's own stream-compaction self-test
// (stream_compaction/src/main.cpp:14-146 + testing_helpers.hpp) against the C++ host mirror
// (cuda_pathtracer_amd/host/stream_compaction.h -> libpt_amd.so).  The expected values come
// from the CPU oracle (oracle/sc_oracle.cpp, test infrastructure), and all four namespaces of the
// mirror (CPU, Naive, Efficient, Thrust) are checked against it: b = expected, c = result,
// printCmpResult after each case.  Exit status != 0 on any
// mismatch.  Inputs are seeded (the reference uses time()).
//
//   test_stream_compaction [SIZE_LOG2=20]
#include <execinfo.h>
#include <unistd.h>

#include <csignal>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <random>
#include <vector>

// the reference self-test's include block, as stream_compaction/src/main.cpp:2-5 writes it
// (forwarding headers cuda_pathtracer_amd/host/stream_compaction/*.h; built with -I host only)
#include <stream_compaction/cpu.h>
#include <stream_compaction/naive.h>
#include <stream_compaction/efficient.h>
#include <stream_compaction/thrust.h>

extern "C" {   // oracle/sc_oracle.cpp (CPU::scan / compactWithoutScan / compactWithScan)
void oracle_scan(int64_t n, int32_t* out, const int32_t* in);
int64_t oracle_compact_without_scan(int64_t n, int32_t* out, const int32_t* in);
int64_t oracle_compact_with_scan(int64_t n, int32_t* out, const int32_t* in);
}

namespace {

int g_failures = 0;

void genArray(int n, int* a, int maxval, std::mt19937& rng) {   // testing_helpers.hpp genArray
    std::uniform_int_distribution<int> d(0, maxval - 1);
    for (int i = 0; i < n; ++i) a[i] = d(rng);
}
void zeroArray(int n, int* a) { std::memset(a, 0, sizeof(int) * (size_t)n); }
void printDesc(const char* desc) { std::printf("==== %s ====\n", desc); }
int cmpArrays(int n, const int* a, const int* b) {
    for (int i = 0; i < n; ++i)
        if (a[i] != b[i]) {
            std::printf("    a[%d] = %d, b[%d] = %d\n", i, a[i], i, b[i]);
            return 1;
        }
    return 0;
}
void printCmpResult(int n, const int* a, const int* b) {
    const int bad = cmpArrays(n, a, b);
    std::printf("    %s \n", bad ? "FAIL VALUE" : "passed");
    g_failures += bad;
}
void printCmpLenResult(int n, int expN, const int* a, const int* b) {
    const int bad = (n != expN) ? 1 : cmpArrays(n, a, b);
    if (n != expN) std::printf("    expected %d elements, got %d\n", expN, n);
    std::printf("    %s \n", bad ? "FAIL VALUE" : "passed");
    g_failures += bad;
}
void printElapsedTime(float ms, const char* note) { std::printf("   elapsed time: %.4fms    %s\n", ms, note); }

}  // namespace

void on_fault(int sig) {   // print where a crash happened (stdout is unbuffered below)
    void* frames[64];
    const int n = backtrace(frames, 64);
    std::fprintf(stderr, "signal %d, backtrace:\n", sig);
    backtrace_symbols_fd(frames, n, 2);
    _exit(128 + sig);
}

int main(int argc, char** argv) {
    std::setvbuf(stdout, nullptr, _IONBF, 0);
    std::signal(SIGSEGV, on_fault);
    std::signal(SIGABRT, on_fault);
    const int lg = argc > 1 ? std::atoi(argv[1]) : 20;
    const int SIZE = 1 << lg;
    const int NPOT = SIZE - 3;
    std::vector<int> av(SIZE), bv(SIZE), cv(SIZE);
    int *a = av.data(), *b = bv.data(), *c = cv.data();
    std::mt19937 rng(0x5EED);
    using namespace StreamCompaction;

    std::printf("\n****************\n** SCAN TESTS **\n****************\n");
    genArray(SIZE - 1, a, 50, rng);   // leave a 0 at the end to test that edge case
    a[SIZE - 1] = 0;
    zeroArray(SIZE, b);
    oracle_scan(SIZE, b, a);

    zeroArray(SIZE, c);
    printDesc("work-efficient scan, power-of-two");
    Efficient::scan(SIZE, c, a);
    printElapsedTime(Efficient::timer().getGpuElapsedTimeForPreviousOperation(), "(HIP Measured)");
    printCmpResult(SIZE, b, c);

    oracle_scan(NPOT, b, a);
    zeroArray(SIZE, c);
    printDesc("work-efficient scan, non-power-of-two");
    Efficient::scan(NPOT, c, a);
    printElapsedTime(Efficient::timer().getGpuElapsedTimeForPreviousOperation(), "(HIP Measured)");
    printCmpResult(NPOT, b, c);

    // the other three namespaces (main.cpp:31-85), each against the oracle
    for (int npot = 0; npot < 2; ++npot) {
        const int n = npot ? NPOT : SIZE;
        oracle_scan(n, b, a);
        const char* tag = npot ? "non-power-of-two" : "power-of-two";
        char desc[96];
        zeroArray(SIZE, c);
        std::snprintf(desc, sizeof desc, "cpu scan, %s", tag);
        printDesc(desc);
        CPU::scan(n, c, a);
        printElapsedTime(CPU::timer().getCpuElapsedTimeForPreviousOperation(), "(std::chrono Measured)");
        printCmpResult(n, b, c);
        zeroArray(SIZE, c);
        std::snprintf(desc, sizeof desc, "naive scan, %s", tag);
        printDesc(desc);
        Naive::scan(n, c, a);
        printElapsedTime(Naive::timer().getGpuElapsedTimeForPreviousOperation(), "(HIP Measured)");
        printCmpResult(n, b, c);
        zeroArray(SIZE, c);
        std::snprintf(desc, sizeof desc, "thrust scan, %s", tag);
        printDesc(desc);
        Thrust::scan(n, c, a);
        printElapsedTime(Thrust::timer().getGpuElapsedTimeForPreviousOperation(), "(HIP Measured)");
        printCmpResult(n, b, c);
    }
    for (int n : {1, 2, 3, 5, 64, 65, 1000}) {   // naive: ceil(log2 n) passes, odd and even
        if (n > SIZE) continue;
        oracle_scan(n, b, a);
        zeroArray(n, c);
        Naive::scan(n, c, a);
        char desc[64];
        std::snprintf(desc, sizeof desc, "naive scan, n = %d", n);
        printDesc(desc);
        printCmpResult(n, b, c);
    }

    // small sizes the reference's padded scan could not do
    for (int n : {1, 2, 3, 7, 64, 65, 8191, 8193}) {
        if (n > SIZE) continue;
        oracle_scan(n, b, a);
        zeroArray(n, c);
        Efficient::scan(n, c, a);
        char desc[64];
        std::snprintf(desc, sizeof desc, "work-efficient scan, n = %d", n);
        printDesc(desc);
        printCmpResult(n, b, c);
    }

    std::printf("\n*****************************\n** STREAM COMPACTION TESTS **\n*****************************\n");
    genArray(SIZE - 1, a, 4, rng);
    a[SIZE - 1] = 0;
    zeroArray(SIZE, b);
    const int expectedCount = (int)oracle_compact_without_scan(SIZE, b, a);
    const int expectedNPOT = (int)oracle_compact_without_scan(NPOT, c, a);
    {   // the oracle's two CPU variants agree (cpu.cu:40-79)
        std::vector<int> w(SIZE);
        const int k = (int)oracle_compact_with_scan(SIZE, w.data(), a);
        printDesc("cpu compact with scan == without scan");
        printCmpLenResult(k, expectedCount, b, w.data());
    }
    std::vector<int> bn(c, c + SIZE);
    for (int npot = 0; npot < 2; ++npot) {   // CPU::compactWithoutScan / compactWithScan (main.cpp:103-126)
        const int n = npot ? NPOT : SIZE;
        const int* expect = npot ? bn.data() : b;
        const int ecount = npot ? expectedNPOT : expectedCount;
        std::vector<int> w(SIZE, 0);
        printDesc(npot ? "cpu compact without scan, non-power-of-two" : "cpu compact without scan, power-of-two");
        int k = CPU::compactWithoutScan(n, w.data(), a);
        printElapsedTime(CPU::timer().getCpuElapsedTimeForPreviousOperation(), "(std::chrono Measured)");
        printCmpLenResult(k, ecount, expect, w.data());
        std::fill(w.begin(), w.end(), 0);
        printDesc(npot ? "cpu compact with scan, non-power-of-two" : "cpu compact with scan, power-of-two");
        k = CPU::compactWithScan(n, w.data(), a);
        printElapsedTime(CPU::timer().getCpuElapsedTimeForPreviousOperation(), "(std::chrono Measured)");
        printCmpLenResult(k, ecount, expect, w.data());
    }

    zeroArray(SIZE, c);
    printDesc("work-efficient compact, power-of-two");
    int count = Efficient::compact(SIZE, c, a);
    printElapsedTime(Efficient::timer().getGpuElapsedTimeForPreviousOperation(), "(HIP Measured)");
    printCmpLenResult(count, expectedCount, b, c);

    zeroArray(SIZE, c);
    printDesc("work-efficient compact, non-power-of-two");
    count = Efficient::compact(NPOT, c, a);
    printElapsedTime(Efficient::timer().getGpuElapsedTimeForPreviousOperation(), "(HIP Measured)");
    printCmpLenResult(count, expectedNPOT, bn.data(), c);

    std::printf("\n%s (%d failure(s))\n", g_failures ? "FAILED" : "ALL PASSED", g_failures);
    return g_failures ? 1 : 0;
}
