// tools/pinned_bw.cpp — host CPU bandwidth on page-locked memory from hipHostMalloc against
// malloc'd memory (reads, writes, and the 16-B -> 20-B record widening of the host pipeline),
// on N threads.   pinned_bw [MB] [threads]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

struct Rec { uint32_t a, b, c, d, e; };

template <typename F>
static double timed(int T, F f) {
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++) th.emplace_back(f, t);
    for (auto& x : th) x.join();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

int main(int argc, char** argv) {
    const size_t mb = argc > 1 ? std::atoi(argv[1]) : 256;
    const int T = argc > 2 ? std::atoi(argv[2]) : 8;
    const size_t n = mb << 20;
    const size_t nrec = n / 20;
    for (int pinned = 0; pinned < 2; pinned++) {
        uint8_t *src = nullptr, *dst = nullptr;
        if (pinned) {
            if (hipHostMalloc((void**)&src, n, hipHostMallocDefault) != hipSuccess || hipHostMalloc((void**)&dst, n + n / 4, hipHostMallocDefault) != hipSuccess)
                return 1;
        } else {
            src = (uint8_t*)std::aligned_alloc(4096, n);
            dst = (uint8_t*)std::aligned_alloc(4096, n + n / 4);
        }
        std::memset(src, 1, n);
        std::memset(dst, 0, n + n / 4);
        volatile uint64_t sink = 0;
        const double tr = timed(T, [&](int t) {
            const uint64_t* p = (const uint64_t*)src;
            uint64_t s = 0;
            for (size_t i = n / 8 * t / T; i < n / 8 * (t + 1) / T; i++) s += p[i];
            sink += s;
        });
        const double tw = timed(T, [&](int t) {
            std::memset(dst + n * t / T, 2, n * (t + 1) / T - n * t / T);
        });
        const size_t nr = n / 16;
        const double tx = timed(T, [&](int t) {
            const uint32_t* r = (const uint32_t*)src;
            Rec* o = (Rec*)dst;
            for (size_t i = nr * t / T; i < nr * (t + 1) / T && i < nrec; i++)
                o[i] = Rec{(uint32_t)i, r[4 * i], r[4 * i + 1], r[4 * i + 2], r[4 * i + 3]};
        });
        std::printf("{\"memory\": \"%s\", \"threads\": %d, \"MB\": %zu, \"read_GBs\": %.1f, \"write_GBs\": %.1f, \"widen16to20_Mrec_s\": %.1f}\n",
                    pinned ? "hipHostMalloc" : "malloc", T, mb, n / tr / 1e9, n / tw / 1e9, std::min(nr, nrec) / tx / 1e6);
        if (pinned) { (void)hipHostFree(src); (void)hipHostFree(dst); }
        else { std::free(src); std::free(dst); }
    }
    return 0;
}
