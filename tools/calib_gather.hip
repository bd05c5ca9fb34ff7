// Calibration of the access shape the search kernels use: each lane gathers one random
// 64-B rank block (the OccBlock of kernels.h) from a table of a given size.
//
//   calib_gather [table_MB ...]          prints one JSON line per (shape, table size)
//
// Shapes: "gather16"   — one random 16-B load per lane and iteration (a rank entry, rent1/rent2:
//                        the deep kernels' load; FETCH_SIZE / TCC_EA0_RDREQ_DRAM_32B per load
//                        under --pmc calibrate the counters for this shape);
//         "gather64"   — one random 64-B block per lane (4 × 16-B loads, the rank query);
//         "gather128"  — one random 128-B line per lane (8 × 16-B loads);
//         "stream16"   — coalesced 16-B-per-lane streaming read of the whole table (the
//                        shape MI355X_MICROARCH.md calibrates FETCH_SIZE on);
//         "stream4"    — coalesced 4-B-per-lane streaming read (the item arrays' shape);
//         "chainK_wW"  — the deep walk's shape (k_deep_fast): every lane walks patterns of
//                        8 dependent steps, each step one random 16-B load per interval end
//                        (K = 1 or 2 loads issued together) whose address depends on the
//                        previous step's values; W = waves per SIMD the launch is held to
//                        (dynamic LDS), so the ceiling is measured at a kernel's occupancy.
//   calib_gather --chain [table_MB ...]   runs only the chain shapes
//   calib_gather --tlb [table_MB ...]     gather16 with 64-bit indices over tables up to 128 GB: the
//                        rate of random 16-B loads as the table outgrows the GPU's address translation
//                        caches (the wide k-mer table is 34 GB at C3)
//   calib_gather --scatter [table_MB ...] random 16-B stores (the per-pattern result writes)
//   calib_gather --window [table_MB ...]  one 16-B load per random 64-B block within a window that
//                        slides over the table (row-bucketed items): accesses/s per window size
// Algorithmic bytes are known exactly, so running this under
// `rocprofv3 --pmc FETCH_SIZE` gives the FETCH_SIZE → bytes factor for each shape, and the
// timed rate is the practical ceiling of the rank-block gathers (vs HBM peak 8 TB/s).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <string>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            std::exit(2);                                                            \
        }                                                                            \
    } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// each lane: `iters` random blocks of LINES16 × 16 B
template <int LINES16>
__global__ void __launch_bounds__(256) k_gather(const uint4* __restrict__ t, uint32_t nblk, uint32_t iters, uint32_t seed,
                                                uint32_t* __restrict__ sink) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t h = mix(g ^ seed), acc = 0;
    for (uint32_t i = 0; i < iters; i++) {
        h = mix(h + i);
        const uint4* p = t + (size_t)(h % nblk) * LINES16;
        uint4 v[LINES16];
#pragma unroll
        for (int k = 0; k < LINES16; k++) v[k] = p[k];
#pragma unroll
        for (int k = 0; k < LINES16; k++) acc ^= v[k].x + v[k].y + v[k].z + v[k].w;
    }
    if (acc == 0x12345678u) sink[g] = acc;  // keeps the loads alive; never true in practice
}

// gather16 over a table of n16 16-B entries (n16 may exceed 2^32)
__global__ void __launch_bounds__(256) k_gather16w(const uint4* __restrict__ t, uint64_t n16, uint32_t iters, uint32_t seed,
                                                   uint32_t* __restrict__ sink) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t h = mix(g ^ seed), acc = 0;
    for (uint32_t i = 0; i < iters; i++) {
        h = mix(h + i);
        const uint64_t x = ((uint64_t)mix(h ^ 0x9e3779b9u) << 32 | h) % n16;
        const uint4 v = t[x];
        acc ^= v.x + v.y + v.z + v.w;
    }
    if (acc == 0x12345678u) sink[g] = acc;
}

static void tlb(size_t mb, uint32_t* sink, hipEvent_t a, hipEvent_t b) {
    const size_t bytes = mb << 20;
    uint4* t;
    CK(hipMalloc(&t, bytes));
    CK(hipMemset(t, 7, bytes));
    const uint32_t grid = 256 * 32, block = 256, iters = 64;
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_gather16w, dim3(grid), dim3(block), 0, 0, t, (uint64_t)(bytes / 16), iters, 23u + rep, sink);
        CK(hipGetLastError());
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        if (rep > 0 && ms < best) best = ms;
    }
    const double loads = (double)grid * block * iters;
    std::printf("{\"shape\": \"gather16_tlb\", \"table_MB\": %zu, \"loads\": %.0f, \"best_ms\": %.4f, \"loads_per_s\": %.4g}\n", mb,
                loads, best, loads / (best * 1e-3));
    std::fflush(stdout);
    CK(hipFree(t));
}

// random 16-B stores (the deep kernels' per-pattern result writes, Res[o] at input order o): under
// --pmc TCC_EA0_RDREQ_sum / TCC_EA0_WRREQ_sum they show whether a partial-line store costs a DRAM read
__global__ void __launch_bounds__(256) k_scatter16(uint4* __restrict__ t, uint64_t n16, uint32_t iters, uint32_t seed) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t h = mix(g ^ seed);
    for (uint32_t i = 0; i < iters; i++) {
        h = mix(h + i);
        const uint64_t x = ((uint64_t)mix(h ^ 0x9e3779b9u) << 32 | h) % n16;
        t[x] = make_uint4(h, g, i, seed);
    }
}

static void scatter(size_t mb, hipEvent_t a, hipEvent_t b) {
    const size_t bytes = mb << 20;
    uint4* t;
    CK(hipMalloc(&t, bytes));
    CK(hipMemset(t, 7, bytes));
    const uint32_t grid = 256 * 32, block = 256, iters = 64;
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_scatter16, dim3(grid), dim3(block), 0, 0, t, (uint64_t)(bytes / 16), iters, 31u + rep);
        CK(hipGetLastError());
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        if (rep > 0 && ms < best) best = ms;
    }
    const double stores = (double)grid * block * iters;
    std::printf("{\"shape\": \"scatter16\", \"table_MB\": %zu, \"stores\": %.0f, \"launches\": 5, \"best_ms\": %.4f, \"stores_per_s\": %.4g}\n",
                mb, stores, best, stores / (best * 1e-3));
    std::fflush(stdout);
    CK(hipFree(t));
}

// the deep walk's access shape: per lane, patterns of `steps` dependent steps; each step
// issues K independent random 16-B loads (the two interval ends) and the next step's
// addresses depend on the loaded values
template <int K>
__global__ void __launch_bounds__(256) k_chain(const uint4* __restrict__ t, uint32_t n16, uint32_t pats, uint32_t steps, uint32_t seed,
                                               uint32_t* __restrict__ sink) {
    extern __shared__ uint32_t hold[];  // occupancy limiter only
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (uint32_t p = 0; p < pats; p++) {
        uint32_t h[K];
#pragma unroll
        for (int k = 0; k < K; k++) h[k] = mix(g * 2654435761u ^ (seed + p * 7919u + k * 104729u));
        for (uint32_t s = 0; s < steps; s++) {
            uint4 v[K];
#pragma unroll
            for (int k = 0; k < K; k++) v[k] = t[h[k] % n16];
#pragma unroll
            for (int k = 0; k < K; k++) h[k] = mix(h[k] ^ v[k].x ^ v[k].w);
        }
#pragma unroll
        for (int k = 0; k < K; k++) acc ^= h[k];
    }
    if (acc == 0x12345678u) { sink[g] = acc; hold[threadIdx.x] = acc; }
}

// bucketed gathers: access i (grid-stride order, so the lanes in flight hold neighbouring i)
// reads one random 64-B block (one 16-B load of it: the rank query's first half) within a
// window of `wblk` blocks that slides over the table as i grows — items partitioned by row
// bucket and stepped bucket after bucket.  wblk = nblk: fully random.
__global__ void __launch_bounds__(256) k_gather_win(const uint4* __restrict__ t, uint32_t nblk, uint64_t n, uint32_t wblk, uint32_t seed,
                                                    uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    const uint32_t nwin = nblk / wblk;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t w = (uint32_t)(i * nwin / n);
        const uint32_t h = mix((uint32_t)i ^ seed);
        const uint4 v = t[((size_t)w * wblk + h % wblk) * 4];
        acc ^= v.x + v.w;
    }
    if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

__global__ void __launch_bounds__(256) k_stream4(const uint32_t* __restrict__ t, size_t n4, uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) acc ^= t[i];
    if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

__global__ void __launch_bounds__(256) k_stream(const uint4* __restrict__ t, size_t n16, uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = t[i];
        acc ^= v.x + v.y + v.z + v.w;
    }
    if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

static void chains(const std::vector<size_t>& mbs, uint32_t* sink, hipEvent_t a, hipEvent_t b) {
    const uint32_t block = 256, steps = 8;
    int cus = 256;
    {
        hipDeviceProp_t pr;
        if (hipGetDeviceProperties(&pr, 0) == hipSuccess) cus = pr.multiProcessorCount;
    }
    for (size_t mb : mbs) {
        const size_t bytes = mb << 20;
        uint4* t;
        CK(hipMalloc(&t, bytes));
        CK(hipMemset(t, 3, bytes));
        for (int K = 1; K <= 2; K++)
            for (int waves : {2, 4, 6, 8}) {
                // waves per SIMD = blocks per CU (a 256-thread block is one wave per SIMD)
                const size_t lds = (160u * 1024u) / (size_t)waves - 256;
                const uint32_t grid = (uint32_t)cus * (uint32_t)waves * 4, pats = 16;
                float best = 1e30f;
                for (int rep = 0; rep < 4; rep++) {
                    CK(hipEventRecord(a));
                    if (K == 1) hipLaunchKernelGGL(k_chain<1>, dim3(grid), dim3(block), lds, 0, t, (uint32_t)(bytes / 16), pats, steps, 5u + rep, sink);
                    else hipLaunchKernelGGL(k_chain<2>, dim3(grid), dim3(block), lds, 0, t, (uint32_t)(bytes / 16), pats, steps, 5u + rep, sink);
                    CK(hipGetLastError());
                    CK(hipEventRecord(b));
                    CK(hipEventSynchronize(b));
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, a, b));
                    if (rep > 0 && ms < best) best = ms;
                }
                const double loads = (double)grid * block * pats * steps * K;
                std::printf("{\"shape\": \"chain%d_w%d\", \"table_MB\": %zu, \"loads_16B\": %.0f, \"best_ms\": %.4f, "
                            "\"lines_per_s\": %.4g, \"dependent_steps_per_s\": %.4g}\n",
                            K, waves, mb, loads, best, loads / (best * 1e-3), loads / K / (best * 1e-3));
                std::fflush(stdout);
            }
        CK(hipFree(t));
    }
}

static void windows(size_t mb, uint32_t* sink, hipEvent_t a, hipEvent_t b) {
    const size_t bytes = mb << 20;
    uint4* t;
    CK(hipMalloc(&t, bytes));
    CK(hipMemset(t, 5, bytes));
    const uint32_t nblk = (uint32_t)(bytes / 64);
    const uint64_t n = 1ull << 30;  // accesses per launch
    for (size_t wkb : {(size_t)256, (size_t)512, (size_t)1024, (size_t)2048, (size_t)4096, (size_t)8192, (size_t)16384, (size_t)65536,
                       (size_t)262144, (size_t)0}) {
        const uint32_t wblk = wkb ? (uint32_t)std::min<size_t>(nblk, wkb * 1024 / 64) : nblk;
        float best = 1e30f;
        for (int rep = 0; rep < 4; rep++) {
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(k_gather_win, dim3(256 * 64), dim3(256), 0, 0, t, nblk, n, wblk, 11u + rep, sink);
            CK(hipGetLastError());
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            if (rep > 0 && ms < best) best = ms;
        }
        std::printf("{\"shape\": \"gather_window\", \"table_MB\": %zu, \"window_KB\": %zu, \"accesses\": %llu, \"best_ms\": %.4f, "
                    "\"accesses_per_s\": %.4g}\n", mb, (size_t)wblk * 64 / 1024, (unsigned long long)n, best, n / (best * 1e-3));
        std::fflush(stdout);
    }
    CK(hipFree(t));
}

int main(int argc, char** argv) {
    std::vector<size_t> mbs;
    bool chain_only = false, window_only = false, tlb_only = false, scatter_only = false;
    for (int i = 1; i < argc; i++) {
        if (std::string(argv[i]) == "--chain") chain_only = true;
        else if (std::string(argv[i]) == "--window") window_only = true;
        else if (std::string(argv[i]) == "--tlb") tlb_only = true;
        else if (std::string(argv[i]) == "--scatter") scatter_only = true;
        else {
            char* end = nullptr;
            const unsigned long long v = std::strtoull(argv[i], &end, 10);
            if (!end || *end || v < 16) {  // a table under 16 MB (or not a number) is refused, not launched
                std::fprintf(stderr, "calib_gather: bad table size '%s' (MB, >= 16)\n", argv[i]);
                return 2;
            }
            if (v > 131072) {  // 128 GB at most
                std::fprintf(stderr, "calib_gather: table size '%s' MB too large\n", argv[i]);
                return 2;
            }
            mbs.push_back(v);
        }
    }
    if (mbs.empty()) mbs = {16, 100, 200, 1024, 4096};
    uint32_t* sink;
    const uint32_t grid = 256 * 32, block = 256, iters = 64;
    CK(hipMalloc(&sink, (size_t)grid * block * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    if (tlb_only) {
        for (size_t mb : mbs) tlb(mb, sink, a, b);
        return 0;
    }
    if (scatter_only) {
        for (size_t mb : mbs) scatter(mb, a, b);
        return 0;
    }
    for (size_t mb : mbs)
        if (mb > 16384) {  // the other shapes index with 32 bits
            std::fprintf(stderr, "calib_gather: tables over 16384 MB only with --tlb\n");
            return 2;
        }
    if (window_only) {
        for (size_t mb : mbs) windows(mb, sink, a, b);
        return 0;
    }
    chains(mbs, sink, a, b);
    if (chain_only) return 0;
    for (size_t mb : mbs) {
        const size_t bytes = mb << 20;
        uint4* t;
        CK(hipMalloc(&t, bytes));
        CK(hipMemset(t, 1, bytes));
        for (int shape = 0; shape < 5; shape++) {
            float best = 1e30f;
            double alg = 0;
            for (int rep = 0; rep < 5; rep++) {
                CK(hipEventRecord(a));
                if (shape == 0) {
                    hipLaunchKernelGGL(k_gather<4>, dim3(grid), dim3(block), 0, 0, t, (uint32_t)(bytes / 64), iters, 17u + rep, sink);
                    alg = (double)grid * block * iters * 64;
                } else if (shape == 1) {
                    hipLaunchKernelGGL(k_gather<8>, dim3(grid), dim3(block), 0, 0, t, (uint32_t)(bytes / 128), iters, 17u + rep, sink);
                    alg = (double)grid * block * iters * 128;
                } else if (shape == 2) {
                    hipLaunchKernelGGL(k_stream, dim3(grid), dim3(block), 0, 0, t, bytes / 16, sink);
                    alg = (double)bytes;
                } else if (shape == 4) {
                    hipLaunchKernelGGL(k_gather<1>, dim3(grid), dim3(block), 0, 0, t, (uint32_t)(bytes / 16), iters, 17u + rep, sink);
                    alg = (double)grid * block * iters * 16;
                } else {
                    hipLaunchKernelGGL(k_stream4, dim3(grid), dim3(block), 0, 0, reinterpret_cast<const uint32_t*>(t), bytes / 4, sink);
                    alg = (double)bytes;
                }
                CK(hipGetLastError());
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                if (rep > 0 && ms < best) best = ms;
            }
            const char* nm = shape == 0 ? "gather64" : shape == 1 ? "gather128" : shape == 2 ? "stream16" : shape == 3 ? "stream4" : "gather16";
            std::printf("{\"shape\": \"%s\", \"table_MB\": %zu, \"bytes_per_launch\": %.0f, \"best_ms\": %.4f, \"GBps\": %.1f, "
                        "\"accesses_per_launch\": %.0f, \"launches\": 5}\n", nm, mb, alg, best, alg / best / 1e6,
                        shape == 0 ? alg / 64 : shape == 1 ? alg / 128 : shape == 4 ? alg / 16 : alg / (shape == 2 ? 16 : 4));
            std::fflush(stdout);
        }
        CK(hipFree(t));
    }
    return 0;
}
