// PCIe transfer shapes of the host pipeline (edsbwt_search_lines) on one MI355X:
//   h2d, d2h        hipMemcpyAsync page-locked <-> device, alone
//   both            H2D and D2H on two streams at once (full duplex?)
//   zc_write        a kernel storing to mapped page-locked host memory (records written
//                   straight to the host instead of a D2H copy)
//   zc_read         a kernel loading from mapped page-locked host memory
//   h2d+zc_write    an H2D copy while a kernel writes to host memory
// Prints one JSON line per shape: bytes and GB/s (best of 4).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <string>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            std::exit(2);                                                      \
        }                                                                      \
    } while (0)

__global__ void k_zc_write(uint4* __restrict__ h, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        h[i] = make_uint4((uint32_t)i, 1, 2, 3);
}
__global__ void k_zc_read(const uint4* __restrict__ h, size_t n16, uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = h[i];
        acc ^= v.x + v.w;
    }
    if (acc == 0x1234567u) sink[threadIdx.x] = acc;
}

int main(int argc, char** argv) {
    const size_t bytes = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 256) << 20;
    void *h1, *h2, *d1, *d2;
    uint32_t* sink;
    CK(hipHostMalloc(&h1, bytes, hipHostMallocDefault));
    CK(hipHostMalloc(&h2, bytes, hipHostMallocDefault));
    CK(hipMalloc(&d1, bytes));
    CK(hipMalloc(&d2, bytes));
    CK(hipMalloc(&sink, 4096));
    CK(hipMemset(d1, 1, bytes));
    CK(hipMemset(d2, 2, bytes));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    void* hd2 = nullptr;
    CK(hipHostGetDevicePointer(&hd2, h2, 0));
    void* hd1 = nullptr;
    CK(hipHostGetDevicePointer(&hd1, h1, 0));
    const char* names[] = {"h2d", "d2h", "both", "zc_write", "zc_read", "h2d+zc_write"};
    for (int shape = 0; shape < 6; shape++) {
        double best = 1e30;
        for (int rep = 0; rep < 5; rep++) {
            CK(hipDeviceSynchronize());
            hipEvent_t a, b;
            CK(hipEventCreate(&a));
            CK(hipEventCreate(&b));
            auto t0 = __builtin_readcyclecounter();
            (void)t0;
            CK(hipEventRecord(a, s1));
            CK(hipStreamWaitEvent(s2, a, 0));
            if (shape == 0 || shape == 2 || shape == 5) CK(hipMemcpyAsync(d1, h1, bytes, hipMemcpyHostToDevice, s1));
            if (shape == 1 || shape == 2) CK(hipMemcpyAsync(h2, d2, bytes, hipMemcpyDeviceToHost, s2));
            if (shape == 3 || shape == 5) hipLaunchKernelGGL(k_zc_write, dim3(1024), dim3(256), 0, s2, (uint4*)hd2, bytes / 16);
            if (shape == 4) hipLaunchKernelGGL(k_zc_read, dim3(1024), dim3(256), 0, s2, (const uint4*)hd1, bytes / 16, sink);
            hipEvent_t c;
            CK(hipEventCreate(&c));
            CK(hipEventRecord(c, s2));
            CK(hipStreamWaitEvent(s1, c, 0));
            CK(hipEventRecord(b, s1));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            if (rep > 0 && ms < best) best = ms;
            CK(hipEventDestroy(a));
            CK(hipEventDestroy(b));
            CK(hipEventDestroy(c));
        }
        const double moved = (shape == 2 || shape == 5) ? 2.0 * bytes : (double)bytes;
        std::printf("{\"shape\": \"%s\", \"bytes\": %.0f, \"best_ms\": %.3f, \"GBps\": %.1f}\n", names[shape], moved, best, moved / best / 1e6);
        std::fflush(stdout);
    }
    return 0;
}
