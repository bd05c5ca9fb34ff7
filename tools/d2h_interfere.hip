// How a device -> host download disturbs kernels on another stream (edsbwt_search_lines'
// pipeline: chunk k's records go down while chunk k+1 is searched).  For each kind of
// page-locked destination, a 64 MB hipMemcpyAsync D2H on one stream and, beside it, a chain of
// 32 tiny kernels on another: prints the download time and the chain's time (alone: ~0.1 ms).
//   d2h_interfere [MB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            std::exit(2);                                                      \
        }                                                                      \
    } while (0)

__global__ void k_tiny(uint32_t* p) { if (threadIdx.x == 0) p[blockIdx.x] += 1; }
__global__ void k_out(const uint4* __restrict__ s, uint4* __restrict__ d, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) d[i] = s[i];
}

int main(int argc, char** argv) {
    const size_t bytes = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 64) << 20;
    void *dsrc, *ddst;
    uint32_t* dt;
    CK(hipMalloc(&dsrc, bytes));
    CK(hipMalloc(&ddst, bytes));
    CK(hipMalloc(&dt, 4096));
    CK(hipMemset(dsrc, 1, bytes));
    void* h[5];
    const char* hn[5] = {"hostmalloc_default", "hostmalloc_noncoherent", "host_register", "hostmalloc_mapped_coherent", "none"};
    CK(hipHostMalloc(&h[0], bytes, hipHostMallocDefault));
    CK(hipHostMalloc(&h[1], bytes, hipHostMallocNonCoherent));
    h[2] = std::aligned_alloc(4096, bytes);
    CK(hipHostRegister(h[2], bytes, hipHostRegisterDefault));
    CK(hipHostMalloc(&h[3], bytes, hipHostMallocMapped | hipHostMallocCoherent));
    h[4] = nullptr;
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t a1, b1, a2, b2;
    CK(hipEventCreate(&a1)); CK(hipEventCreate(&b1)); CK(hipEventCreate(&a2)); CK(hipEventCreate(&b2));
    // modes: 0 D2H memcpy into h[k]; 1 H2D memcpy from h[k]; 2 kernel stores into mapped h[k]; 3 D2D
    const char* mn[4] = {"d2h_memcpy", "h2d_memcpy", "d2h_kernel_256blk", "d2d_memcpy"};
    for (int mode = 0; mode < 4; mode++)
        for (int k = 0; k < 5; k++) {
            if ((mode == 3) != (k == 4)) continue;
            void* hp = h[k];
            void* hdev = nullptr;
            if (mode == 2 && hipHostGetDevicePointer(&hdev, hp, 0) != hipSuccess) { (void)hipGetLastError(); continue; }
            double best_copy = 1e30, best_chain = 1e30;
            for (int rep = 0; rep < 5; rep++) {
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(a1, s1));
                if (mode == 0) CK(hipMemcpyAsync(hp, dsrc, bytes, hipMemcpyDeviceToHost, s1));
                if (mode == 1) CK(hipMemcpyAsync(ddst, hp, bytes, hipMemcpyHostToDevice, s1));
                if (mode == 2) hipLaunchKernelGGL(k_out, dim3(256), dim3(256), 0, s1, (const uint4*)dsrc, (uint4*)hdev, bytes / 16);
                if (mode == 3) CK(hipMemcpyAsync(ddst, dsrc, bytes, hipMemcpyDeviceToDevice, s1));
                CK(hipEventRecord(b1, s1));
                CK(hipEventRecord(a2, s2));
                for (int t = 0; t < 32; t++) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s2, dt);
                CK(hipEventRecord(b2, s2));
                CK(hipDeviceSynchronize());
                float m1 = 0, m2 = 0;
                CK(hipEventElapsedTime(&m1, a1, b1));
                CK(hipEventElapsedTime(&m2, a2, b2));
                if (rep > 0) {
                    if (m1 < best_copy) best_copy = m1;
                    if (m2 < best_chain) best_chain = m2;
                }
            }
            std::printf("{\"mode\": \"%s\", \"host\": \"%s\", \"MB\": %zu, \"copy_ms\": %.3f, \"GBps\": %.1f, \"chain32_ms\": %.3f}\n", mn[mode], hn[k],
                        bytes >> 20, best_copy, bytes / best_copy / 1e6, best_chain);
            std::fflush(stdout);
        }
    // what makes hipMemcpyAsync D2H take the blit-kernel path instead of SDMA: destination
    // offset (the pipeline's records land at 20-B multiples), a wait on another stream's event
    {
        const size_t offs[4] = {0, 4, 20, 256};
        for (int w = 0; w < 2; w++)
            for (size_t o : offs) {
                double best_copy = 1e30, best_chain = 1e30;
                for (int rep = 0; rep < 5; rep++) {
                    CK(hipDeviceSynchronize());
                    hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s2, dt);
                    CK(hipEventRecord(a2, s2));
                    if (w) CK(hipStreamWaitEvent(s1, a2, 0));
                    CK(hipEventRecord(a1, s1));
                    CK(hipMemcpyAsync((char*)h[0] + o, dsrc, bytes - 256, hipMemcpyDeviceToHost, s1));
                    CK(hipEventRecord(b1, s1));
                    CK(hipEventRecord(a2, s2));
                    for (int t = 0; t < 32; t++) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s2, dt);
                    CK(hipEventRecord(b2, s2));
                    CK(hipDeviceSynchronize());
                    float m1 = 0, m2 = 0;
                    CK(hipEventElapsedTime(&m1, a1, b1));
                    CK(hipEventElapsedTime(&m2, a2, b2));
                    if (rep > 0) {
                        if (m1 < best_copy) best_copy = m1;
                        if (m2 < best_chain) best_chain = m2;
                    }
                }
                std::printf("{\"mode\": \"d2h_offset\", \"dst_offset\": %zu, \"cross_stream_wait\": %d, \"copy_ms\": %.3f, \"chain32_ms\": %.3f}\n", o, w,
                            best_copy, best_chain);
                std::fflush(stdout);
            }
    }
    // the chain alone
    double best = 1e30;
    for (int rep = 0; rep < 5; rep++) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a2, s2));
        for (int t = 0; t < 32; t++) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s2, dt);
        CK(hipEventRecord(b2, s2));
        CK(hipDeviceSynchronize());
        float m2 = 0;
        CK(hipEventElapsedTime(&m2, a2, b2));
        if (rep > 0 && m2 < best) best = m2;
    }
    std::printf("{\"mode\": \"chain_alone\", \"chain32_ms\": %.3f}\n", best);
    return 0;
}
