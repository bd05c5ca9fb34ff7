// Both PCIe directions at once, as edsbwt_search_lines needs them (chunk k+2 up while chunk
// k-1's records come down), and what each shape does to kernels beside it:
//   sdma_both      hipMemcpyAsync H2D and D2H on two streams (the runtime may put both on one
//                  SDMA engine, which then serves them one after the other)
//   zcread_sdma    H2D as kernel loads from mapped page-locked memory (a CU-masked stream)
//                  while D2H is an SDMA copy
//   zcread_alone   the kernel-load H2D alone
// plus a chain of 32 tiny kernels on a third stream (alone ~0.1 ms).   duplex [MB] [CUs]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            std::exit(2);                                                      \
        }                                                                      \
    } while (0)

__global__ void k_tiny(uint32_t* p) { if (threadIdx.x == 0) p[blockIdx.x] += 1; }
__global__ void __launch_bounds__(256) k_zc_up(const uint4* __restrict__ h, uint4* __restrict__ d, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) d[i] = h[i];
}

int main(int argc, char** argv) {
    const size_t bytes = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 64) << 20;
    const int cus = argc > 2 ? std::atoi(argv[2]) : 32;
    void *hin, *hout, *din, *dout;
    uint32_t* dt;
    CK(hipHostMalloc(&hin, bytes, hipHostMallocDefault));
    CK(hipHostMalloc(&hout, bytes, hipHostMallocDefault));
    CK(hipMalloc(&din, bytes));
    CK(hipMalloc(&dout, bytes));
    CK(hipMalloc(&dt, 4096));
    CK(hipMemset(dout, 1, bytes));
    void* hin_dev = nullptr;
    CK(hipHostGetDevicePointer(&hin_dev, hin, 0));
    hipDeviceProp_t prop{};
    CK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    const int stride = cus > 0 && cus < ncu ? ncu / cus : 1;
    for (int i = 0, got = 0; i < ncu && got < (cus > 0 ? cus : ncu); i++)
        if (i % stride == 0) { mask[i / 32] |= 1u << (i % 32); got++; }
    hipStream_t up, down, comp;
    CK(hipExtStreamCreateWithCUMask(&up, (uint32_t)mask.size(), mask.data()));
    CK(hipStreamCreateWithFlags(&down, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&comp, hipStreamNonBlocking));
    hipEvent_t a, bu, bd, c0, c1;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&bu)); CK(hipEventCreate(&bd)); CK(hipEventCreate(&c0)); CK(hipEventCreate(&c1));
    const char* names[4] = {"sdma_both", "zcread_sdma", "zcread_alone", "sdma_h2d_alone"};
    for (int shape = 0; shape < 4; shape++)
        for (int blocks : {64, 256, 1024}) {
            if (shape == 0 || shape == 3) { if (blocks != 64) continue; }
            double bt = 1e30, bup = 1e30, bdn = 1e30, bch = 1e30;
            for (int rep = 0; rep < 5; rep++) {
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(a, up));
                CK(hipStreamWaitEvent(down, a, 0));
                CK(hipStreamWaitEvent(comp, a, 0));
                if (shape == 0 || shape == 3) CK(hipMemcpyAsync(din, hin, bytes, hipMemcpyHostToDevice, up));
                else hipLaunchKernelGGL(k_zc_up, dim3(blocks), dim3(256), 0, up, (const uint4*)hin_dev, (uint4*)din, bytes / 16);
                CK(hipEventRecord(bu, up));
                if (shape < 2) CK(hipMemcpyAsync(hout, dout, bytes, hipMemcpyDeviceToHost, down));
                CK(hipEventRecord(bd, down));
                CK(hipEventRecord(c0, comp));
                for (int t = 0; t < 32; t++) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, comp, dt);
                CK(hipEventRecord(c1, comp));
                CK(hipDeviceSynchronize());
                float mu = 0, md = 0, mc = 0;
                CK(hipEventElapsedTime(&mu, a, bu));
                CK(hipEventElapsedTime(&md, a, bd));
                CK(hipEventElapsedTime(&mc, c0, c1));
                const double tot = mu > md ? mu : md;
                if (rep > 0 && tot < bt) { bt = tot; bup = mu; bdn = md; bch = mc; }
            }
            const double moved = (shape < 2 ? 2.0 : 1.0) * bytes;
            std::printf("{\"shape\": \"%s\", \"blocks\": %d, \"cus\": %d, \"MB_each\": %zu, \"total_ms\": %.3f, \"up_ms\": %.3f, \"down_ms\": %.3f, "
                        "\"GBps\": %.1f, \"chain32_ms\": %.3f}\n",
                        names[shape], shape == 0 || shape == 3 ? 0 : blocks, cus, bytes >> 20, bt, bup, bdn, moved / bt / 1e6, bch);
            std::fflush(stdout);
        }
    return 0;
}
