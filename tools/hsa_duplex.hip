// Both PCIe directions at once on SDMA engines chosen explicitly (hsa_amd_memory_async_copy_on_engine),
// each direction driven by its own host thread, as the search_lines pipeline would: the HIP
// runtime otherwise tends to put H2D and D2H copies on one engine, which serves them in turn.
//   hsa_duplex [MB per copy] [copies]
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <thread>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            std::exit(2);                                                      \
        }                                                                      \
    } while (0)
#define HK(x)                                                                  \
    do {                                                                       \
        hsa_status_t s_ = (x);                                                 \
        if (s_ != HSA_STATUS_SUCCESS) {                                        \
            const char* m_ = nullptr;                                          \
            hsa_status_string(s_, &m_);                                        \
            std::fprintf(stderr, "%s: %s\n", #x, m_ ? m_ : "?");               \
            std::exit(3);                                                      \
        }                                                                      \
    } while (0)

struct Agents { hsa_agent_t gpu{}, cpu{}; bool have_gpu = false, have_cpu = false; };
static hsa_status_t find_agents(hsa_agent_t a, void* d) {
    Agents* A = static_cast<Agents*>(d);
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU && !A->have_gpu) { A->gpu = a; A->have_gpu = true; }
    if (t == HSA_DEVICE_TYPE_CPU && !A->have_cpu) { A->cpu = a; A->have_cpu = true; }
    return HSA_STATUS_SUCCESS;
}
__global__ void k_tiny(uint32_t* p) { if (threadIdx.x == 0) p[blockIdx.x] += 1; }

static double now_ms() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
    const size_t bytes = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 48) << 20;
    const int ncopies = argc > 2 ? std::atoi(argv[2]) : 6;
    CK(hipSetDevice(0));
    void *hin, *hout, *din, *dout;
    uint32_t* dt;
    CK(hipHostMalloc(&hin, bytes, hipHostMallocDefault));
    CK(hipHostMalloc(&hout, bytes, hipHostMallocDefault));
    CK(hipMalloc(&din, bytes));
    CK(hipMalloc(&dout, bytes));
    CK(hipMalloc(&dt, 4096));
    CK(hipMemset(dout, 1, bytes));
    CK(hipDeviceSynchronize());
    Agents A;
    HK(hsa_iterate_agents(find_agents, &A));
    uint32_t m_up = 0, m_down = 0, r_up = 0, r_down = 0;
    HK(hsa_amd_memory_copy_engine_status(A.gpu, A.cpu, &m_up));
    HK(hsa_amd_memory_copy_engine_status(A.cpu, A.gpu, &m_down));
    (void)hsa_amd_memory_get_preferred_copy_engine(A.gpu, A.cpu, &r_up);
    (void)hsa_amd_memory_get_preferred_copy_engine(A.cpu, A.gpu, &r_down);
    std::printf("{\"engines_h2d_mask\": \"0x%x\", \"engines_d2h_mask\": \"0x%x\", \"preferred_h2d\": \"0x%x\", \"preferred_d2h\": \"0x%x\"}\n", m_up, m_down,
                r_up, r_down);
    auto run = [&](bool up, hsa_amd_sdma_engine_id_t eng, int n) {
        hsa_signal_t sig;
        HK(hsa_signal_create(1, 0, nullptr, &sig));
        for (int i = 0; i < n; i++) {
            hsa_signal_store_relaxed(sig, 1);
            if (up) HK(hsa_amd_memory_async_copy_on_engine(din, A.gpu, hin, A.cpu, bytes, 0, nullptr, sig, eng, true));
            else HK(hsa_amd_memory_async_copy_on_engine(hout, A.cpu, dout, A.gpu, bytes, 0, nullptr, sig, eng, true));
            hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
        }
        HK(hsa_signal_destroy(sig));
    };
    struct Shape { const char* name; int up_eng, down_eng; };
    // engine ids: bit positions (0: direction not run)
    const Shape shapes[] = {{"h2d_e0", 0x1, 0}, {"d2h_e0", 0, 0x1}, {"h2d_e0+d2h_e0", 0x1, 0x1}, {"h2d_e0+d2h_e1", 0x1, 0x2},
                            {"h2d_e1+d2h_e0", 0x2, 0x1}, {"h2d_e2+d2h_e3", 0x4, 0x8}};
    hipStream_t cs;
    CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    for (const Shape& sh : shapes) {
        if ((sh.up_eng && !(m_up & sh.up_eng)) || (sh.down_eng && !(m_down & sh.down_eng))) {
            std::printf("{\"shape\": \"%s\", \"skipped\": \"engine not available\"}\n", sh.name);
            continue;
        }
        double best = 1e30, chain = 0;
        for (int rep = 0; rep < 3; rep++) {
            CK(hipDeviceSynchronize());
            const double t0 = now_ms();
            std::thread tu, td;
            if (sh.up_eng) tu = std::thread(run, true, (hsa_amd_sdma_engine_id_t)sh.up_eng, ncopies);
            if (sh.down_eng) td = std::thread(run, false, (hsa_amd_sdma_engine_id_t)sh.down_eng, ncopies);
            // tiny kernels beside the copies
            hipEvent_t a, b;
            CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
            CK(hipEventRecord(a, cs));
            for (int t = 0; t < 32; t++) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, cs, dt);
            CK(hipEventRecord(b, cs));
            if (tu.joinable()) tu.join();
            if (td.joinable()) td.join();
            const double t1 = now_ms();
            CK(hipEventSynchronize(b));
            float mc = 0;
            CK(hipEventElapsedTime(&mc, a, b));
            if (t1 - t0 < best) { best = t1 - t0; chain = mc; }
        }
        const double moved = (double)bytes * ncopies * ((sh.up_eng ? 1 : 0) + (sh.down_eng ? 1 : 0));
        std::printf("{\"shape\": \"%s\", \"MB_per_copy\": %zu, \"copies\": %d, \"ms\": %.3f, \"GBps\": %.1f, \"chain32_ms\": %.3f}\n", sh.name, bytes >> 20,
                    ncopies, best, moved / best / 1e6, chain);
        std::fflush(stdout);
    }
    return 0;
}
