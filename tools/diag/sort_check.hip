// Diagnostic: hipcub radix sort of u64 keys over bits [begin, 64) with u32 values.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <vector>
int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 7, K = argc > 2 ? atoi(argv[2]) : 6, bps = argc > 3 ? atoi(argv[3]) : 4;
    size_t P = 1; for (int t = 0; t < K; t++) P *= B;
    const int spc = 64 / bps;
    std::vector<uint64_t> h(P);
    for (size_t i = 0; i < P; i++) {  // reversed codes of the K-mer i (last char = digit 0), code+1 per symbol
        uint64_t key = 0, x = i;
        for (int t = 0; t < spc; t++) {
            uint64_t v = 0;
            if (t < K) { v = x % B + 2; x /= B; }
            key = (key << bps) | v;
        }
        h[i] = key;
    }
    uint64_t *dk, *dk2; uint32_t *dv, *dv2;
    hipMalloc(&dk, P * 8); hipMalloc(&dk2, P * 8); hipMalloc(&dv, P * 4); hipMalloc(&dv2, P * 4);
    hipMemcpy(dk, h.data(), P * 8, hipMemcpyHostToDevice);
    std::vector<uint32_t> iv(P); for (size_t i = 0; i < P; i++) iv[i] = i;
    hipMemcpy(dv, iv.data(), P * 4, hipMemcpyHostToDevice);
    const int begin = argc > 4 ? atoi(argv[4]) : bps * (spc - K), end = argc > 5 ? atoi(argv[5]) : bps * spc;
    hipStream_t s; hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    size_t tb = 0; void* tmp = nullptr;
    hipcub::DeviceRadixSort::SortPairs(nullptr, tb, dk, dk2, dv, dv2, (int)P, begin, end, s);
    hipMalloc(&tmp, tb);
    hipcub::DeviceRadixSort::SortPairs(tmp, tb, dk, dk2, dv, dv2, (int)P, begin, end, s);
    hipStreamSynchronize(s);
    std::vector<uint64_t> o(P);
    hipMemcpy(o.data(), dk2, P * 8, hipMemcpyDeviceToHost);
    size_t bad = 0, runs = 1;
    const uint64_t top = ~0ull << (64 - bps);
    for (size_t i = 1; i < P; i++) { bad += o[i] < o[i - 1]; runs += (o[i] & top) != (o[i - 1] & top); }
    printf("B=%d K=%d bps=%d P=%zu bits [%d,%d) temp=%zu: descents %zu, first-symbol runs %zu (want %d)\n", B, K, bps, P, begin, end, tb, bad, runs, B);
    return bad != 0;
}
