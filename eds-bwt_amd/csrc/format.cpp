// eds-bwt_amd/csrc/format.cpp — multi-threaded CSV body formatter for the records
// of <patterns>output_M_LF.csv ("%u\t%u\t%u\t%u\t%u\n", MOVE_EDSBWTSearch.cpp:365).
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/edsbwt.h"

namespace {
inline int ndig(uint32_t v) {
    int n = 1;
    while (v >= 10) { v /= 10; n++; }
    return n;
}
inline char* put(char* p, uint32_t v, int nd) {
    char* e = p + nd;
    do { *--e = (char)('0' + v % 10); v /= 10; } while (v);
    return p + nd;
}
inline uint64_t row_len(const edsbwt_occ& o) {
    return (uint64_t)ndig(o.pat) + ndig(o.word) + ndig(o.seg) + ndig(o.word_in_seg) + ndig(o.offset) + 5;
}
}  // namespace

extern "C" uint64_t edsbwt_format_csv(const edsbwt_occ* occ, uint64_t nocc, char* buf, uint64_t cap, int threads) {
    if (threads < 1) threads = 1;
    uint64_t T = std::min<uint64_t>((uint64_t)threads, std::max<uint64_t>(1, nocc / 65536));
    std::vector<uint64_t> sz(T + 1, 0);
    auto lo = [&](uint64_t t) { return nocc * t / T; };
    {
        std::vector<std::thread> th;
        for (uint64_t t = 0; t < T; t++)
            th.emplace_back([&, t] {
                uint64_t s = 0;
                for (uint64_t i = lo(t); i < lo(t + 1); i++) s += row_len(occ[i]);
                sz[t + 1] = s;
            });
        for (auto& x : th) x.join();
    }
    for (uint64_t t = 0; t < T; t++) sz[t + 1] += sz[t];
    if (!buf) return sz[T];
    if (cap < sz[T]) return 0;
    std::vector<std::thread> th;
    for (uint64_t t = 0; t < T; t++)
        th.emplace_back([&, t] {
            char* p = buf + sz[t];
            for (uint64_t i = lo(t); i < lo(t + 1); i++) {
                const edsbwt_occ& o = occ[i];
                p = put(p, o.pat, ndig(o.pat)); *p++ = '\t';
                p = put(p, o.word, ndig(o.word)); *p++ = '\t';
                p = put(p, o.seg, ndig(o.seg)); *p++ = '\t';
                p = put(p, o.word_in_seg, ndig(o.word_in_seg)); *p++ = '\t';
                p = put(p, o.offset, ndig(o.offset)); *p++ = '\n';
            }
        });
    for (auto& x : th) x.join();
    return sz[T];
}
