// eds-bwt_amd/csrc/format.cpp — host byte work around the search: the multi-threaded CSV
// body formatter for the records of <patterns>output_M_LF.csv ("%u\t%u\t%u\t%u\t%u\n",
// MOVE_EDSBWTSearch.cpp:365), and the 2-bit packer of fixed-length DNA pattern lines that
// shrinks the host pipeline's uploads four-fold (engine.hip search_host_hsa).
#include <immintrin.h>

#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
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

// The same rows written straight to a file descriptor at byte offset `at` (the CLI's
// <patterns>output_M_LF.csv after its header): each thread formats its contiguous range of
// records into a private 8 MB buffer and pwrite()s it at the range's offset (the first pass
// sizes the ranges), so no buffer of the whole CSV is built and the page-cache copies run in
// parallel.  Returns the bytes written, or -1 (errno set) when a write fails.
extern "C" int64_t edsbwt_write_csv(const edsbwt_occ* occ, uint64_t nocc, int fd, uint64_t at, int threads) {
    if (threads < 1) threads = 1;
    const uint64_t T = std::min<uint64_t>((uint64_t)threads, std::max<uint64_t>(1, nocc / 65536));
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
    std::vector<int> err(T, 0);
    std::vector<std::thread> th;
    for (uint64_t t = 0; t < T; t++)
        th.emplace_back([&, t] {
            constexpr size_t kBuf = 8u << 20, kRowMax = 5 * 11;
            std::vector<char> buf(kBuf);
            uint64_t pos = at + sz[t];
            char* p = buf.data();
            auto flush = [&]() -> bool {
                const size_t n = (size_t)(p - buf.data());
                size_t done = 0;
                while (done < n) {
                    const ssize_t w = pwrite(fd, buf.data() + done, n - done, (off_t)(pos + done));
                    if (w < 0) {
                        if (errno == EINTR) continue;
                        err[t] = errno;
                        return false;
                    }
                    done += (size_t)w;
                }
                pos += n;
                p = buf.data();
                return true;
            };
            for (uint64_t i = lo(t); i < lo(t + 1); i++) {
                if ((size_t)(p - buf.data()) + kRowMax > kBuf && !flush()) return;
                const edsbwt_occ& o = occ[i];
                p = put(p, o.pat, ndig(o.pat)); *p++ = '\t';
                p = put(p, o.word, ndig(o.word)); *p++ = '\t';
                p = put(p, o.seg, ndig(o.seg)); *p++ = '\t';
                p = put(p, o.word_in_seg, ndig(o.word_in_seg)); *p++ = '\t';
                p = put(p, o.offset, ndig(o.offset)); *p++ = '\n';
            }
            flush();
        });
    for (auto& x : th) x.join();
    for (uint64_t t = 0; t < T; t++)
        if (err[t]) { errno = err[t]; return -1; }
    return (int64_t)sz[T];
}

// ---- fixed-length line packing.  A chunk of the pattern file (getline lines,
// MOVE_EDSBWTSearch.cpp:111) whose lines all hold exactly L bytes of A/C/G/T (1 <= L <= 32),
// each ended by '\n' (the chunk's last line may lack it), goes over PCIe as 2 bits per base:
// code (byte >> 1) & 3 (A 0, C 1, T 2, G 3), line p at out + p*S with S = ceil(L/4) bytes,
// base j at bits 2*(j%4) of byte j/4.  The device restores the same bytes (kernels.hip
// k_unpack_lines), so the search sees what the unpacked chunk would have given it.

// lines of such a chunk (0: the chunk does not have that form at its first line / its size)
extern "C" uint64_t edsbwt_lines_fixed(const uint8_t* s, uint64_t nb, uint32_t* L_out) {
    if (!nb) return 0;
    const void* nl = std::memchr(s, '\n', std::min<uint64_t>(nb, 33));
    if (!nl) return 0;
    const uint64_t L = (uint64_t)((const uint8_t*)nl - s);
    if (L == 0 || L > 32) return 0;
    uint64_t P = nb / (L + 1);
    const uint64_t r = nb % (L + 1);
    if (r == L) P++;            // a last line without '\n'
    else if (r != 0) return 0;
    *L_out = (uint32_t)L;
    return P;
}

namespace {
__attribute__((target("avx2"))) int pack_avx2(const uint8_t* s, uint64_t nb, uint32_t L, uint64_t p0, uint64_t p1, const uint8_t* end,
                                              uint8_t* out) {
    const __m256i cA = _mm256_set1_epi8('A'), cC = _mm256_set1_epi8('C'), cG = _mm256_set1_epi8('G'), cT = _mm256_set1_epi8('T');
    const __m256i k3 = _mm256_set1_epi8(3), m1 = _mm256_set1_epi16(0x0401), m2 = _mm256_set1_epi32(0x00100001);
    const __m256i shuf = _mm256_setr_epi8(0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,  //
                                          0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1);
    const uint32_t need = L == 32 ? 0xFFFFFFFFu : (1u << L) - 1u;
    const uint64_t cmask = L == 32 ? ~0ull : (1ull << (2 * L)) - 1ull;
    const uint64_t stride = L + 1, S = (L + 3) / 4;
    for (uint64_t p = p0; p < p1; p++) {
        const uint8_t* q = s + p * stride;
        __m256i v;
        if (q + 32 <= end) {
            v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(q));
        } else {  // the caller's buffer ends within 32 bytes
            alignas(32) uint8_t tmp[32] = {0};
            std::memcpy(tmp, q, (size_t)(end - q));
            v = _mm256_load_si256(reinterpret_cast<const __m256i*>(tmp));
        }
        const __m256i acgt = _mm256_or_si256(_mm256_or_si256(_mm256_cmpeq_epi8(v, cA), _mm256_cmpeq_epi8(v, cC)),
                                             _mm256_or_si256(_mm256_cmpeq_epi8(v, cG), _mm256_cmpeq_epi8(v, cT)));
        if (((uint32_t)_mm256_movemask_epi8(acgt) & need) != need) return 0;
        if (p * stride + L < nb ? q[L] != '\n' : p + 1 != p1) return 0;
        const __m256i x = _mm256_and_si256(_mm256_srli_epi16(v, 1), k3);                  // a code per byte
        const __m256i z = _mm256_madd_epi16(_mm256_maddubs_epi16(x, m1), m2);             // 4 codes per u32
        const __m256i w = _mm256_shuffle_epi8(z, shuf);                                   // ... their low bytes
        const uint64_t codes = (((uint64_t)(uint32_t)_mm_cvtsi128_si32(_mm256_extracti128_si256(w, 1)) << 32) |
                                (uint32_t)_mm_cvtsi128_si32(_mm256_castsi256_si128(w))) & cmask;
        // an 8-byte store spills into the following lines' bytes: only while they are still in this
        // range (another thread packs [p1, ...) concurrently), else the line's own S bytes
        if ((p1 - p) * S >= 8) std::memcpy(out + p * S, &codes, 8);
        else std::memcpy(out + p * S, &codes, S);
    }
    return 1;
}

// the bulk of a range for L <= 31, where each line's '\n' falls inside its own 32-byte window: one
// table lookup (pshufb on the low nibble: 'A' 'C' 'G' 'T' '\n' map to themselves, any other byte
// to a value it is not) validates the L bases and the '\n' together, the two code bits come from
// two movemasks spread by pdep, and the verdict is accumulated without a branch per line.  Covers
// the lines [p0, the returned p) whose window lies inside the buffer and whose 8-byte store stays
// inside the range; *bad is nonzero when one of them is not L A/C/G/T bytes then '\n'.
__attribute__((target("avx2,bmi2"))) uint64_t pack_bulk_avx2(const uint8_t* s, uint64_t nb, uint32_t L, uint64_t p0, uint64_t p1,
                                                            const uint8_t* end, uint8_t* out, uint32_t* bad) {
    const char X = (char)0x80;
    const __m256i lut = _mm256_setr_epi8(X, 'A', X, 'C', 'T', X, X, 'G', X, X, '\n', X, X, X, X, X,  //
                                         X, 'A', X, 'C', 'T', X, X, 'G', X, X, '\n', X, X, X, X, X);
    const __m256i nl = _mm256_set1_epi8('\n');
    const uint32_t need = (2u << L) - 1u, nlbit = 1u << L;  // bytes 0..L; L = 31: all 32
    const uint64_t cmask = (1ull << (2 * L)) - 1ull;
    const uint64_t stride = L + 1, S = (L + 3) / 4;
    const uint64_t room = (uint64_t)(end - s);
    uint64_t pe = p1;
    // window inside the buffer, the '\n' inside the chunk, the 8-byte store inside [p0, p1)
    pe = std::min(pe, room >= 32 ? (room - 32) / stride + 1 : 0);
    pe = std::min(pe, nb > L ? (nb - 1 - L) / stride + 1 : 0);
    const uint64_t tail = (8 + S - 1) / S;
    pe = p1 >= tail ? std::min(pe, p1 - tail + 1) : 0;
    if (pe <= p0) return p0;
    uint32_t acc = 0;
    for (uint64_t p = p0; p < pe; p++) {
        const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + p * stride));
        const uint32_t ok = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(_mm256_shuffle_epi8(lut, v), v));
        const uint32_t isnl = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, nl));
        acc |= ((ok & need) ^ need) | ((isnl & need) ^ nlbit);
        const uint64_t lo = (uint32_t)_mm256_movemask_epi8(_mm256_slli_epi16(v, 6));  // byte bit 1: code bit 0
        const uint64_t hi = (uint32_t)_mm256_movemask_epi8(_mm256_slli_epi16(v, 5));  // byte bit 2: code bit 1
        const uint64_t codes = (_pdep_u64(lo, 0x5555555555555555ull) | _pdep_u64(hi, 0xAAAAAAAAAAAAAAAAull)) & cmask;
        std::memcpy(out + p * S, &codes, 8);
    }
    *bad = acc;
    return pe;
}
}  // namespace

// pack lines [p0, p1) of a chunk edsbwt_lines_fixed accepted (L bases each); `end` is the first
// byte of the caller's buffer that may not be read.  Returns 0 when a line is not L A/C/G/T bytes
// then '\n' (or the CPU lacks AVX2): the caller then sends the raw bytes.
extern "C" int edsbwt_pack_lines(const uint8_t* s, uint64_t nb, uint32_t L, uint64_t p0, uint64_t p1, const uint8_t* end, uint8_t* out) {
    if (L == 0 || L > 32 || !__builtin_cpu_supports("avx2")) return 0;
    // the bulk path where pdep is a fast instruction (not on the first two Zen generations)
    // (EDSBWT_PACK_BULK=0: the per-line path only)
    static const bool bulk = __builtin_cpu_supports("bmi2") && !__builtin_cpu_is("znver1") && !__builtin_cpu_is("znver2") &&
                             !(std::getenv("EDSBWT_PACK_BULK") && std::atoi(std::getenv("EDSBWT_PACK_BULK")) == 0);
    if (bulk && L <= 31) {
        uint32_t bad = 0;
        const uint64_t p = pack_bulk_avx2(s, nb, L, p0, p1, end, out, &bad);
        if (bad) return 0;
        p0 = p;
    }
    return pack_avx2(s, nb, L, p0, p1, end, out);
}
