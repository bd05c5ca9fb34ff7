// eds-bwt_amd/csrc/kernels.hip — hand-written gfx950 kernels of the EDS-BWT
// backward search (MOVE_EDSBWTSearch.cpp:228-625 re-designed as a level-synchronous
// walk over a trie of reversed patterns).
//
// Rank/LF layout ("occ block", 128 B = one L2 line, 256 BWT rows):
//   u32 cnt[8]      rank of code c before the block's first row
//   u64 plane[3][4] the 3-bit code of each of the 256 rows, bit-sliced
// rank_c(L, x) = cnt[c] + popcount of rows < x&255 whose 3 bits equal c.
// One 128-B line answers the rank of every symbol at once, so the backward step
// LF_c([b,e]) of MOVE_EDSBWTSearch.cpp:424-510 costs two line reads, and the
// '#'-rank of dollars_in_interval (:607-625) comes out of the same two lines.
#include "kernels.h"

namespace edsbwt {

// ---------------------------------------------------------------- occ blocks
#if EDSBWT_OCC_ROWS == 256
__device__ __forceinline__ void load_block(const OccBlock* __restrict__ occ, uint32_t blk, uint4 (&v)[8]) {
    const uint4* p = reinterpret_cast<const uint4*>(occ + blk);
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = p[i];
}

__device__ __forceinline__ uint64_t u64_of(uint4 v, int hi) {
    return hi ? ((uint64_t)v.w << 32 | v.z) : ((uint64_t)v.y << 32 | v.x);
}

// rank of every code < sigma at row x (rows [0,x) counted)
__device__ __forceinline__ void rank_all(const OccBlock* __restrict__ occ, uint32_t x, uint32_t sigma, uint32_t* out) {
    uint4 v[8];
    load_block(occ, x >> 8, v);
    const uint32_t r = x & 255u;
    const uint32_t wq = r >> 6, bit = r & 63u;
    uint64_t p0[4], p1[4], p2[4], m[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        p0[q] = u64_of(v[2 + (q >> 1)], q & 1);
        p1[q] = u64_of(v[4 + (q >> 1)], q & 1);
        p2[q] = u64_of(v[6 + (q >> 1)], q & 1);
        m[q] = (uint32_t)q < wq ? ~0ull : ((uint32_t)q == wq ? ((1ull << bit) - 1ull) : 0ull);
    }
    const uint32_t cnt[8] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
#pragma unroll
    for (uint32_t c = 0; c < 8; c++) {
        if (c < sigma) {
            uint32_t acc = cnt[c];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                uint64_t e = ((c & 1) ? p0[q] : ~p0[q]) & ((c & 2) ? p1[q] : ~p1[q]) & ((c & 4) ? p2[q] : ~p2[q]);
                acc += (uint32_t)__popcll(e & m[q]);
            }
            out[c] = acc;
        } else {
            out[c] = 0;
        }
    }
}

// symbol code at row x and its rank (one line): LF(x) = C[code] + rank
__device__ __forceinline__ uint32_t sym_rank(const OccBlock* __restrict__ occ, uint32_t x, uint32_t* rank) {
    uint4 v[8];
    load_block(occ, x >> 8, v);
    const uint32_t r = x & 255u;
    const uint32_t wq = r >> 6, bit = r & 63u;
    uint64_t p0[4], p1[4], p2[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        p0[q] = u64_of(v[2 + (q >> 1)], q & 1);
        p1[q] = u64_of(v[4 + (q >> 1)], q & 1);
        p2[q] = u64_of(v[6 + (q >> 1)], q & 1);
    }
    uint64_t w0 = p0[0], w1 = p1[0], w2 = p2[0];
#pragma unroll
    for (int q = 1; q < 4; q++)
        if ((uint32_t)q == wq) { w0 = p0[q]; w1 = p1[q]; w2 = p2[q]; }
    const uint32_t c = (uint32_t)((w0 >> bit) & 1) | (uint32_t)(((w1 >> bit) & 1) << 1) | (uint32_t)(((w2 >> bit) & 1) << 2);
    const uint32_t cnt[8] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t cc = 0; cc < 8; cc++)
        if (cc == c) acc = cnt[cc];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        uint64_t mq = (uint32_t)q < wq ? ~0ull : ((uint32_t)q == wq ? ((1ull << bit) - 1ull) : 0ull);
        uint64_t e = ((c & 1) ? p0[q] : ~p0[q]) & ((c & 2) ? p1[q] : ~p1[q]) & ((c & 4) ? p2[q] : ~p2[q]);
        acc += (uint32_t)__popcll(e & mq);
    }
    *rank = acc;
    return c;
}

// rank of '#' (code 0) and of code c at row x from one occ-block line
__device__ __forceinline__ void rank2(const OccBlock* __restrict__ occ, uint32_t x, uint32_t c, uint32_t& r0, uint32_t& rc) {
    uint4 v[8];
    load_block(occ, x >> 8, v);
    const uint32_t r = x & 255u;
    const uint32_t wq = r >> 6, bit = r & 63u;
    const uint32_t cnt[8] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
    uint32_t a0 = cnt[0], ac = 0;
#pragma unroll
    for (uint32_t cc = 1; cc < 8; cc++)
        if (cc == c) ac = cnt[cc];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint64_t p0 = u64_of(v[2 + (q >> 1)], q & 1);
        const uint64_t p1 = u64_of(v[4 + (q >> 1)], q & 1);
        const uint64_t p2 = u64_of(v[6 + (q >> 1)], q & 1);
        const uint64_t mq = (uint32_t)q < wq ? ~0ull : ((uint32_t)q == wq ? ((1ull << bit) - 1ull) : 0ull);
        a0 += (uint32_t)__popcll(~p0 & ~p1 & ~p2 & mq);
        const uint64_t e = ((c & 1) ? p0 : ~p0) & ((c & 2) ? p1 : ~p1) & ((c & 4) ? p2 : ~p2);
        ac += (uint32_t)__popcll(e & mq);
    }
    r0 = a0;
    rc = (c == 0) ? a0 : ac;
}

__device__ __forceinline__ uint32_t rank_all_pair(const OccBlock* __restrict__ occ, uint32_t x0, uint32_t x1, uint32_t sigma, uint32_t* o0,
                                                  uint32_t* o1) {
    rank_all(occ, x0, sigma, o0);
    rank_all(occ, x1, sigma, o1);
    return 0;  // two block reads
}

__device__ __forceinline__ uint32_t rank2_pair(const OccBlock* __restrict__ occ, uint32_t x0, uint32_t x1, uint32_t c, uint32_t& h0, uint32_t& r0,
                                               uint32_t& h1, uint32_t& r1) {
    rank2(occ, x0, c, h0, r0);
    rank2(occ, x1, c, h1, r1);
    return 0;  // two block reads
}
#else  // 64 rows per 64-B block
struct OccV {
    uint32_t cnt[8];
    uint64_t p0, p1, p2, samp;
};
__device__ __forceinline__ OccV load_block(const OccBlock* __restrict__ occ, uint32_t blk) {
    const uint4* p = reinterpret_cast<const uint4*>(occ + blk);
    const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
    OccV o;
    o.cnt[0] = a.x; o.cnt[1] = a.y; o.cnt[2] = a.z; o.cnt[3] = a.w;
    o.cnt[4] = b.x; o.cnt[5] = b.y; o.cnt[6] = b.z; o.cnt[7] = b.w;
    o.p0 = (uint64_t)c.y << 32 | c.x;
    o.p1 = (uint64_t)c.w << 32 | c.z;
    o.p2 = (uint64_t)d.y << 32 | d.x;
    o.samp = (uint64_t)d.w << 32 | d.z;
    return o;
}

__device__ __forceinline__ void rank_all_v(const OccV& v, uint32_t x, uint32_t sigma, uint32_t* out) {
    const uint64_t m = (1ull << (x & 63u)) - 1ull;
#pragma unroll
    for (uint32_t c = 0; c < 8; c++) {
        const uint64_t e = ((c & 1) ? v.p0 : ~v.p0) & ((c & 2) ? v.p1 : ~v.p1) & ((c & 4) ? v.p2 : ~v.p2);
        out[c] = c < sigma ? v.cnt[c] + (uint32_t)__popcll(e & m) : 0u;
    }
}

__device__ __forceinline__ void rank_all(const OccBlock* __restrict__ occ, uint32_t x, uint32_t sigma, uint32_t* out) {
    rank_all_v(load_block(occ, x >> 6), x, sigma, out);
}

// ranks at x0 <= x1 (an interval's b and e+1): narrow intervals share one block, so
// the second block is read only by lanes whose ends fall in different blocks.
// Returns 1 when one block served both.
__device__ __forceinline__ uint32_t rank_all_pair(const OccBlock* __restrict__ occ, uint32_t x0, uint32_t x1, uint32_t sigma, uint32_t* o0,
                                                  uint32_t* o1) {
    // only lanes whose ends lie in different blocks read a second line (measured: issuing
    // both reads unconditionally costs the level step more than the serialisation saves)
    const bool same = (x1 >> 6) == (x0 >> 6);
    OccV v = load_block(occ, x0 >> 6);
    rank_all_v(v, x0, sigma, o0);
    if (!same) v = load_block(occ, x1 >> 6);
    rank_all_v(v, x1, sigma, o1);
    return same;
}

__device__ __forceinline__ uint32_t sym_rank(const OccBlock* __restrict__ occ, uint32_t x, uint32_t* rank) {
    const OccV v = load_block(occ, x >> 6);
    const uint32_t bit = x & 63u;
    const uint64_t m = (1ull << bit) - 1ull;
    const uint32_t c = (uint32_t)((v.p0 >> bit) & 1) | (uint32_t)(((v.p1 >> bit) & 1) << 1) | (uint32_t)(((v.p2 >> bit) & 1) << 2);
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t cc = 0; cc < 8; cc++)
        if (cc == c) acc = v.cnt[cc];
    const uint64_t e = ((c & 1) ? v.p0 : ~v.p0) & ((c & 2) ? v.p1 : ~v.p1) & ((c & 4) ? v.p2 : ~v.p2);
    *rank = acc + (uint32_t)__popcll(e & m);
    return c;
}

__device__ __forceinline__ void rank2_v(const OccV& v, uint32_t x, uint32_t c, uint32_t& r0, uint32_t& rc) {
    const uint64_t m = (1ull << (x & 63u)) - 1ull;
    uint32_t ac = 0;
#pragma unroll
    for (uint32_t cc = 1; cc < 8; cc++)
        if (cc == c) ac = v.cnt[cc];
    r0 = v.cnt[0] + (uint32_t)__popcll(~v.p0 & ~v.p1 & ~v.p2 & m);
    const uint64_t e = ((c & 1) ? v.p0 : ~v.p0) & ((c & 2) ? v.p1 : ~v.p1) & ((c & 4) ? v.p2 : ~v.p2);
    rc = (c == 0) ? r0 : ac + (uint32_t)__popcll(e & m);
}

__device__ __forceinline__ void rank2(const OccBlock* __restrict__ occ, uint32_t x, uint32_t c, uint32_t& r0, uint32_t& rc) {
    rank2_v(load_block(occ, x >> 6), x, c, r0, rc);
}

__device__ __forceinline__ uint32_t rank2_pair(const OccBlock* __restrict__ occ, uint32_t x0, uint32_t x1, uint32_t c, uint32_t& h0, uint32_t& r0,
                                               uint32_t& h1, uint32_t& r1) {
    // both reads back to back, no branch between them (k_deep's intervals are narrow: the
    // second read is nearly always the same line and k_deep is latency-bound)
    const bool same = (x1 >> 6) == (x0 >> 6);
    const OccV v0 = load_block(occ, x0 >> 6);
    const OccV v1 = load_block(occ, x1 >> 6);
    rank2_v(v0, x0, c, h0, r0);
    rank2_v(v1, x1, c, h1, r1);
    return same;
}
#endif

// every symbol's rank at x from the all-symbol rank entries (kernels.h rk16; sigma <= 5)
__device__ __forceinline__ void rk16_rank_v(uint4 v, uint4 s, uint32_t x, uint32_t* out) {
    const uint32_t m = (1u << (x & 15u)) - 1u;
    const uint32_t p0 = v.z & 0xFFFFu, p1 = v.z >> 16, p2 = v.w & 0xFFFFu;
    const uint32_t r1 = s.x + (v.x & 0xFFFFu) + (uint32_t)__popc(p0 & ~p1 & ~p2 & m);
    const uint32_t r2 = s.y + (v.x >> 16) + (uint32_t)__popc(~p0 & p1 & ~p2 & m);
    const uint32_t r3 = s.z + (v.y & 0xFFFFu) + (uint32_t)__popc(p0 & p1 & ~p2 & m);
    const uint32_t r4 = s.w + (v.y >> 16) + (uint32_t)__popc(~p0 & ~p1 & p2 & m);
    out[0] = x - (r1 + r2 + r3 + r4);
    out[1] = r1; out[2] = r2; out[3] = r3; out[4] = r4;
    out[5] = out[6] = out[7] = 0u;
}
// ranks of every symbol at both interval ends x0 <= x1: one 16-B entry per end (one when both
// fall in the same 16 rows), else the 64-B occ blocks.  Returns 1 when one load served both.
__device__ __forceinline__ uint32_t rank_all_pair_any(const KIdx& X, uint32_t x0, uint32_t x1, uint32_t* o0, uint32_t* o1) {
    if (X.rk16) {
        const bool same = (x0 >> 4) == (x1 >> 4);
        const uint4 v0 = X.rk16[x0 >> 4], s0 = X.rk16sup[x0 >> 16];
        rk16_rank_v(v0, s0, x0, o0);
        if (same) {
            rk16_rank_v(v0, s0, x1, o1);
        } else {
            rk16_rank_v(X.rk16[x1 >> 4], X.rk16sup[x1 >> 16], x1, o1);
        }
        return same;
    }
    return rank_all_pair(X.occ, x0, x1, X.sigma, o0, o1);
}

// one 16-B rank entry (kernels.h): rank of its code and of its '#' (or '#'-or-(c1,'#')) rows at x
__device__ __forceinline__ void rent_rank(uint4 v, uint32_t x, uint32_t& r, uint32_t& h) {
    const uint32_t m = (1u << (x & 31u)) - 1u;
    r = v.x + (uint32_t)__popc(v.y & m);
    h = v.z + (uint32_t)__popc(v.w & m);
}
// '#'-rank and c-rank at both interval ends (x0 = b, x1 = e + 1): one 16-B rank entry per
// end when built, else the occ blocks.  Returns 1 when one block served both ends.
__device__ __forceinline__ uint32_t rank2_any(const KIdx& X, uint32_t x0, uint32_t x1, uint32_t c, uint32_t& h0, uint32_t& r0, uint32_t& h1,
                                              uint32_t& r1) {
    if (X.rent1) {
        const uint4 v0 = X.rent1[(size_t)(x0 >> 5) * X.sigma + c];
        const uint4 v1 = X.rent1[(size_t)(x1 >> 5) * X.sigma + c];
        rent_rank(v0, x0, r0, h0);
        rent_rank(v1, x1, r1, h1);
        return (x0 >> 5) == (x1 >> 5);
    }
    return rank2_pair(X.occ, x0, x1, c, h0, r0, h1, r1);
}

// cnt | kResRow: the pattern's one interval is [off, off + occ) itself, not in the archive
// (the deep kernels' single-interval results: no archive write, no archive read in k_tasks)
constexpr uint32_t kResRow = 0x80000000u;
// cnt | kResRow | kResPos: the pattern's one occurrence is the text position itself (single-row
// text compare, k_deep_fast): off = offset << 32 | word, occ = 1 — no row, no archive
constexpr uint32_t kResPos = 0x40000000u;
constexpr uint32_t kResCnt = 0x3FFFFFFFu;  // the interval count in cnt
// k_deep queue entries (i, d, z, w): z = b, w = e — the pattern goes on from depth d with the one
// interval [b, e] (rows < 2^32 - 16, engine.hip); z = kQNode — from its node's items at the cutover
// depth (nid / ioff / iend); z = kQWide, w = the D-mer id — on the direct start with the wide k-mer
// table, from the D-mer's list read from its wide entry, where lists of up to kWideInline
// intervals are held inline.  The producer names the kind (k_deep does not infer it)
constexpr uint32_t kQNode = 0xFFFFFFFFu, kQWide = 0xFFFFFFFEu;
constexpr int kWideInline = 3;
// a kResPos result carries the whole record: cnt = kResRow | kResPos | word-in-segment (< 2^30),
// occ = segment; its occurrence count is 1
__device__ __forceinline__ uint32_t res_occ(const Res& r) { return (r.cnt & kResPos) ? 1u : r.occ; }
__device__ __forceinline__ uint32_t res_cnt(const Res& r) { return (r.cnt & kResPos) ? 1u : (r.cnt & kResCnt); }

// 32 characters of the reversed text from reversed index r (bits 2j = character r + j)
__device__ __forceinline__ uint64_t rtext_window(const uint64_t* __restrict__ rt, uint64_t r) {
    const uint64_t q = r >> 5;
    const uint32_t sh = (uint32_t)(r & 31u) * 2u;
    const uint64_t a = rt[q];
    if (!sh) return a;
    return (a >> sh) | (rt[q + 1] << (64u - sh));
}
// the packed start's remaining symbols (2 bits each, closed by a 1 bit): symbols past the 32nd
// (a pattern too long for the packed start, which the deferred checks send to the redo) are
// dropped rather than shifted out of range; and its length back from the closing bit
__device__ __forceinline__ uint64_t pk_digit(uint64_t v, uint32_t n) { return n < 32 ? v << (2 * n) : 0ull; }
__device__ __forceinline__ uint32_t pk_len(uint32_t D0, uint64_t rem) { return rem ? D0 + (uint32_t)(63 - __builtin_clzll(rem)) / 2 : D0; }
// rare per-pattern events (deep-kernel overflows): lst[0] counts, the pattern ids follow
__device__ __forceinline__ void flag_push(uint32_t* __restrict__ lst, uint32_t i) { lst[1 + atomicAdd(lst, 1u)] = i; }
__device__ __forceinline__ void put_res(Res* __restrict__ r, size_t o, uint64_t off, uint32_t cnt, uint32_t occ) {
    reinterpret_cast<uint4*>(r)[o] = make_uint4((uint32_t)off, (uint32_t)(off >> 32), cnt, occ);
}

#define GRID_STRIDE(i, n) for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < (size_t)(n); i += (size_t)gridDim.x * blockDim.x)

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// block-wide sum (256 threads), result valid in thread 0
__device__ __forceinline__ unsigned long long block_sum(unsigned long long x, unsigned long long* sh) {
    x = wave_sum(x);
    __syncthreads();  // sh may still be read by a previous block_sum
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = x;
    __syncthreads();
    unsigned long long t = 0;
    if (threadIdx.x == 0)
        for (uint32_t w = 0; w < blockDim.x / 64; w++) t += sh[w];
    return t;
}

// exclusive prefix sum of x over the 64 lanes of the wave
__device__ __forceinline__ unsigned long long wave_excl_scan(unsigned long long x) {
    const uint32_t lane = threadIdx.x & 63;
    unsigned long long inc = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long y = __shfl_up(inc, (unsigned)o, 64);
        if (lane >= (uint32_t)o) inc += y;
    }
    return inc - x;
}



// statistics counters: block-reduced, then one atomic per block into one of kStatShards
// 128-B lines (the host folds the shards), so no address takes every block's add.
// Every thread of the block must call it.
constexpr uint32_t kStatShards = 32, kStatStride = 32, kStatSlots = kStatShards * kStatStride;
// statistic slots (zeroed once per search, folded at its end)
enum : uint32_t { ST_DEEP_STEPS = 0, ST_DEEP_HASH = 1, ST_LOC_STEPS = 2, ST_STEP_BLOCKS = 3, ST_DEEP_BLOCKS = 4, ST_LOC_OFFSETS = 5,
                  ST_CLK_RANK = 6, ST_CLK_RUNS = 7, ST_CLK_REST = 8, ST_CLK_STEPS = 9, ST_CLK_HASH_STEPS = 10,
                  ST_DEEP_PAIR_LINES = 11,  // of ST_DEEP_BLOCKS, the rank-entry lines
                  ST_TEXT_CHARS = 12, ST_TEXT_ROWS = 13,  // characters decided / single rows met by the text compare
                  ST_DEEPQ_STEPS = 14, ST_DEEPQ_BLOCKS = 15,  // k_deep's own (ST_DEEP_*: k_deep_fast's)
                  ST_LVL_SINGLE = 16,  // k_lvl_items input items of one row (b == e)
                  ST_DF_LANE_ROUNDS = 17, ST_DF_WAVE_ROUNDS = 18,  // k_deep_fast: dependent load rounds of the
                  // lanes' patterns, and 64 x the slowest lane's per pattern slot (lane utilisation)
                  ST_DW_BLOCKS = 19, ST_DW_STEPS = 20,  // k_deep_wave's lines and interval steps
                  ST_DEEPQ_PATS = 21,  // queue entries k_deep read
                  // fused counts (deferred direct start): the deep kernels write each final count and add
                  // found / occurrences / intervals here; k_gather_checks folds them (no k_count_found pass)
                  ST_FC_FOUND = 22, ST_FC_OCC = 23,
                  // debug build (-DEDSBWT_DEBUG_CHECKS, libedsbwt_dbg.so): failed invariant checks per kind;
                  // search() throws when any is non-zero (engine.hip check_debug)
                  ST_DBG_QUEUE = 24, ST_DBG_PACKED = 25, ST_DBG_WIDE = 26, ST_DBG_LIST = 27,
                  // profiling build (-DEDSBWT_DEEP_CLOCKS): k_deep_direct's loads by kind — per-row text
                  // entries, segment-table rows, whole-word rows, and D-mer entries of one row
                  ST_CLK_DD_SROW = 28, ST_CLK_DD_SEG = 29, ST_CLK_DD_WROW = 30, ST_CLK_DD_ONE = 31 };
#ifdef EDSBWT_DEBUG_CHECKS
#define DBG_CHECK(cond, var) \
    do {                     \
        if (!(cond)) (var)++; \
    } while (0)
#else
#define DBG_CHECK(cond, var) \
    do {                     \
    } while (0)
#endif
// k_deep phase clocks (profiling build, -DEDSBWT_DEEP_CLOCKS): shader cycles summed over lanes
#ifdef EDSBWT_DEEP_CLOCKS
#define DEEP_CLK(v) const uint64_t v = __builtin_readcyclecounter()
#define DEEP_CLK_ADD(acc, x) acc += (x)
#define DD_CNT(v) (v)++
#else
#define DEEP_CLK(v)
#define DEEP_CLK_ADD(acc, x)
#define DD_CNT(v)
#endif
__device__ __forceinline__ void stat_add(unsigned long long* __restrict__ stats, uint32_t k, unsigned long long v, unsigned long long* sh) {
    v = block_sum(v, sh);
    if (threadIdx.x == 0 && v) atomicAdd(stats + (blockIdx.x % kStatShards) * kStatStride + k, v);
}

// a final result's count into counts[o] (fused counts), and the lane's found / occurrence sums in
// two u32 registers: the occurrence sum saturates at 2^32 - 1, which fails the deferred checks'
// record-capacity test (a batch with that many records is searched again on the checked path).
// The interval total is not kept: the deferred path that fuses counts (count-only) never builds
// the task list it bounds.  (Round 5 also summed the per-pattern locate's 64-pattern record tiles
// here — a register and an atomic per put in every deep kernel — and measured it slower than
// k_count_tiles' pass: removed)
struct CountSums {
    uint32_t f = 0, occ = 0;
    __device__ __forceinline__ void put(uint32_t* __restrict__ counts, size_t o, uint32_t occ_) {
        if (!counts) return;
        counts[o] = occ_;
        f += occ_ > 0;
        occ = occ + occ_ < occ ? 0xFFFFFFFFu : occ + occ_;
    }
    // every thread of the block
    __device__ __forceinline__ void flush(const uint32_t* counts, unsigned long long* __restrict__ ctr, unsigned long long* sh) {
        if (!counts) return;
        stat_add(ctr, ST_FC_FOUND, f, sh);
        stat_add(ctr, ST_FC_OCC, occ, sh);
    }
};

// ------------------------------------------------------ sharded appends
// Appends are wave-aggregated: one atomic per wave per buffer.  Call with every
// lane of the wave active.
__device__ __forceinline__ uint32_t wave_append(uint32_t* __restrict__ counter, uint32_t n) {
    const int lane = threadIdx.x & 63;
    uint32_t x = n;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    const uint32_t total = __shfl(x, 63, 64);
    uint32_t base = 0;
    if (lane == 63 && total) base = atomicAdd(counter, total);
    base = __shfl(base, 63, 64);
    return base + x - n;
}

// three appends (counters cnt[0..2] of one shard line) with one atomic round trip
__device__ __forceinline__ void wave_append3(uint32_t* __restrict__ cnt, uint32_t n0, uint32_t n1, uint32_t n2, uint32_t& a0, uint32_t& a1,
                                             uint32_t& a2) {
    const int lane = threadIdx.x & 63;
    uint32_t x = n0, y = n1, z = n2;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t px = __shfl_up(x, o, 64), py = __shfl_up(y, o, 64), pz = __shfl_up(z, o, 64);
        if (lane >= o) { x += px; y += py; z += pz; }
    }
    uint32_t b0 = 0, b1 = 0, b2 = 0;
    if (lane == 63) {
        if (x) b0 = atomicAdd(cnt + 0, x);
        if (y) b1 = atomicAdd(cnt + 1, y);
        if (z) b2 = atomicAdd(cnt + 2, z);
    }
    a0 = __shfl(b0, 63, 64) + x - n0;
    a1 = __shfl(b1, 63, 64) + y - n1;
    a2 = __shfl(b2, 63, 64) + z - n2;
}

// Appends go to NSHARD independent regions (counter k of shard s at cnt[s*32+k],
// one 128-B line per shard) so that no single address takes every wave's atomic;
// k_unshard packs the regions afterwards.
#ifndef EDSBWT_NSHARD
#define EDSBWT_NSHARD 64
#endif
constexpr uint32_t NSHARD = EDSBWT_NSHARD;

// grid-stride loop whose trip count is uniform across each block (so wave-wide
// shuffles inside it see every lane); `valid` marks the lanes past the end
#define UNIFORM_STRIDE(i, valid, n)                                                                                     \
    for (size_t i##_b = (size_t)blockIdx.x * blockDim.x; i##_b < (size_t)(n); i##_b += (size_t)gridDim.x * blockDim.x) \
        if (const size_t i = i##_b + threadIdx.x; true)                                                                  \
            if (const bool valid = i < (size_t)(n); true)

template <typename T>
__device__ __forceinline__ size_t upper_bound_dev(const T* __restrict__ a, size_t n, T key) {
    size_t lo = 0, hi = n;
    while (lo < hi) {
        size_t mid = (lo + hi) >> 1;
        if (a[mid] <= key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// ------------------------------------------------------------ pattern trie
__global__ void k_lens(const uint64_t* __restrict__ off, uint64_t P, uint32_t* __restrict__ len) {
    GRID_STRIDE(i, P) len[i] = (uint32_t)(off[i + 1] - off[i]);
}

// Sort codes of the reversed pattern, BPS bits each (3 when sigma+2 <= 8, else 4),
// SPC = 64/BPS per u64 chunk, most significant first: 0 = end of pattern, 1+code
// for alphabet symbols, sigma+1 for bytes outside it.  Chunk c of pattern i at
// keys[c*P + i].  A block's patterns are contiguous in `bytes`, so the block stages
// their bytes in LDS with coalesced 4-B loads (spans over kKeySpan bytes read global
// memory directly).  Also writes len[] and counts patterns holding the end-marker '#'.
constexpr uint32_t kKeySpan = 12288;  // bytes of one block-round's patterns staged in LDS (12 KB: 13 blocks per CU overlap their loads)
template <int BPS>
__global__ void __launch_bounds__(256) k_keys(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, uint64_t P,
                                              const uint8_t* __restrict__ code_of, uint32_t sigma, uint32_t nch, uint64_t* __restrict__ keys,
                                              uint32_t* __restrict__ len, unsigned long long* __restrict__ n_term,
                                              uint32_t D, uint32_t E, uint32_t* __restrict__ kid, uint64_t* __restrict__ pv,
                                              uint32_t* __restrict__ hist, uint32_t hshift) {
    // kid / pv (direct start), from the chunks still in registers: kid = the D-mer id of the
    // pattern's last D symbols (last character least significant digit, as k_ktab_count reads
    // a node's); a D-mer holding '#' or a byte outside the alphabet has no list: kid = E
    // (= B^D), whose list is empty.  pv = the packed start (B <= 4, at most 16 symbols after
    // depth D): input index in bits [0, 31), the remaining symbols' 2-bit digits from bit 31
    // up, closed by a 1 bit; a symbol outside the alphabet there also gives kid = E.
    constexpr uint32_t SPC = 64 / BPS;
    __shared__ uint32_t sbuf[kKeySpan / 4 + 2];
    __shared__ uint8_t scode[256];
    __shared__ unsigned long long sh[4];
    for (uint32_t t = threadIdx.x; t < 256; t += blockDim.x) {
        const uint32_t c = code_of[t];
        scode[t] = (uint8_t)(c < sigma ? c + 1 : sigma + 1);
    }
    unsigned long long nt = 0;
    for (size_t base = (size_t)blockIdx.x * blockDim.x; base < P; base += (size_t)gridDim.x * blockDim.x) {
        const size_t nb = min((size_t)blockDim.x, (size_t)P - base);
        const uint64_t s0 = off[base], s1 = off[base + nb];
        const uint64_t w0 = s0 & ~3ull;
        const bool staged = s1 - w0 <= kKeySpan && ((uintptr_t)bytes & 3) == 0;
        __syncthreads();  // previous round's readers are done with sbuf (and scode is ready)
        if (staged) {
            const uint32_t nw = (uint32_t)((s1 - w0 + 3) / 4);
            const uint32_t* src = reinterpret_cast<const uint32_t*>(bytes + w0);
            for (uint32_t t = threadIdx.x; t < nw; t += blockDim.x) sbuf[t] = src[t];
        }
        __syncthreads();
        const size_t i = base + threadIdx.x;
        if (i < P) {
            const uint64_t a = off[i];
            const uint32_t L = (uint32_t)(off[i + 1] - a);
            len[i] = L;
            const uint8_t* sg = bytes + a;
            const uint32_t so = (uint32_t)(a - w0);
            uint32_t term = 0;
            uint64_t kc0 = 0, kc1 = 0;
            for (uint32_t c = 0; c < nch; c++) {
                uint64_t key = 0;
                for (uint32_t t = 0; t < SPC; t++) {
                    const uint32_t pos = c * SPC + t;
                    uint64_t v = 0;
                    if (pos < L) {
                        // the staged bytes straight from LDS (a block-uniform branch: no flat
                        // loads through a pointer that may be LDS or global)
                        uint32_t ch;
                        if (staged) {
                            const uint32_t k = so + L - 1 - pos;
                            ch = (sbuf[k >> 2] >> (8 * (k & 3))) & 0xffu;
                        } else {
                            ch = sg[L - 1 - pos];
                        }
                        v = scode[ch];
                        term |= ch == '#';
                    }
                    key = (key << BPS) | v;
                }
                if (!pv) keys[(size_t)c * P + i] = key;  // the packed start needs no key chunks
                if (c == 0) kc0 = key;
                if (c == 1) kc1 = key;
            }
            nt += term;
            if (kid) {
                const uint32_t B = sigma - 1;
                uint32_t x = 0, mul = 1;
                bool ok = true;
                for (uint32_t t = 0; t < D; t++) {
                    const uint32_t v = (uint32_t)(kc0 >> (BPS * (SPC - 1 - t))) & ((1u << BPS) - 1u);
                    ok &= v >= 2 && v <= B + 1;
                    x += (v - 2) * mul;
                    mul *= B;
                }
                if (pv) {  // L <= D + 16 <= 2 * SPC: the remaining symbols lie in chunks 0 and 1
                    uint64_t rem = 0;
                    uint32_t n = 0;
                    for (uint32_t t = D; t < L; t++) {
                        const uint64_t k = t < SPC ? kc0 : kc1;
                        const uint32_t v = (uint32_t)(k >> (BPS * (SPC - 1 - (t < SPC ? t : t - SPC)))) & ((1u << BPS) - 1u);
                        ok &= v >= 2 && v <= B + 1;
                        rem |= pk_digit((v - 2) & 3u, n);
                        n++;
                    }
                    rem |= pk_digit(1, n);
                    pv[i] = rem << 31 | (uint64_t)i;
                }
                kid[i] = ok ? x : E;
                if (hist) atomicAdd(&hist[(ok ? x : E) >> hshift], 1u);  // bucket sizes for k_bucket_scatter
            }
        }
    }
    nt = block_sum(nt, sh);
    if (threadIdx.x == 0 && nt) atomicAdd(n_term, nt);
}

__global__ void k_iota(uint32_t* __restrict__ a, uint64_t n) { GRID_STRIDE(i, n) a[i] = (uint32_t)i; }

// The packed direct start's keys straight from the bytes (k_keys builds the 3-bit sort chunks
// first and reads kid / pv back out of them): per pattern, reading its characters from the end,
// the D-mer id of the last D symbols (last character least significant digit), the packed
// start (input index, then the remaining <= 16 symbols as 2-bit digits closed by a 1 bit), the
// length, and whether it holds '#'.  A symbol outside the B <= 4 non-'#' symbols gives kid = E.
__global__ void __launch_bounds__(256) k_keys_packed(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, uint64_t P,
                                                     const uint8_t* __restrict__ code_of, uint32_t sigma, uint32_t* __restrict__ len,
                                                     unsigned long long* __restrict__ n_term, uint32_t D, uint32_t E,
                                                     uint32_t* __restrict__ kid, uint64_t* __restrict__ pv) {
    __shared__ uint32_t sbuf[kKeySpan / 4 + 2];
    __shared__ uint8_t scode[256];
    __shared__ unsigned long long sh[4];
    const uint32_t B = sigma - 1;
    for (uint32_t t = threadIdx.x; t < 256; t += blockDim.x) {
        const uint32_t c = code_of[t];
        // digit + 1 for the B non-'#' symbols, 0 for '#' and bytes outside the alphabet
        scode[t] = (uint8_t)(c >= 1 && c < sigma ? c : 0);
    }
    unsigned long long nt = 0;
    for (size_t base = (size_t)blockIdx.x * blockDim.x; base < P; base += (size_t)gridDim.x * blockDim.x) {
        const size_t nb = min((size_t)blockDim.x, (size_t)P - base);
        const uint64_t s0 = off[base], s1 = off[base + nb];
        const uint64_t w0 = s0 & ~3ull;
        const bool staged = s1 - w0 <= kKeySpan && ((uintptr_t)bytes & 3) == 0;
        __syncthreads();
        if (staged) {
            const uint32_t nw = (uint32_t)((s1 - w0 + 3) / 4);
            const uint32_t* src = reinterpret_cast<const uint32_t*>(bytes + w0);
            for (uint32_t t = threadIdx.x; t < nw; t += blockDim.x) sbuf[t] = src[t];
        }
        __syncthreads();
        const size_t i = base + threadIdx.x;
        if (i < P) {
            const uint64_t a = off[i];
            const uint32_t L = (uint32_t)(off[i + 1] - a);
            len[i] = L;
            const uint32_t so = (uint32_t)(a - w0);
            uint32_t x = 0, mul = 1, n = 0;
            uint64_t rem = 0;
            bool ok = true, term = false;
            for (uint32_t t = 0; t < L; t++) {
                const uint32_t k = L - 1 - t;
                const uint32_t ch = staged ? (sbuf[(so + k) >> 2] >> (8 * ((so + k) & 3))) & 0xffu : bytes[a + k];
                const uint32_t v = scode[ch];
                term |= ch == '#';
                ok &= v != 0;
                if (t < D) {
                    x += (v - 1) * mul;
                    mul *= B;
                } else {
                    rem |= pk_digit((v - 1) & 3u, n);
                    n++;
                }
            }
            nt += term;
            rem |= pk_digit(1, n);
            pv[i] = rem << 31 | (uint64_t)i;
            kid[i] = ok ? x : E;
        }
    }
    nt = block_sum(nt, sh);
    if (threadIdx.x == 0 && nt) atomicAdd(n_term, nt);
}

// per byte of x: 0x80 where the byte is zero, else 0 (exact, no borrow between bytes)
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) { return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u; }
// k_keys_packed for the alphabet {#, A, C, G, T} (codes 0..4: DNA, C3's): four characters per
// LDS word, their digits by byte compares (SWAR) instead of one table lookup and one
// multiply-add per character.  The pattern's digits form V (its last character least
// significant): kid = the low 2D bits, the packed start = the rest, closed by a 1 bit — the same
// values k_keys_packed writes (its per-character loop is kept for patterns over 32 characters).
// One pattern's D-mer id and packed start over {#, A, C, G, T} (k_keys_acgt, and the fused
// direct start k_deep_direct<MINW, true>): its bytes from the block's LDS stage (sbuf, so = its
// offset there) when staged, else from global memory.  x = the D-mer id (E when a byte is outside
// the alphabet), rem = the remaining symbols closed by a 1 bit, term = '#' in the pattern or
// (lmax != 0) a length outside [lmin, lmax].
__device__ __forceinline__ void acgt_key(const uint8_t* __restrict__ bytes, uint64_t a, uint32_t L, bool staged, const uint32_t* sbuf,
                                         uint32_t so, uint32_t D, uint32_t E, uint32_t lmin, uint32_t lmax, uint32_t& x_out,
                                         uint64_t& rem_out, bool& term_out) {
    uint64_t V = 0;
    bool ok = true, term = lmax != 0 && (L < lmin || L > lmax);
    if (L <= 32) {
        for (uint32_t j = 0; j < L; j += 4) {
            const uint32_t n = min(4u, L - j);
            uint32_t w;
            if (staged) {
                const uint32_t o = so + j;
                w = __builtin_amdgcn_alignbyte(sbuf[(o >> 2) + 1], sbuf[o >> 2], o & 3u);
            } else {
                w = 0;
                for (uint32_t t = 0; t < n; t++) w |= (uint32_t)bytes[a + j + t] << (8 * t);
            }
            const uint32_t live = n == 4 ? 0x80808080u : (0x80808080u >> (8 * (4 - n)));  // the n bytes in the pattern
            const uint32_t mC = zero_bytes(w ^ 0x43434343u), mG = zero_bytes(w ^ 0x47474747u), mT = zero_bytes(w ^ 0x54545454u);
            const uint32_t hit = zero_bytes(w ^ 0x41414141u) | mC | mG | mT;
            ok &= (hit & live) == live;
            term |= (zero_bytes(w ^ 0x23232323u) & live) != 0;
            const uint32_t bad = ~hit & 0x80808080u;  // '#' or outside the alphabet: digit 3, as (0 - 1) & 3
            const uint32_t q = ((mC | mT | bad) >> 7) | ((mG | mT | bad) >> 6);  // digit (A 0, C 1, G 2, T 3) per byte
            const uint32_t pk = ((q & 3u) << 6) | (((q >> 8) & 3u) << 4) | (((q >> 16) & 3u) << 2) | ((q >> 24) & 3u);
            V = (V << (2 * n)) | (pk >> (8 - 2 * n));
        }
        if (L <= D) {
            x_out = ok ? (uint32_t)V : E;
            rem_out = 1ull;
        } else {
            x_out = ok ? (uint32_t)(V & ((1ull << (2 * D)) - 1ull)) : E;
            rem_out = (V >> (2 * D)) | pk_digit(1, L - D);
        }
    } else {  // rare: longer patterns keep k_keys_packed's per-character order
        uint32_t x = 0, mul = 1, nn = 0;
        uint64_t rem = 0;
        for (uint32_t t = 0; t < L; t++) {
            const uint32_t ch = bytes[a + L - 1 - t];
            const uint32_t v = ch == 'A' ? 1u : ch == 'C' ? 2u : ch == 'G' ? 3u : ch == 'T' ? 4u : 0u;
            term |= ch == '#';
            ok &= v != 0;
            if (t < D) { x += (v - 1) * mul; mul *= 4u; }
            else { rem |= pk_digit((v - 1) & 3u, nn); nn++; }
        }
        rem |= pk_digit(1, nn);
        x_out = ok ? x : E;
        rem_out = rem;
    }
    term_out = term;
}

// acgt_key for a pattern of L <= 32 bytes held in registers: W[k] = its bytes 4k .. 4k + 3 (fully
// unrolled, so W stays in VGPRs)
__device__ __forceinline__ void acgt_key_regs(const uint32_t (&W)[8], uint32_t L, uint32_t D, uint32_t E, uint32_t lmin, uint32_t lmax,
                                              uint32_t& x_out, uint64_t& rem_out, bool& term_out) {
    uint64_t V = 0;
    bool ok = true, term = lmax != 0 && (L < lmin || L > lmax);
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) {
        const uint32_t j = 4 * k;
        if (j < L) {
            const uint32_t n = min(4u, L - j);
            const uint32_t w = W[k];
            const uint32_t live = n == 4 ? 0x80808080u : (0x80808080u >> (8 * (4 - n)));
            const uint32_t mC = zero_bytes(w ^ 0x43434343u), mG = zero_bytes(w ^ 0x47474747u), mT = zero_bytes(w ^ 0x54545454u);
            const uint32_t hit = zero_bytes(w ^ 0x41414141u) | mC | mG | mT;
            ok &= (hit & live) == live;
            term |= (zero_bytes(w ^ 0x23232323u) & live) != 0;
            const uint32_t bad = ~hit & 0x80808080u;
            const uint32_t q = ((mC | mT | bad) >> 7) | ((mG | mT | bad) >> 6);
            const uint32_t pk = ((q & 3u) << 6) | (((q >> 8) & 3u) << 4) | (((q >> 16) & 3u) << 2) | ((q >> 24) & 3u);
            V = (V << (2 * n)) | (pk >> (8 - 2 * n));
        }
    }
    if (L <= D) {
        x_out = ok ? (uint32_t)V : E;
        rem_out = 1ull;
    } else {
        x_out = ok ? (uint32_t)(V & ((1ull << (2 * D)) - 1ull)) : E;
        rem_out = (V >> (2 * D)) | pk_digit(1, L - D);
    }
    term_out = term;
}

// Stage the bytes of the block's patterns [base, base + nb) in LDS (16-B aligned words from
// w0 = off[base] & ~15) when they fit kKeySpan and the buffer is 16-B aligned; every thread of
// the block calls it.  Returns whether they were staged.
__device__ __forceinline__ bool stage_patterns(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, size_t base, size_t nb,
                                               uint4* sbuf4, uint64_t& w0) {
    const uint64_t s0 = off[base], s1 = off[base + nb];
    w0 = s0 & ~15ull;
    const bool staged = s1 - w0 + 16 <= kKeySpan && ((uintptr_t)bytes & 15) == 0;
    __syncthreads();
    if (staged) {
        const uint32_t nw = (uint32_t)((s1 - w0 + 15) / 16);
        const uint4* src = reinterpret_cast<const uint4*>(bytes + w0);
        for (uint32_t t = threadIdx.x; t < nw; t += blockDim.x) sbuf4[t] = src[t];
    }
    __syncthreads();
    return staged;
}

__global__ void __launch_bounds__(256) k_keys_acgt(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, uint64_t P,
                                                   uint32_t* __restrict__ len, unsigned long long* __restrict__ n_term, uint32_t D,
                                                   uint32_t E, uint32_t* __restrict__ kid, uint64_t* __restrict__ pv, uint32_t lmin,
                                                   uint32_t lmax) {
    // lmax != 0: the batch's lengths were not measured (no k_lminmax read-back); a pattern outside
    // [lmin, lmax] counts as one holding '#', so the deferred check sends the batch to the checked path
    __shared__ uint4 sbuf4[kKeySpan / 16 + 2];
    __shared__ unsigned long long sh[4];
    const uint32_t* sbuf = reinterpret_cast<const uint32_t*>(sbuf4);
    unsigned long long nt = 0;
    for (size_t base = (size_t)blockIdx.x * blockDim.x; base < P; base += (size_t)gridDim.x * blockDim.x) {
        const size_t nb = min((size_t)blockDim.x, (size_t)P - base);
        uint64_t w0;
        const bool staged = stage_patterns(bytes, off, base, nb, sbuf4, w0);
        const size_t i = base + threadIdx.x;
        if (i < P) {
            const uint64_t a = off[i];
            const uint32_t L = (uint32_t)(off[i + 1] - a);
            len[i] = L;
            uint32_t x;
            uint64_t rem;
            bool term;
            acgt_key(bytes, a, L, staged, sbuf, (uint32_t)(a - w0), D, E, lmin, lmax, x, rem, term);
            nt += term;
            pv[i] = rem << 31 | (uint64_t)i;
            kid[i] = x;
        }
    }
    nt = block_sum(nt, sh);
    if (threadIdx.x == 0 && nt) atomicAdd(n_term, nt);
}

// direct start: patterns grouped by their D-mer's leading bits (kid >> shift) for locality —
// neighbouring lanes then read neighbouring table entries and rows.  cur[] holds each
// bucket's first slot (exclusive scan of k_keys' histogram) and is advanced by atomics, so
// the order inside a bucket is arbitrary: nothing downstream depends on it (results are
// written by input index, carried in the packed start)
__global__ void k_bucket_scatter(uint64_t P, const uint32_t* __restrict__ kid, const uint64_t* __restrict__ pv, uint32_t shift,
                                 uint32_t* __restrict__ cur, uint32_t* __restrict__ kid_out, uint64_t* __restrict__ pv_out) {
    GRID_STRIDE(i, P) {
        const uint32_t k = kid[i];
        const uint32_t at = atomicAdd(&cur[k >> shift], 1u);
        kid_out[at] = k;
        pv_out[at] = pv[i];
    }
}

// group of a pattern = its last k characters' sort codes (0 past the pattern's start),
// i.e. its depth-k node of the reversed-pattern trie, in base sigma+2
__global__ void k_pattern_group(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, uint64_t P,
                                const uint8_t* __restrict__ code_of, uint32_t sigma, uint32_t k, uint32_t* __restrict__ gid) {
    GRID_STRIDE(i, P) {
        const uint64_t a = off[i], L = off[i + 1] - a;
        uint32_t g = 0;
        for (uint32_t t = 0; t < k; t++) {
            uint32_t v = 0;
            if (t < L) {
                const uint32_t c = code_of[bytes[a + L - 1 - t]];
                v = c < sigma ? c + 1 : sigma + 1;
            }
            g = g * (sigma + 2) + v;
        }
        gid[i] = g;
    }
}

__global__ void k_eq_flag(const uint32_t* __restrict__ v, uint64_t n, uint32_t x, uint32_t* __restrict__ flag) {
    GRID_STRIDE(i, n) flag[i] = v[i] == x;
}

__global__ void k_gather_key(const uint64_t* __restrict__ keys_c, const uint32_t* __restrict__ perm, uint64_t P, uint64_t* __restrict__ out) {
    GRID_STRIDE(i, P) out[i] = keys_c[perm[i]];
}

// Sorted order, from the sorted key chunks alone (chunk 0 in k0, chunks 1.. in
// krest[(c-1)*P + i]; neighbours are adjacent, so every read coalesces):
//   slen[i] = pattern length (its codes are nonzero up to the end of the pattern);
//   lcp[i]  = common reversed prefix (= common suffix) of neighbours i-1, i;
//   *ties  += neighbours equal in chunk 0 but not later (the order is then not a trie order)
template <int BPS>
__device__ __forceinline__ uint32_t key_len(const uint64_t* __restrict__ k0, const uint64_t* __restrict__ krest, uint32_t nch, uint64_t P,
                                            size_t i) {
    constexpr uint32_t SPC = 64 / BPS;
    for (int c = (int)nch - 1; c >= 0; c--) {
        const uint64_t k = c == 0 ? k0[i] : krest[(size_t)(c - 1) * P + i];
        if (k) return (uint32_t)c * SPC + SPC - (uint32_t)__builtin_ctzll(k) / BPS;
    }
    return 0;
}

template <int BPS>
__global__ void __launch_bounds__(256) k_slen_lcp(const uint64_t* __restrict__ k0, const uint64_t* __restrict__ krest, uint32_t nch, uint64_t P,
                                                  uint32_t* __restrict__ slen, uint32_t* __restrict__ lcp, unsigned long long* __restrict__ ties) {
    constexpr uint32_t SPC = 64 / BPS, LEAD = 64 - SPC * BPS;
    __shared__ unsigned long long sh[4];
    unsigned long long nt = 0;
    GRID_STRIDE(i, P) {
        const uint32_t la = key_len<BPS>(k0, krest, nch, P, i);
        slen[i] = la;
        if (i == 0) { lcp[0] = 0; continue; }
        const uint32_t lb = key_len<BPS>(k0, krest, nch, P, i - 1);
        uint32_t l = SPC * nch;
        for (uint32_t c = 0; c < nch; c++) {
            const uint64_t x = c == 0 ? (k0[i] ^ k0[i - 1]) : (krest[(size_t)(c - 1) * P + i] ^ krest[(size_t)(c - 1) * P + i - 1]);
            if (x) {
                l = c * SPC + ((uint32_t)__clzll(x) - LEAD) / BPS;
                nt += c > 0;
                break;
            }
        }
        l = l < la ? l : la;
        l = l < lb ? l : lb;
        lcp[i] = l;
    }
    nt = block_sum(nt, sh);
    if (threadIdx.x == 0 && nt) atomicAdd(ties, nt);
}

// After the chunk-0 sort: order each tie group (run of equal chunk 0) by the later chunks,
// one thread per group, insertion sort (linear on groups of identical patterns).  Groups
// over kTieMax members are left alone and counted: the caller then runs the full sort.
constexpr uint32_t kTieMax = 256;
__global__ void __launch_bounds__(256) k_fix_ties(const uint64_t* __restrict__ k0, uint64_t* __restrict__ krest, uint32_t nch, uint64_t P,
                                                  uint32_t* __restrict__ perm, unsigned long long* __restrict__ big) {
    GRID_STRIDE(i, P) {
        if (i + 1 >= P || k0[i] != k0[i + 1] || (i > 0 && k0[i - 1] == k0[i])) continue;
        size_t j = i + 1;
        while (j < P && k0[j] == k0[i] && j - i <= kTieMax) j++;
        if (j - i > kTieMax) { atomicAdd(big, 1ull); continue; }
        auto less = [&](size_t a, size_t b) {  // chunk-wise (later chunks) a < b
            for (uint32_t c = 1; c < nch; c++) {
                const uint64_t x = krest[(size_t)(c - 1) * P + a], y = krest[(size_t)(c - 1) * P + b];
                if (x != y) return x < y;
            }
            return false;
        };
        for (size_t a = i + 1; a < j; a++) {
            size_t b = a;
            while (b > i && less(b, b - 1)) {  // bubble a down to its place
                const uint32_t tp = perm[b]; perm[b] = perm[b - 1]; perm[b - 1] = tp;
                for (uint32_t c = 1; c < nch; c++) {
                    uint64_t* r = krest + (size_t)(c - 1) * P;
                    const uint64_t t = r[b]; r[b] = r[b - 1]; r[b - 1] = t;
                }
                b--;
            }
        }
    }
}

// longest pattern, from the offsets alone (small grid, one atomic per block)
__global__ void __launch_bounds__(256) k_lmax(const uint64_t* __restrict__ off, uint64_t P, unsigned long long* __restrict__ out) {
    __shared__ unsigned int smx;
    if (threadIdx.x == 0) smx = 0;
    __syncthreads();
    uint32_t mx = 0;
    GRID_STRIDE(i, P) mx = max(mx, (uint32_t)(off[i + 1] - off[i]));
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, o, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(&smx, mx);
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(out, (unsigned long long)smx);
}

// longest and shortest pattern: out[0] = max length, out[1] = ~min length (both by atomicMax)
__global__ void __launch_bounds__(256) k_lminmax(const uint64_t* __restrict__ off, uint64_t P, unsigned long long* __restrict__ out) {
    __shared__ unsigned int smx, smn;
    if (threadIdx.x == 0) smx = smn = 0;
    __syncthreads();
    uint32_t mx = 0, nmn = 0;
    // four lengths per thread and round: two 16-B loads and the next group's first offset
    // (a 16-B aligned array; else one offset pair at a time)
    const uint64_t P4 = ((uintptr_t)off & 15) == 0 ? P / 4 : 0;
    const ulonglong2* o2 = reinterpret_cast<const ulonglong2*>(off);
    GRID_STRIDE(g, P4) {
        const ulonglong2 a = o2[2 * g], b = o2[2 * g + 1];
        const uint64_t c = off[4 * g + 4];
        const uint32_t l0 = (uint32_t)(a.y - a.x), l1 = (uint32_t)(b.x - a.y), l2 = (uint32_t)(b.y - b.x), l3 = (uint32_t)(c - b.y);
        mx = max(max(mx, max(l0, l1)), max(l2, l3));
        nmn = max(max(nmn, max(~l0, ~l1)), max(~l2, ~l3));
    }
    GRID_STRIDE(j, P - 4 * P4) {
        const uint64_t i = 4 * P4 + j;
        const uint32_t L = (uint32_t)(off[i + 1] - off[i]);
        mx = max(mx, L);
        nmn = max(nmn, ~L);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        mx = max(mx, (uint32_t)__shfl_xor(mx, o, 64));
        nmn = max(nmn, (uint32_t)__shfl_xor(nmn, o, 64));
    }
    if ((threadIdx.x & 63) == 0) { atomicMax(&smx, mx); atomicMax(&smn, nmn); }
    __syncthreads();
    if (threadIdx.x == 0) { atomicMax(out, (unsigned long long)smx); atomicMax(out + 1, (unsigned long long)smn); }
}

// node starts at depth D: pattern i is the first member of a depth-D node
__global__ void k_node_flags(const uint32_t* __restrict__ slen, const uint32_t* __restrict__ lcp, uint64_t P, uint32_t D, uint32_t* __restrict__ flag) {
    GRID_STRIDE(i, P) flag[i] = (slen[i] >= D && lcp[i] < D) ? 1u : 0u;
}

// nscan = exclusive scan of flags (P+1 entries); skey = the sorted patterns'
// reversed-code chunk holding depth D (BPS bits per symbol, most significant first)
// node-start flag of pattern i at depth D (scanned on the fly by the host's transform scan)
// a result's occurrence count (the per-pattern locate's scan input, read straight from the results)
struct ResOcc {
    __host__ __device__ __forceinline__ uint32_t operator()(const Res& r) const {
        return (r.cnt & 0x40000000u) ? 1u : r.occ;  // res_occ (kResPos: one occurrence)
    }
};

struct NodeFlag {
    const uint32_t* slen;
    const uint32_t* lcp;
    uint32_t D;
    __host__ __device__ __forceinline__ uint32_t operator()(uint32_t i) const { return (slen[i] >= D && lcp[i] < D) ? 1u : 0u; }
};

template <int BPS>
__global__ void k_node_build(uint64_t P, uint32_t D, const uint32_t* __restrict__ slen, const uint64_t* __restrict__ skey, uint32_t sigma,
                             const uint32_t* __restrict__ lcp, const uint32_t* __restrict__ nscan,
                             const uint32_t* __restrict__ nid_prev, uint32_t* __restrict__ nid_cur,
                             uint32_t* __restrict__ node_first, uint32_t* __restrict__ node_parent, uint8_t* __restrict__ node_char) {
    constexpr uint32_t SPC = 64 / BPS;
    const uint32_t sh = BPS * (SPC - 1 - ((D - 1) % SPC));
    GRID_STRIDE(i, P) {
        if (slen[i] < D) { nid_cur[i] = 0xFFFFFFFFu; continue; }
        const uint32_t f = lcp[i] < D;
        const uint32_t id = nscan[i] + f - 1;
        nid_cur[i] = id;
        if (f) {
            node_first[id] = (uint32_t)i;
            node_parent[id] = nid_prev[i];
            const uint32_t v = (uint32_t)(skey[i] >> sh) & ((1u << BPS) - 1u);
            node_char[id] = (uint8_t)((v >= 1 && v <= sigma) ? v - 1 : 0xFF);
        }
    }
}

// children of each parent are contiguous: [child_first[p], child_end[p])
__global__ void k_child_links(const uint32_t* __restrict__ node_parent, uint32_t M, uint32_t* __restrict__ child_first, uint32_t* __restrict__ child_end) {
    GRID_STRIDE(u, M) {
        const uint32_t p = node_parent[u];
        if (u == 0 || node_parent[u - 1] != p) child_first[p] = (uint32_t)u;
        if (u + 1 == M || node_parent[u + 1] != p) child_end[p] = (uint32_t)u + 1;
    }
}

// ---------------------------------------------------------- interval lists
// owner-sorted list → [off[u], end[u]) per owner (arrays zeroed by the caller)
__global__ void k_bounds(const uint32_t* __restrict__ owner, uint64_t n, uint32_t* __restrict__ off, uint32_t* __restrict__ end) {
    GRID_STRIDE(t, n) {
        const uint32_t u = owner[t];
        if (t == 0 || owner[t - 1] != u) off[u] = (uint32_t)t;
        if (t + 1 == n || owner[t + 1] != u) end[u] = (uint32_t)t + 1;
    }
}

// EXPAND: rank of every symbol at b and at e+1 (2 occ-block lines per interval)
__global__ void __launch_bounds__(256) k_expand(const uint32_t* __restrict__ ib, const uint32_t* __restrict__ ie, uint64_t n, KIdx X,
                                                uint32_t* __restrict__ ocb, uint32_t* __restrict__ oce) {
    GRID_STRIDE(j, n) {
        uint32_t rb[8], re[8];
        rank_all_pair_any(X, ib[j], ie[j] + 1, rb, re);
        uint4* pb = reinterpret_cast<uint4*>(ocb + j * 8);
        uint4* pe = reinterpret_cast<uint4*>(oce + j * 8);
        pb[0] = make_uint4(rb[0], rb[1], rb[2], rb[3]);
        pb[1] = make_uint4(rb[4], rb[5], rb[6], rb[7]);
        pe[0] = make_uint4(re[0], re[1], re[2], re[3]);
        pe[1] = make_uint4(re[4], re[5], re[6], re[7]);
    }
}

// LINK step 1: number of '#' rows in each interval whose node has children
// (dollars_in_interval, MOVE_EDSBWTSearch.cpp:607-625)
__global__ void k_hash_counts(const uint32_t* __restrict__ owner, const uint32_t* __restrict__ ocb, const uint32_t* __restrict__ oce,
                              const uint32_t* __restrict__ child_first, const uint32_t* __restrict__ child_end, uint64_t n,
                              uint32_t* __restrict__ h) {
    GRID_STRIDE(j, n) {
        const uint32_t u = owner[j];
        h[j] = (child_end[u] > child_first[u]) ? oce[j * 8] - ocb[j * 8] : 0u;
    }
}

// LINK step 2: one key per '#' row: (owner << 32 | segment of its word) when the
// word is past segment 1 (index > first_symbol_index, :620), else a sentinel.
__global__ void k_link_emit(uint64_t H, const uint32_t* __restrict__ hoff, uint64_t n, const uint32_t* __restrict__ ocb,
                            const uint32_t* __restrict__ owner, const uint32_t* __restrict__ eof_seg,
                            uint64_t* __restrict__ keys, unsigned long long* __restrict__ nvalid) {
    GRID_STRIDE(t, H) {
        const size_t j = upper_bound_dev<uint32_t>(hoff, n, (uint32_t)t) - 1;
        const uint32_t k = ocb[j * 8] + ((uint32_t)t - hoff[j]);
        const uint32_t s = eof_seg[k];
        uint64_t key = ~0ull;
        if (s) {
            key = ((uint64_t)owner[j] << 32) | s;
            atomicAdd(nvalid, 1ull);
        }
        keys[t] = key;
    }
}

// LINK step 3: union of previous-segment ranges [seg_lo[s], s-1] per owner
// (the deque walk of link(), :533-561, yields exactly these maximal runs, ascending)
// keys: node << sb | segment
// seg_chain (optional): bit s set when seg_lo[s] != s - 1 (segment s - 1 holds an empty word); a
// clear bit settles a key that does not touch its predecessor without the seg_lo gather (an
// 11 MB bitmap at C5 stays in the caches, seg_lo's 352 MB does not)
// cb = 1: the keys are node << (sb + 1) | segment << 1 | chain bit (KIdx::link_cb), and a clear
// chain bit settles the key with no read at all
__global__ void k_run_flags(const uint64_t* __restrict__ keys, uint64_t V, const uint32_t* __restrict__ seg_lo, uint32_t sb,
                            uint32_t* __restrict__ flag, const uint32_t* __restrict__ seg_chain, uint32_t cb) {
    const uint64_t sm = (1ull << sb) - 1;
    const uint32_t ns = sb + cb;
    // four keys per lane, a grid stride apart: their seg_lo gathers (random, L2-missing) are
    // independent and in flight together
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t0 < V; t0 += 4 * stride) {
        uint32_t f[4], s[4], sp[4];
        bool need[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const size_t t = t0 + q * stride;
            f[q] = 1;
            need[q] = false;
            s[q] = sp[q] = 0;
            if (t < V && t) {
                const uint64_t k = keys[t], kp = keys[t - 1];
                s[q] = (uint32_t)((k >> cb) & sm);
                sp[q] = (uint32_t)((kp >> cb) & sm);
                if ((kp >> ns) == (k >> ns)) {
                    // seg_lo[s] <= s - 1: a key one segment after (or equal to) its
                    // predecessor continues the run without the gather
                    if (sp[q] + 1 >= s[q]) f[q] = 0;
                    else need[q] = cb ? (k & 1) != 0 : !seg_chain || ((seg_chain[s[q] >> 5] >> (s[q] & 31)) & 1);
                }
            }
        }
        uint32_t lo[4];
#pragma unroll
        for (int q = 0; q < 4; q++) lo[q] = need[q] ? seg_lo[s[q]] : 0u;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const size_t t = t0 + q * stride;
            if (need[q] && lo[q] <= sp[q]) f[q] = 0;
            if (t < V) flag[t] = f[q];
        }
    }
}

__global__ void k_run_build(const uint64_t* __restrict__ keys, uint64_t V, const uint32_t* __restrict__ flag, const uint32_t* __restrict__ rscan,
                            const uint32_t* __restrict__ seg_lo, const uint32_t* __restrict__ seg_start, uint32_t sb,
                            uint32_t* __restrict__ rb, uint32_t* __restrict__ re, uint32_t* __restrict__ rown,
                            uint32_t* __restrict__ nruns) {
    GRID_STRIDE(t, V) {
        if (nruns && t + 1 == V) *nruns = rscan[t] + flag[t];
        const uint64_t k = keys[t];
        const uint32_t s = (uint32_t)(k & ((1ull << sb) - 1));
        const uint32_t r = rscan[t] + flag[t] - 1;
        if (flag[t]) {
            rb[r] = seg_start[seg_lo[s]];
            rown[r] = (uint32_t)(k >> sb);
        }
        if (t + 1 == V || flag[t + 1]) re[r] = seg_start[s] - 1;
    }
}

// order-free path: a run is kept as its first and last segment (s_first, s_last): it
// covers the words of segments [seg_lo[s_first], s_last - 1], whose c-ranks at both
// ends the segment table holds — no row lookups here, no occ lines in k_lvl_dollar
__global__ void k_run_build_seg(const uint64_t* __restrict__ keys, uint64_t V, const uint32_t* __restrict__ flag,
                                const uint32_t* __restrict__ rscan, uint32_t sb, uint32_t* __restrict__ rs0, uint32_t* __restrict__ rs1,
                                uint32_t* __restrict__ rown, uint32_t* __restrict__ nruns, uint32_t cb) {
    GRID_STRIDE(t, V) {
        if (nruns && t + 1 == V) *nruns = rscan[t] + flag[t];
        const uint64_t k = keys[t];
        const uint32_t s = (uint32_t)((k >> cb) & ((1ull << sb) - 1));
        const uint32_t r = rscan[t] + flag[t] - 1;
        if (flag[t]) {
            rs0[r] = s;
            rown[r] = (uint32_t)(k >> (sb + cb));
        }
        if (t + 1 == V || flag[t + 1]) rs1[r] = s;
    }
}

// STEP: per child node, its parent's list [dollar ranges..., own intervals...]
// stepped by the child's symbol (backward_search_step + updateSingleInterval,
// :376-510; concatenation order of :300).
__global__ void k_task_counts(uint32_t M, const uint32_t* __restrict__ node_parent, const uint32_t* __restrict__ doff, const uint32_t* __restrict__ dend,
                              const uint32_t* __restrict__ ioff, const uint32_t* __restrict__ iend, uint32_t* __restrict__ tcnt) {
    GRID_STRIDE(u, M) {
        const uint32_t p = node_parent[u];
        tcnt[u] = (dend[p] - doff[p]) + (iend[p] - ioff[p]);
    }
}

__global__ void __launch_bounds__(256) k_step(uint64_t T, const uint32_t* __restrict__ toff, uint32_t M,
                                              const uint32_t* __restrict__ node_parent, const uint8_t* __restrict__ node_char,
                                              const uint32_t* __restrict__ doff, const uint32_t* __restrict__ dend,
                                              const uint32_t* __restrict__ ioff,
                                              const uint32_t* __restrict__ docb, const uint32_t* __restrict__ doce,
                                              const uint32_t* __restrict__ iocb, const uint32_t* __restrict__ ioce, KIdx X,
                                              uint32_t* __restrict__ ob, uint32_t* __restrict__ oe, uint32_t* __restrict__ ou,
                                              uint32_t* __restrict__ flag) {
    GRID_STRIDE(t, T) {
        const uint32_t u = (uint32_t)(upper_bound_dev<uint32_t>(toff, M, (uint32_t)t) - 1);
        const uint32_t p = node_parent[u];
        const uint32_t j = (uint32_t)t - toff[u];
        const uint32_t nd = dend[p] - doff[p];
        const uint32_t c = node_char[u];
        uint32_t f = 0, b = 0, e = 0;
        if (c < X.sigma) {
            uint32_t lo, hi;
            if (j < nd) {
                const size_t s = (size_t)(doff[p] + j) * 8 + c;
                lo = docb[s];
                hi = doce[s];
            } else {
                const size_t s = (size_t)(ioff[p] + j - nd) * 8 + c;
                lo = iocb[s];
                hi = ioce[s];
            }
            if (hi > lo) {
                f = 1;
                b = X.C[c] + lo;
                e = X.C[c] + hi - 1;
            }
        }
        ob[t] = b;
        oe[t] = e;
        ou[t] = u;
        flag[t] = f;
    }
}

// stream compaction (order-preserving): fscan = exclusive scan of flag
__global__ void k_compact3(uint64_t n, const uint32_t* __restrict__ flag, const uint32_t* __restrict__ fscan,
                           const uint32_t* __restrict__ a, const uint32_t* __restrict__ b, const uint32_t* __restrict__ c,
                           uint32_t* __restrict__ oa, uint32_t* __restrict__ ob, uint32_t* __restrict__ oc) {
    GRID_STRIDE(t, n) {
        if (flag[t]) {
            const uint32_t d = fscan[t];
            oa[d] = a[t];
            ob[d] = b[t];
            oc[d] = c[t];
        }
    }
}

// adjacency merge inside each child (:309-324): a new run unless start == last.end+1
__global__ void k_merge_flags(uint64_t n, const uint32_t* __restrict__ cb, const uint32_t* __restrict__ ce, const uint32_t* __restrict__ cu,
                              uint32_t* __restrict__ flag) {
    GRID_STRIDE(t, n) {
        uint32_t f = 1;
        if (t && cu[t] == cu[t - 1] && cb[t] == ce[t - 1] + 1) f = 0;
        flag[t] = f;
    }
}

__global__ void k_merge_build(uint64_t n, const uint32_t* __restrict__ flag, const uint32_t* __restrict__ mscan,
                              const uint32_t* __restrict__ cb, const uint32_t* __restrict__ ce, const uint32_t* __restrict__ cu,
                              uint32_t* __restrict__ nb, uint32_t* __restrict__ ne, uint32_t* __restrict__ nu) {
    GRID_STRIDE(t, n) {
        const uint32_t r = mscan[t] + flag[t] - 1;
        if (flag[t]) {
            nb[r] = cb[t];
            nu[r] = cu[t];
        }
        if (t + 1 == n || flag[t + 1]) ne[r] = ce[t];
    }
}

// ------------------------------------------------------------- deep phase
// One thread per pattern whose trie node stopped sharing work: the rest of
// backwardSearch (link → step both piles → merge, MOVE_EDSBWTSearch.cpp:254-325)
// runs with the interval lists in registers (at most K each).  A pattern whose
// lists outgrow K, or whose link reads more than K '#' rows at once, is flagged and
// re-run by the level-synchronous path, which has no size limit.
// Symbol codes of sorted pattern i from its reversed sort-code chunks (chunk 0 in k0,
// chunk c >= 1 at krest[(c-1)*P + i]; BPS bits per symbol, most significant first): the
// deep kernels read a pattern's remaining symbols one coalesced chunk at a time instead of
// byte by byte.  code(d) = symbol code of the d-th character from the pattern's end (d < its
// length); >= sigma for a byte outside the alphabet.
template <int BPS>
struct SymReader {
    const uint64_t* k0;
    const uint64_t* krest;
    uint64_t P;
    size_t i;
    uint64_t cur = 0;
    uint32_t chunk = ~0u;
    __device__ __forceinline__ uint32_t code(uint32_t d) {
        constexpr uint32_t SPC = 64 / BPS;
        const uint32_t c = d / SPC, t = d - c * SPC;
        if (c != chunk) {
            cur = c == 0 ? k0[i] : krest[(size_t)(c - 1) * P + i];
            chunk = c;
        }
        return (uint32_t)((cur >> (BPS * (SPC - 1 - t))) & ((1u << BPS) - 1u)) - 1u;
    }
};

// Deep stage, two kernels.  k_deep_fast walks every pattern whose list is one interval
// with two registers, as long as no step meets '#' rows (no link); a pattern that needs
// a list or a link is queued as (pattern, depth, b, e) — b = ~0u: "from its node's
// items" — and k_deep finishes the queued ones with register lists.  The queue is
// sharded like the item appends (region s at s*qcap, counter s at qcnt[s*32]).
template <int BPS, int MINW = 1>  // MINW: waves per SIMD the register budget is held to (1: no bound)
__global__ void __launch_bounds__(256, MINW) k_deep_fast(uint64_t P, uint32_t D0, const uint32_t* __restrict__ slen, const uint32_t* __restrict__ perm,
                                                   const uint64_t* __restrict__ k0, const uint64_t* __restrict__ krest, uint32_t ind,
                                                   const uint32_t* __restrict__ nid,
                                                   const uint32_t* __restrict__ ioff, const uint32_t* __restrict__ iend,
                                                   const uint32_t* __restrict__ ib, const uint32_t* __restrict__ ie, KIdx X, uint64_t abase,
                                                   uint32_t K, uint32_t* __restrict__ ab, uint32_t* __restrict__ ae,
                                                   Res* __restrict__ res,
                                                   uint4* __restrict__ q, uint32_t qcap, uint32_t* __restrict__ qcnt,
                                                   unsigned long long* __restrict__ ctr, const uint64_t* __restrict__ pv,
                                                   uint32_t* __restrict__ perm_out, const uint64_t* __restrict__ kt1,
                                                   uint64_t* __restrict__ q2, const uint4* __restrict__ kt1w) {
    uint32_t n_steps = 0, n_blk = 0, n_pl = 0, n_text = 0, n_trow = 0, n_lane = 0, n_wave = 0;  // per lane (widened at the end)
    const uint32_t sh = blockIdx.x % NSHARD;
    q += (size_t)sh * qcap;
    if (q2) q2 += (size_t)sh * qcap;
    UNIFORM_STRIDE(i, valid, P) {
        uint32_t want = 0;
        uint32_t rounds = valid ? 1u : 0u;  // dependent load rounds of this lane's pattern
        uint4 w = make_uint4(0, 0, 0, 0);
        // ind: slen and the key chunks are in input order, pattern i (sorted) is input perm[i].
        // pv (packed direct start): input index and remaining symbols sorted along with the
        // D-mers, so neither slen nor the key chunks are read; perm is written for k_deep
        uint32_t pi, L;
        uint64_t rem = 0, pvv = 0;
        if (pv) {
            const uint64_t v = valid ? pv[i] : 0ull;
            pvv = v;
            pi = (uint32_t)(v & 0x7fffffffu);
            rem = v >> 31;
            L = valid ? pk_len(D0, rem) : 0u;
            if (valid) perm_out[i] = pi;
        } else {
            pi = valid && ind ? perm[i] : (uint32_t)i;
            L = valid ? slen[pi] : 0u;
        }
        const uint32_t u = L > D0 ? nid[i] : 0u;
        // kt1 (direct start): the D-mer's one interval inline, or its list's length; kt1w (the
        // wide form) also holds a one-row entry's sample and the 32 text characters before it
        const bool dtab = kt1 || kt1w;
        uint64_t ent = 0, win1 = 0;
        uint4 s1 = make_uint4(0, 0, 0, 0);
        if (L > D0 && kt1w) {
            const uint4 w0 = kt1w[(size_t)X.kt1_ws * u];
            s1 = kt1w[(size_t)X.kt1_ws * u + 1];
            ent = (uint64_t)w0.y << 32 | w0.x;
            win1 = (uint64_t)w0.w << 32 | w0.z;
        } else if (L > D0 && kt1) {
            ent = kt1[u];
        }
        const uint32_t n0 = L <= D0 ? 0u : dtab ? ((ent >> 63) ? 1u : (uint32_t)(ent >> 32)) : iend[u] - ioff[u];
        if (n0 > 1) {
            want = 1;
            // (the wide table: k_deep reads the list from the D-mer's entry, w.w)
            w = make_uint4((uint32_t)i, D0, kt1w ? kQWide : kQNode, kt1w ? u : 0u);
        } else if (n0 == 1) {
            uint32_t b, e;
            uint32_t g1 = ~0u;  // the row's text position when the table entry holds it
            if (dtab) {
                if (X.kt1_pos && ((ent >> 62) & 1)) {
                    b = e = (uint32_t)ent & 0x7fffffffu;
                    g1 = (uint32_t)(ent >> 31) & 0x7fffffffu;
                } else {
                    b = (uint32_t)ent;
                    e = (uint32_t)(ent >> 32) & 0x7fffffffu;
                }
            } else {
                b = ib[ioff[u]];
                e = ie[ioff[u]];
            }
            SymReader<BPS> sym{k0, krest, P, pi};
            auto code_at = [&](uint32_t dd) -> uint32_t {
                return pv ? 1u + (uint32_t)((rem >> (2 * (dd - D0))) & 3u) : sym.code(dd);
            };
            bool alive = true;
            uint32_t d = D0;
            bool pair_skip = false;  // the pair entry just found '#' rows: take one step
            uint32_t tri_from = 0;   // no three-step attempt before this depth (one just failed)
            bool posres = false;     // answered by the text compare: (word, offset) result written
            for (bool first = true; X.rtext && b == e && d < L; first = false) {
                // One row = one text position (word w, offset o): while no '#' row is met (o > 0)
                // each backward step keeps one row and succeeds iff the text character before it
                // equals the pattern's, so the next k = min(o, m) characters are decided by comparing
                // them with the text (MOVE_EDSBWTSearch.cpp:424-510 stepping one row)
                rounds++;
                // the wide entry brought the first row's sample and text window with it (one line)
                // (or the per-row entry: sample, text position and window in one line)
                const bool wide = first && g1 != ~0u && kt1w, sr = !wide && X.srow;
                uint4 s;
                uint32_t g;
                uint64_t w0 = win1;
                if (wide) {
                    s = s1;
                    g = g1;
                } else if (sr) {
                    s = X.srow[2 * (size_t)b];
                    const uint4 t2 = X.srow[2 * (size_t)b + 1];
                    g = t2.x;
                    w0 = (uint64_t)t2.w << 32 | t2.z;
                } else {
                    s = X.samples[b];
                    g = first && g1 != ~0u ? g1 : X.gpos[b];
                }
                n_blk += wide || sr ? 1 : first && g1 != ~0u ? 2 : 3;
                n_trow++;
                const uint32_t m = L - d, k = min(s.y, m);
                bool eq = true, valid_codes = true;
                const uint64_t r0 = X.tlen - g;  // reversed index of the text character before row b's suffix
                for (uint32_t j = 0; j < k && eq; j += 32) {
                    const uint32_t n = min(32u, k - j);
                    const uint64_t mask = n == 32 ? ~0ull : ((1ull << (2 * n)) - 1ull);
                    uint64_t want = 0;
                    if (pv) {
                        want = (rem >> (2 * (d + j - D0))) & mask;  // the packed start's 2-bit digits (<= 16)
                    } else {
                        for (uint32_t t = 0; t < n; t++) {
                            const uint32_t c = code_at(d + j + t);
                            if (c == 0) { valid_codes = false; break; }  // '#' in the pattern: walk it
                            if (c >= X.sigma) { eq = false; break; }      // outside the alphabet: no match
                            want |= (uint64_t)(c - 1) << (2 * t);
                        }
                        if (!valid_codes || !eq) break;
                    }
                    eq = ((((wide || sr) && j == 0 ? w0 : rtext_window(X.rtext, r0 + j)) ^ want) & mask) == 0;
                }
                if (!valid_codes) break;  // '#' in the pattern: the walk below takes it
                if (!eq) {
                    alive = false;
                    d = L;
                    break;
                }
                if (s.y >= m) {
                    if (s.w <= kResCnt) {  // else (a segment of 2^30 words) the walk below decides
                        posres = true;
                        n_text += m;
                        d = L;
                        put_res(res, pv ? pi : perm[i], (uint64_t)(s.y - m) << 32 | s.x, kResRow | kResPos | s.w, s.z);
                    }
                    break;
                }
                // the word's first o characters matched: its whole-word row is the '#' row of word
                // s.x, so the next step is the link (:512-563) from ONE segment, s.z — the words of
                // segments [seg_lo[s.z], s.z - 1] by the next character, one interval from the
                // segment table (what k_deep would do after a rank and an eof_seg read)
                n_text += s.y;
                d += s.y;
                const uint32_t c = code_at(d);
                if (c == 0 || c >= X.sigma) {  // '#' or outside the alphabet: the walk below decides
                    b = e = X.wrow[s.x];
                    n_blk++;
                    break;
                }
                if (s.z < 2) {  // the first segment: no previous words (eof_seg 0)
                    alive = false;
                    d = L;
                    break;
                }
                const uint32_t* et = X.segtab + (size_t)s.z * X.seg_stride;
                const uint32_t rx = et[1 + c], ry = et[X.seg_hi + c];
                n_blk++;
                n_steps++;
                if (ry <= rx) {
                    alive = false;
                    d = L;
                    break;
                }
                b = X.C[c] + rx;
                e = X.C[c] + ry - 1;
                d++;
            }
            for (; d < L; d++) {
                const uint32_t c = code_at(d);
                if (c >= X.sigma) { alive = false; break; }
                rounds++;
                // three characters from one rank entry per end (rent3), as the pair below
                if (X.rent3 && d >= tri_from && d + 2 < L && c != 0) {
                    const uint32_t c2 = code_at(d + 1), c3 = code_at(d + 2);
                    if (c2 != 0 && c2 < X.sigma && c3 != 0 && c3 < X.sigma) {
                        const uint32_t B = X.sigma - 1;
                        const uint32_t t = ((c - 1) * B + (c2 - 1)) * B + (c3 - 1);
                        const uint4 v0 = X.rent3[(size_t)(b >> 5) * X.r3stride + t];
                        const uint4 v1 = X.rent3[(size_t)((e + 1) >> 5) * X.r3stride + t];
                        uint32_t p0, x0, p1, x1;
                        rent_rank(v0, b, p0, x0);
                        rent_rank(v1, e + 1, p1, x1);
                        const uint32_t nl = (b >> 5) == ((e + 1) >> 5) ? 1 : 2;
                        n_blk += nl;
                        n_pl += nl;
                        if (x1 == x0 && p1 > p0) {
                            n_steps += 3;
                            b = X.PC3[t] + p0;
                            e = X.PC3[t] + p1 - 1;
                            d += 2;
                            continue;
                        }
                        tri_from = d + 3;
                    }
                }
                // two characters from one rank entry per interval end, when no row of [b, e]
                // holds '#' or (c, '#') and the pattern survives both; else one step
                if (X.rent2 && !pair_skip && d + 1 < L && c != 0) {
                    const uint32_t c2 = code_at(d + 1);
                    if (c2 != 0 && c2 < X.sigma) {
                        const uint32_t p = 1 + (c - 1) * X.sigma + c2;
                        const uint4 v0 = X.rent2[(size_t)(b >> 5) * X.r2stride + p - 1];
                        const uint4 v1 = X.rent2[(size_t)((e + 1) >> 5) * X.r2stride + p - 1];
                        uint32_t p0, x0, p1, x1;
                        rent_rank(v0, b, p0, x0);
                        rent_rank(v1, e + 1, p1, x1);
                        const uint32_t nl = (b >> 5) == ((e + 1) >> 5) ? 1 : 2;
                        n_blk += nl;
                        n_pl += nl;
                        if (x1 == x0 && p1 > p0) {
                            n_steps += 2;
                            b = X.PC[p] + p0;
                            e = X.PC[p] + p1 - 1;
                            d++;
                            continue;
                        }
                        pair_skip = true;
                    }
                } else {
                    pair_skip = false;
                }
                uint32_t h0, h1, sb, se;
                const uint32_t nl = 2 - rank2_any(X, b, e + 1, c, h0, sb, h1, se);
                n_blk += nl;
                if (X.rent1) n_pl += nl;
                if (h1 > h0) { want = 1; break; }  // '#' rows: the link needs k_deep
                n_steps++;
                if (se <= sb) { alive = false; break; }
                b = X.C[c] + sb;
                e = X.C[c] + se - 1;
            }
            if (want) {
                w = make_uint4((uint32_t)i, d, b, e);
            } else if (!posres) {
                const uint32_t o = pv ? pi : perm[i];
                const uint64_t at = abase + (uint64_t)i * K;
                if (alive) put_res(res, o, b, 1u | kResRow, e - b + 1);
                else put_res(res, o, at, 0u, 0u);
            }
        }
        const uint32_t at = wave_append(qcnt + sh * 32, want);
        if (want && at < qcap) {
            q[at] = w;
            if (pv) q2[at] = pvv;  // k_deep reads the packed start instead of perm, slen and the key chunks
        }
#ifdef EDSBWT_DEEP_CLOCKS
        uint32_t wmax = rounds;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor(wmax, o, 64));
        n_lane += rounds;
        n_wave += wmax;
#else
        (void)rounds;
#endif
    }
    __shared__ unsigned long long ssum[4];
    stat_add(ctr, ST_DF_LANE_ROUNDS, n_lane, ssum);
    stat_add(ctr, ST_DF_WAVE_ROUNDS, n_wave, ssum);
    stat_add(ctr, ST_DEEP_STEPS, n_steps, ssum);
    stat_add(ctr, ST_DEEP_BLOCKS, n_blk, ssum);
    stat_add(ctr, ST_DEEP_PAIR_LINES, n_pl, ssum);
    stat_add(ctr, ST_TEXT_CHARS, n_text, ssum);
    stat_add(ctr, ST_TEXT_ROWS, n_trow, ssum);
}

// k_deep_fast specialised to the path C3 takes: the packed direct start (pv: input index and
// <= 16 remaining symbols as 2-bit digits) with the wide k-mer table (kt1w) and no three-step
// entries.  Same walk, results, queue entries and counters as k_deep_fast there; without the
// generic key-chunk reader, list offsets and rent3 it needs fewer registers, and the walk is
// latency-bound (C3: 6 waves per SIMD instead of 5 took k_deep_fast from 1.02 to 0.92 ms).
// It writes every pattern's result (an empty list's too), so the result array needs no zeroing.
//
// FUSED (the default on that path, EDSBWT_FUSED_KEYS=0: k_keys_acgt first): the pattern keys are
// computed here from the pattern bytes (each lane's three 16-B words; C3 1.610 against 1.648 ms
// with an LDS stage per block round, profiles/r04_ab2_c3_*.json) instead of being read back from
// k_keys_acgt's kid / pv arrays — one launch and ~0.3 GB of
// C3 stream traffic less.  kid and len are still written for every pattern (k_deep and
// k_deep_wave read the queued ones'), and '#' / unexpected lengths counted into n_term for the
// deferred check.
// per-lane statistics counter that compiles away when the kernel is built without statistics
template <bool ON>
struct LaneCtr {
    uint32_t v = 0;
    __device__ __forceinline__ void operator+=(uint32_t x) {
        if constexpr (ON) v += x;
    }
    __device__ __forceinline__ void operator++(int) {
        if constexpr (ON) v++;
    }
};

// STATS = false (EDSBWT_DEEP_STATS=0): no per-lane work counters (steps, lines, text rows) — five
// registers fewer in a kernel whose time follows its register pressure
template <int MINW, bool FUSED = false, bool STATS = true, bool BACK = true>
__global__ void __launch_bounds__(256, MINW) k_deep_direct(uint64_t P, uint32_t D0, const uint32_t* __restrict__ nid, KIdx X, uint64_t abase,
                                                           uint32_t K, Res* __restrict__ res, uint4* __restrict__ q, uint32_t qcap,
                                                           uint32_t* __restrict__ qcnt, unsigned long long* __restrict__ ctr,
                                                           const uint64_t* __restrict__ pv, uint32_t* __restrict__ perm_out,
                                                           const uint4* __restrict__ kt1w, uint64_t* __restrict__ q2,
                                                           const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                                                           uint32_t* __restrict__ len_out, uint32_t* __restrict__ kid_out,
                                                           unsigned long long* __restrict__ n_term, uint32_t E, uint32_t lmin, uint32_t lmax,
                                                           uint32_t* __restrict__ counts, uint32_t i0) {
    // patterns [i0, P) (i0 > 0: one piece of the batch, engine.hip run_deep_pieces)
    LaneCtr<STATS> n_steps, n_blk, n_pl, n_text, n_trow;  // per lane: < 2^32 (widened at the end)
    CountSums cs;  // counts != nullptr: each final count written here (fused counts)
#ifdef EDSBWT_DEEP_CLOCKS
    uint32_t c_srow = 0, c_seg = 0, c_wrow = 0, c_one = 0;
#endif
    uint32_t nt = 0;  // patterns holding '#' or of unexpected lengths (per lane)
    const uint32_t sh = blockIdx.x % NSHARD;
    q += (size_t)sh * qcap;
    q2 += (size_t)sh * qcap;
    // 32-bit pattern indices (the engine keeps a search's batch below 2^31 patterns): fewer registers
    // and no 64-bit index arithmetic in a kernel whose time follows its register pressure
    const uint32_t P32 = (uint32_t)P, stride32 = gridDim.x * blockDim.x;
    for (uint32_t i_b = i0 + blockIdx.x * blockDim.x; i_b < P32; i_b += stride32) {
        const uint32_t i = i_b + threadIdx.x;
        const bool valid = i < P32;
        uint32_t want = 0;
        uint4 w = make_uint4(0, 0, 0, 0);
        uint32_t pi, L, kx = 0;
        uint64_t rem;
        if constexpr (FUSED) {
            // each lane loads its own pattern's bytes: the three 16-B words from a & ~15 cover
            // L <= 32 bytes (the wave's 64 patterns are consecutive, so those loads share lines);
            // no LDS stage, no block barrier between the lanes' walks
            pi = (uint32_t)i;
            rem = 0;
            L = 0;
            if (valid) {
                const uint64_t a = off[i];
                const uint32_t Lp = (uint32_t)(off[i + 1] - a);
                bool term;
                if (Lp <= 32 && ((uintptr_t)bytes & 15) == 0) {
                    const uint4* src = reinterpret_cast<const uint4*>(bytes + (a & ~15ull));
                    const uint32_t so = (uint32_t)(a & 15), q = so >> 2, sb = so & 3;
                    const uint4 v0 = src[0], v1 = Lp + so > 16 ? src[1] : make_uint4(0, 0, 0, 0),
                                v2 = Lp + so > 32 ? src[2] : make_uint4(0, 0, 0, 0);
                    const uint32_t r[12] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, v2.x, v2.y, v2.z, v2.w};
                    uint32_t W[8];
#pragma unroll
                    for (uint32_t k = 0; k < 8; k++) {  // bytes so + 4k .. so + 4k + 3 of the window (constant indices)
                        const uint32_t x0 = q == 0 ? r[k] : q == 1 ? r[k + 1] : q == 2 ? r[k + 2] : r[k + 3];
                        const uint32_t x1 = q == 0 ? r[k + 1] : q == 1 ? r[k + 2] : q == 2 ? r[k + 3] : r[k + 4];
                        W[k] = __builtin_amdgcn_alignbyte(x1, x0, sb);
                    }
                    acgt_key_regs(W, Lp, D0, E, lmin, lmax, kx, rem, term);
                } else {
                    acgt_key(bytes, a, Lp, false, nullptr, 0u, D0, E, lmin, lmax, kx, rem, term);
                }
                nt += term;
                len_out[i] = Lp;
                kid_out[i] = kx;
                L = pk_len(D0, rem);
            }
        } else {
            const uint64_t v = valid ? pv[i] : 0ull;
            pi = (uint32_t)(v & 0x7fffffffu);
            rem = v >> 31;
            L = valid ? pk_len(D0, rem) : 0u;
        }
        if (valid) perm_out[i] = pi;
        // the D-mer's wide entry: its one interval inline (or its list's length), and for one
        // row with its text position, the row's sample and the 32 text characters before it
        uint64_t ent = 0, win1 = 0;
        uint4 s1 = make_uint4(0, 0, 0, 0);
        uint32_t u = 0;
        if (L > D0) {
            u = FUSED ? kx : nid[i];
            const uint4 w0 = kt1w[(size_t)X.kt1_ws * u];
            s1 = kt1w[(size_t)X.kt1_ws * u + 1];
            ent = (uint64_t)w0.y << 32 | w0.x;
            win1 = (uint64_t)w0.w << 32 | w0.z;
            n_blk++;  // the entry's 32 or 64 B: one line
        }
        const uint32_t n0 = L <= D0 ? 0u : (ent >> 63) ? 1u : (uint32_t)(ent >> 32);
        if (n0 > 1) {
            want = 1;
            w = make_uint4((uint32_t)i, D0, kQWide, u);
        } else if (n0 == 0) {
            if (valid) {
                put_res(res, pi, 0, 0u, 0u);  // no list: count 0 (every result is written here or by k_deep)
                cs.put(counts, pi, 0u);
            }
        } else {
            uint32_t b, e, g1 = ~0u;
            if (X.kt1_pos && ((ent >> 62) & 1)) {
                b = e = (uint32_t)ent & 0x7fffffffu;
                g1 = (uint32_t)(ent >> 31) & 0x7fffffffu;
            } else {
                b = (uint32_t)ent;
                e = (uint32_t)(ent >> 32) & 0x7fffffffu;
            }
            auto code_at = [&](uint32_t dd) -> uint32_t { return 1u + (uint32_t)((rem >> (2 * (dd - D0))) & 3u); };
            bool alive = true, pair_skip = false, posres = false;
            uint32_t d = D0;
            if (g1 != ~0u) DD_CNT(c_one);
            // the row's sample and text window: the wide entry's for the first row (have), loaded
            // for rows reached through a link
            uint4 s = s1;
            uint64_t tw = win1;
            bool have = g1 != ~0u;
            bool ent_row = have && X.kt1_ws == 4;  // s is the entry's row: its link ranks are in the entry
            // the text compare while the interval is one row, rank steps while it holds several, and
            // back to the text compare when a rank step leaves one row (BACK; EDSBWT_DIRECT_BACK=0:
            // rank steps to the end once the interval was wide) — a row's text-compare line replaces a
            // rank-entry line per two characters
            for (;;) {
            while (X.rtext && b == e && d < L) {
                // one row = one text position: the next k = min(o, m) <= 16 characters against the
                // text (MOVE_EDSBWTSearch.cpp:424-510 stepping one row), as in k_deep_fast
                uint32_t g = 0;
                if (!have && X.srow) {  // the row's sample, text position and window in one line
                    s = X.srow[2 * (size_t)b];
                    const uint4 t2 = X.srow[2 * (size_t)b + 1];
                    tw = (uint64_t)t2.w << 32 | t2.z;
                    have = true;
                    n_blk += 1;
                    DD_CNT(c_srow);
                } else if (!have) {
                    s = X.samples[b];
                    g = X.gpos[b];
                    n_blk += 3;
                }  // (else the wide entry's, counted with it)
                n_trow++;
                const uint32_t m = L - d, k = min(s.y, m);
                if (k) {
                    const uint64_t mask = (1ull << (2 * k)) - 1ull;
                    if (!have) tw = rtext_window(X.rtext, X.tlen - g);
                    if (((tw ^ (rem >> (2 * (d - D0)))) & mask) != 0) {
                        alive = false;
                        d = L;
                        break;
                    }
                }
                have = false;
                if (s.y >= m) {
                    if (s.w <= kResCnt) {  // else (a segment of 2^30 words) the walk below decides
                        posres = true;
                        n_text += m;
                        d = L;
                        put_res(res, pi, (uint64_t)(s.y - m) << 32 | s.x, kResRow | kResPos | s.w, s.z);
                        cs.put(counts, pi, 1u);
                    }
                    break;
                }
                // the word matched to its start: the link from its '#' row, one segment (:512-563)
                n_text += s.y;
                d += s.y;
                const uint32_t c = code_at(d);
                if (c >= X.sigma) {
                    b = e = X.wrow[s.x];
                    n_blk++;
                    DD_CNT(c_wrow);
                    break;
                }
                if (s.z < 2) {
                    alive = false;
                    d = L;
                    break;
                }
                uint32_t rx, ry;
                if (ent_row) {  // (the entry's 128-B line, already fetched)
                    const uint32_t* lk = reinterpret_cast<const uint32_t*>(kt1w + 4 * (size_t)u + 2);
                    rx = lk[c - 1];
                    ry = lk[4 + c - 1];
                } else if (X.seglink) {  // the ranks and, for one row, its text-compare entry: one line
                    const uint4* sl = X.seglink + 8 * (size_t)s.z + 2 * (c - 1);
                    const uint4 l0 = sl[0], l1 = sl[1];
                    rx = l0.x;
                    ry = l0.y;
                    if (ry == rx + 1) {
                        s = make_uint4(l0.z, l0.w, l1.x, l1.y);
                        tw = (uint64_t)l1.w << 32 | l1.z;
                        have = true;
                    }
                    n_blk++;
                    DD_CNT(c_seg);
                } else {
                    const uint32_t* et = X.segtab + (size_t)s.z * X.seg_stride;
                    rx = et[1 + c];
                    ry = et[X.seg_hi + c];
                    n_blk++;
                    DD_CNT(c_seg);
                }
                ent_row = false;
                n_steps++;
                if (ry <= rx) {
                    alive = false;
                    d = L;
                    break;
                }
                b = X.C[c] + rx;
                e = X.C[c] + ry - 1;
                d++;
            }
            bool back = false;
            for (; d < L; d++) {
                const uint32_t c = code_at(d);
                if (c >= X.sigma) { alive = false; break; }
                // two characters from one rank entry per interval end (rent2), else one step
                if (X.rent2 && !pair_skip && d + 1 < L) {
                    const uint32_t c2 = code_at(d + 1);
                    if (c2 < X.sigma) {
                        const uint32_t p = 1 + (c - 1) * X.sigma + c2;
                        const uint4 v0 = X.rent2[(size_t)(b >> 5) * X.r2stride + p - 1];
                        const uint4 v1 = X.rent2[(size_t)((e + 1) >> 5) * X.r2stride + p - 1];
                        uint32_t p0, x0, p1, x1;
                        rent_rank(v0, b, p0, x0);
                        rent_rank(v1, e + 1, p1, x1);
                        const uint32_t nl = (b >> 5) == ((e + 1) >> 5) ? 1 : 2;
                        n_blk += nl;
                        n_pl += nl;
                        if (x1 == x0 && p1 > p0) {
                            n_steps += 2;
                            b = X.PC[p] + p0;
                            e = X.PC[p] + p1 - 1;
                            d++;
                            if (BACK && b == e && X.rtext) { d++; back = true; break; }
                            continue;
                        }
                        pair_skip = true;
                    }
                } else {
                    pair_skip = false;
                }
                uint32_t h0, h1, sb, se;
                const uint32_t nl = 2 - rank2_any(X, b, e + 1, c, h0, sb, h1, se);
                n_blk += nl;
                if (X.rent1) n_pl += nl;
                if (h1 > h0) { want = 1; break; }  // '#' rows: the link needs k_deep
                n_steps++;
                if (se <= sb) { alive = false; break; }
                b = X.C[c] + sb;
                e = X.C[c] + se - 1;
                if (BACK && b == e && X.rtext) { d++; back = true; break; }
            }
            if (!back) break;
            }
            if (want) {
                w = make_uint4((uint32_t)i, d, b, e);
            } else if (!posres) {
                if (alive) put_res(res, pi, b, 1u | kResRow, e - b + 1);
                else put_res(res, pi, abase + (uint64_t)i * K, 0u, 0u);
                cs.put(counts, pi, alive ? e - b + 1 : 0u);
            }
        }
        if (want) put_res(res, pi, 0, 0u, 0u);  // the zeroed result the later walks expect
        const uint32_t at = wave_append(qcnt + sh * 32, want);
        if (want && at < qcap) {
            q[at] = w;
            q2[at] = rem << 31 | pi;  // the packed start: k_deep reads it instead of perm, slen and the key chunks
        }
    }
    __shared__ unsigned long long ssum[4];
    stat_add(ctr, ST_DEEP_STEPS, n_steps.v, ssum);
    stat_add(ctr, ST_DEEP_BLOCKS, n_blk.v, ssum);
    stat_add(ctr, ST_DEEP_PAIR_LINES, n_pl.v, ssum);
    stat_add(ctr, ST_TEXT_CHARS, n_text.v, ssum);
    stat_add(ctr, ST_TEXT_ROWS, n_trow.v, ssum);
    cs.flush(counts, ctr, ssum);
#ifdef EDSBWT_DEEP_CLOCKS
    stat_add(ctr, ST_CLK_DD_SROW, c_srow, ssum);
    stat_add(ctr, ST_CLK_DD_SEG, c_seg, ssum);
    stat_add(ctr, ST_CLK_DD_WROW, c_wrow, ssum);
    stat_add(ctr, ST_CLK_DD_ONE, c_one, ssum);
#endif
    if constexpr (FUSED) {
        const unsigned long long ntb = block_sum((unsigned long long)nt, ssum);
        if (threadIdx.x == 0 && ntb) atomicAdd(n_term, ntb);
    }
}

// rank of `lane` among the set lanes of mask m
__device__ __forceinline__ uint32_t lane_rank(uint64_t m, uint32_t lane) { return (uint32_t)__popcll(m & ((1ull << lane) - 1ull)); }

// shard prefix sums of k_deep_fast's queue counters (one block)
__global__ void k_queue_prefix(const uint32_t* __restrict__ qcnt, uint32_t* __restrict__ qpre) {
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (uint32_t t = 0; t < NSHARD; t++) { qpre[t] = s; s += qcnt[t * 32]; }
        qpre[NSHARD] = s;
    }
}

#ifdef EDSBWT_KDEEP_DUMP
constexpr uint32_t kDumpMax = 64;
__device__ uint32_t g_kdeep_dump[kDumpMax * 16];
#endif
// EOFROW: links from '#' rows through KIdx::eofrow (one line per row; costs k_deep 6 VGPRs and a
// wave per SIMD: C3 0.355 against 0.304 ms, profiles/r04_ab_c3_*.json — off by default)
// PACKED: the packed direct start's queue only (q2 != nullptr: each entry's pattern index and remaining
// symbols travel in q2) — the key-chunk reader and the perm / slen reads are compiled out
template <int K, int BPS, int MINW = 1, bool EOFROW = false, bool STATS = true, bool PACKED = false>  // MINW: waves per SIMD the register budget is held to (1: no bound)
__global__ void __launch_bounds__(256, MINW) k_deep(const uint4* __restrict__ q, const uint32_t* __restrict__ qcnt, uint32_t qcap, uint32_t D0,
                                              const uint32_t* __restrict__ slen, const uint32_t* __restrict__ perm,
                                              const uint64_t* __restrict__ k0, const uint64_t* __restrict__ krest, uint32_t ind, uint64_t P,
                                              const uint32_t* __restrict__ nid, const uint32_t* __restrict__ ioff,
                                              const uint32_t* __restrict__ iend, const uint32_t* __restrict__ ib,
                                              const uint32_t* __restrict__ ie, KIdx X, uint64_t abase,
                                              uint32_t* __restrict__ ab, uint32_t* __restrict__ ae, Res* __restrict__ res,
                                              uint32_t* __restrict__ ovf, unsigned long long* __restrict__ ctr, const uint64_t* __restrict__ q2,
                                              const uint4* __restrict__ kt1w, uint32_t* __restrict__ counts, uint32_t qpairs) {
    LaneCtr<STATS> n_steps, n_hash, n_blk, n_text, n_trow, n_q;  // (STATS = false: compiled away)
    CountSums cs;  // n_blk: occ blocks read (per lane, widened at the end)
#ifdef EDSBWT_DEBUG_CHECKS
    uint32_t dbg_q = 0, dbg_p = 0, dbg_w = 0, dbg_l = 0;
#endif
#ifdef EDSBWT_DEEP_CLOCKS
    unsigned long long c_rank = 0, c_runs = 0, c_rest = 0, c_steps = 0, c_hsteps = 0;
#endif
    // the shards' prefix sums of the producers' queue counters (qcnt[s * 32]), by the block's first
    // wave (no k_queue_prefix launch)
    __shared__ uint32_t spre[NSHARD + 1];
    if (threadIdx.x < 64) {
        const uint32_t lane = threadIdx.x;
        uint32_t carry = 0;
        for (uint32_t b0 = 0; b0 < NSHARD; b0 += 64) {
            const uint32_t t = b0 + lane;
            const uint32_t v = t < NSHARD ? qcnt[t * 32] : 0u;
            uint32_t inc = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(inc, (unsigned)o, 64);
                if (lane >= (uint32_t)o) inc += y;
            }
            if (t < NSHARD) spre[t] = carry + inc - v;
            carry += __shfl(inc, 63, 64);
        }
        if (lane == 0) spre[NSHARD] = carry;
    }
    __syncthreads();
    const uint32_t total = spre[NSHARD];
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < total; j += gridDim.x * blockDim.x) {  // (32-bit: fewer registers)
        uint32_t lo = 0, hi = NSHARD;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (spre[mid] <= (uint32_t)j) lo = mid; else hi = mid;
        }
        const size_t qi = (size_t)lo * qcap + ((uint32_t)j - spre[lo]);
        DBG_CHECK((uint32_t)j - spre[lo] < qcap, dbg_q);  // a slot its producer wrote
        const uint4 w = q[qi];
        const uint32_t i = w.x, d0 = w.y;
        DBG_CHECK(i < P && d0 >= D0, dbg_q);
        n_q++;
        // q2 (packed direct start): input index and remaining symbols from the queue entry
        uint32_t pi, L;
        uint64_t rem = 0;
        if (PACKED || q2) {
            const uint64_t v = q2[qi];
            pi = (uint32_t)(v & 0x7fffffffu);
            rem = v >> 31;
            DBG_CHECK(rem != 0 && pi < P, dbg_p);
            L = pk_len(D0, rem);
            DBG_CHECK(L <= D0 + 16 && d0 <= L, dbg_p);
        } else {
            pi = ind ? perm[i] : i;  // slen and key chunks in input order (k_deep_fast)
            L = slen[pi];
        }
        // the entry as one interval [w.z, w.w], assigned BEFORE the branch on the entry's kind: the
        // list arms below only override it, and the interval case writes nothing at the join.  (Round
        // 6, DESIGN.md §0: with the interval's values assigned in its own arm of a three-way branch,
        // this compiler lowered the kind test to a signed range split and wrote those values only on
        // the w.z <= -2 side, so a row entry — w.z < 2^31 — started from stale registers: the round-4
        // miscount and round-5 fault of the unbounded build, profiles/r06_isa_kdeep431_threeway_*.txt)
        uint32_t cb[K], ce[K];
        uint32_t cn = 1;
#pragma unroll
        for (int t = 0; t < K; t++) cb[t] = ce[t] = 0;
        cb[0] = w.z;
        ce[0] = w.w;
#ifdef EDSBWT_KDEEP_DUMP
        uint32_t dump_u = 0xFFFFFFFFu;
#endif
        // a list start (kQWide / kQNode) or the interval above: the only divergent branch on the
        // entry's kind; wide or node list is the uniform kt1w (a kernel argument).
        // EDSBWT_KDEEP_THREEWAY compiles round 5's three-way shape for the test-only libedsbwt_3way.so
#ifdef EDSBWT_KDEEP_THREEWAY
        if (w.z == kQWide) {  // (acac474: the table's presence checked inside the arm)
            if (!kt1w) { flag_push(ovf, (uint32_t)i); continue; }
#else
        if (w.z >= kQWide && kt1w) {
#endif
            // the list's length, offset and (<= 3 intervals) the intervals themselves from the
            // D-mer's 32-B wide entry, w.w = the D-mer (k_ktab_wide) — one line instead of the nid,
            // ioff / iend, ib and ie reads below.  Producers given the wide table write kQWide;
            // another kind, or a D-mer past the table, goes to the wide-list walk (node lists)
            DBG_CHECK(w.z == kQWide && w.w <= X.kt_E, dbg_w);
            if (w.z != kQWide || w.w > X.kt_E) { flag_push(ovf, (uint32_t)i); continue; }
            const uint4 a0 = kt1w[(size_t)X.kt1_ws * w.w], a1 = kt1w[(size_t)X.kt1_ws * w.w + 1];
            n_blk++;
            cn = a0.y;
            // a queued D-mer has a list of >= 2 intervals (one interval is never queued from the
            // start), held in ktab_b / ktab_e at a0.x
            DBG_CHECK(cn >= 2 && (uint64_t)a0.x + cn <= X.kt_n, dbg_w);
            if (cn > K || (cn > kWideInline && (uint64_t)a0.x + cn > X.kt_n)) { flag_push(ovf, (uint32_t)i); continue; }
            const bool inl = cn <= kWideInline;
            if (!inl) n_blk += 2;
            const uint32_t lb[kWideInline] = {a0.z, a1.x, a1.z}, le[kWideInline] = {a0.w, a1.y, a1.w};
#pragma unroll
            for (int t = 0; t < K; t++) {
                const bool on = (uint32_t)t < cn;
                cb[t] = !on ? 0u : inl && t < kWideInline ? lb[t < kWideInline ? t : 0] : ib[a0.x + t];
                ce[t] = !on ? 0u : inl && t < kWideInline ? le[t < kWideInline ? t : 0] : ie[a0.x + t];
            }
#ifdef EDSBWT_KDEEP_THREEWAY
        } else if (w.z == kQNode) {  // (acac474's second divergent arm)
#else
        } else if (w.z >= kQWide) {  // from the node's items at the cutover depth
#endif
            DBG_CHECK(w.z == kQNode, dbg_q);
            const uint32_t u = nid[i];
#ifdef EDSBWT_KDEEP_DUMP
            dump_u = u;
#endif
            cn = iend[u] - ioff[u];
            n_blk += 4;  // nid, ioff / iend, and the list's lines in ib and ie
            if (cn > K) { flag_push(ovf, (uint32_t)i); continue; }
#pragma unroll
            for (int t = 0; t < K; t++) {
                cb[t] = (uint32_t)t < cn ? ib[ioff[u] + t] : 0u;
                ce[t] = (uint32_t)t < cn ? ie[ioff[u] + t] : 0u;
            }
        }
#ifdef EDSBWT_DEBUG_CHECKS
        for (int t = 0; t < K; t++)
            if ((uint32_t)t < cn && !(cb[t] <= ce[t] && ce[t] < X.N)) dbg_l++;
#endif
#ifdef EDSBWT_KDEEP_DUMP
        // (diagnostic builds: the first kDumpMax queue entries' list starts, read back by
        // edsbwt_debug_kdeep_dump — DESIGN.md §0, the three-way list start)
        if (j < kDumpMax) {
            uint32_t* dd = g_kdeep_dump + (size_t)j * 16;
            dd[0] = w.x; dd[1] = w.y; dd[2] = w.z; dd[3] = w.w; dd[4] = cn; dd[5] = dump_u;
#pragma unroll
            for (int t = 0; t < 4; t++) {
                dd[6 + t] = t < K ? cb[t < K ? t : 0] : 0u;
                dd[10 + t] = t < K ? ce[t < K ? t : 0] : 0u;
            }
            dd[14] = pi; dd[15] = 0xD0D0D0D0u;
        }
#endif
        if (PACKED && X.deep_filter && X.srow && X.rtext && X.text_deep && cn > 1 && d0 < L) {
            // a list start of single rows (a D-mer that occurs a few times): each row's text compared
            // up to its word start, the lines issued together; the rows that mismatch leave the list
            // before the first step (they would die in it), so a planted pattern usually goes on
            // with one row — the text compare below — instead of stepping every row
            const uint32_t m = L - d0;
            const uint64_t want = rem >> (2 * (d0 - D0));
            bool ok[K];
#pragma unroll
            for (int t = 0; t < K; t++) {
                ok[t] = (uint32_t)t < cn;
                if ((uint32_t)t < cn && cb[t] == ce[t]) {
                    const uint4 s0 = X.srow[2 * (size_t)cb[t]];
                    const uint4 t2 = X.srow[2 * (size_t)cb[t] + 1];
                    const uint32_t k = min(s0.y, m);  // (<= 16: the packed start's patterns)
                    const uint64_t mask = (1ull << (2 * k)) - 1ull;
                    ok[t] = ((((uint64_t)t2.w << 32 | t2.z) ^ want) & mask) == 0;
                    n_blk++;
                }
            }
            uint32_t keep = 0;
#pragma unroll
            for (int t = 0; t < K; t++) {
                if (ok[t]) {
#pragma unroll
                    for (int v = 0; v <= t; v++)
                        if ((uint32_t)v == keep) { cb[v] = cb[t]; ce[v] = ce[t]; }
                    keep++;
                }
            }
            cn = keep;
        }
        SymReader<BPS> sym{k0, krest, P, pi};
        auto code_at = [&](uint32_t dd) -> uint32_t { return (PACKED || q2) ? 1u + (uint32_t)((rem >> (2 * (dd - D0))) & 3u) : sym.code(dd); };
        bool over = false, posres = false, pskip = false;
        for (uint32_t d = d0; d < L && cn; d++) {
            DEEP_CLK(t0);
            if (X.rtext && X.text_deep && cn == 1 && cb[0] == ce[0]) {
                // a single row: compare with the text as k_deep_fast does
                const uint32_t x0 = cb[0];
                uint4 s;
                uint32_t g;
                uint64_t w0 = 0;
                if (X.srow) {  // sample, text position and window in one line
                    s = X.srow[2 * (size_t)x0];
                    const uint4 t2 = X.srow[2 * (size_t)x0 + 1];
                    g = t2.x;
                    w0 = (uint64_t)t2.w << 32 | t2.z;
                    n_blk += 1;
                } else {
                    s = X.samples[x0];
                    g = X.gpos[x0];
                    n_blk += 3;
                }
                n_trow++;
                const uint32_t m = L - d, k = min(s.y, m);
                bool eq = true, valid_codes = true;
                const uint64_t r0 = X.tlen - g;
                for (uint32_t j = 0; j < k && eq && valid_codes; j += 32) {
                    const uint32_t n = min(32u, k - j);
                    const uint64_t mask = n == 32 ? ~0ull : ((1ull << (2 * n)) - 1ull);
                    uint64_t want = 0;
                    for (uint32_t t = 0; t < n; t++) {
                        const uint32_t c = code_at(d + j + t);
                        if (c == 0) { valid_codes = false; break; }
                        if (c >= X.sigma) { eq = false; break; }
                        want |= (uint64_t)(c - 1) << (2 * t);
                    }
                    if (valid_codes && eq) eq = (((X.srow && j == 0 ? w0 : rtext_window(X.rtext, r0 + j)) ^ want) & mask) == 0;
                }
                if (valid_codes) {
                    if (!eq) { cn = 0; break; }
                    if (s.y >= m) {
                        if (s.w <= kResCnt) {  // else (a segment of 2^30 words) the walk below decides
                            n_text += m;
                            posres = true;
                            put_res(res, (PACKED || q2) ? pi : perm[i], (uint64_t)(s.y - m) << 32 | s.x, kResRow | kResPos | s.w, s.z);
                            cs.put(counts, (PACKED || q2) ? pi : perm[i], 1u);
                            break;
                        }
                    } else {
                        n_text += s.y;
                        d += s.y;
                        // the whole word matched: the link from its one segment, as in k_deep_fast
                        const uint32_t c = code_at(d);
                        if (c != 0 && c < X.sigma) {
                            if (s.z < 2) { cn = 0; break; }
                            const uint32_t* et = X.segtab + (size_t)s.z * X.seg_stride;
                            const uint32_t rx = et[1 + c], ry = et[X.seg_hi + c];
                            n_blk++;
                            n_steps++;
                            if (ry <= rx) { cn = 0; break; }
                            cb[0] = X.C[c] + rx;
                            ce[0] = X.C[c] + ry - 1;
                            continue;  // the loop's d++ consumes c
                        }
                        cb[0] = ce[0] = X.wrow[s.x];
                        n_blk++;
                    }
                }
            }
            const uint32_t code = code_at(d);
            if (code >= X.sigma) { cn = 0; break; }
            const uint32_t c = code;
            // two characters at once (qpairs, rent2): one pair entry per interval end gives the rank
            // of (c, c2) and of the rows coded '#' or (c, '#'); when no interval holds such a row,
            // neither step links (MOVE_EDSBWTSearch.cpp:512-563 is not reached) and every interval
            // maps to [PC[p] + rank_p(b), PC[p] + rank_p(e + 1)) — DESIGN.md §3.  Else (or after a
            // failed try: pskip) one step as below.  The list order is kept, so merges are the same.
            // c = '#' (code 0: a pattern holding '#' on the ordered path) has no pair code — p would
            // wrap below 1 — so it always takes the single step, as in k_deep_fast
            if (qpairs && X.rent2 && !pskip && d + 1 < L && c != 0) {
                const uint32_t c2 = code_at(d + 1);
                if (c2 != 0 && c2 < X.sigma) {
                    const uint32_t p = 1 + (c - 1) * X.sigma + c2;
                    uint32_t pb[K], pe[K];
                    bool clean = true;
#pragma unroll
                    for (int j = 0; j < K; j++) {
                        pb[j] = pe[j] = 0;
                        if ((uint32_t)j < cn) {
                            const uint32_t x0r = cb[j], x1r = ce[j] + 1;
                            const uint4 v0 = X.rent2[(size_t)(x0r >> 5) * X.r2stride + p - 1];
                            const uint4 v1 = X.rent2[(size_t)(x1r >> 5) * X.r2stride + p - 1];
                            uint32_t h0, h1;
                            rent_rank(v0, x0r, pb[j], h0);
                            rent_rank(v1, x1r, pe[j], h1);
                            n_blk += (x0r >> 5) == (x1r >> 5) ? 1 : 2;
                            clean = clean && h0 == h1;
                        }
                    }
                    if (clean) {
                        uint32_t nn = 0, last_e = 0;
                        uint32_t nb[K], ne[K];
#pragma unroll
                        for (int t = 0; t < K; t++) nb[t] = ne[t] = 0;
#pragma unroll
                        for (int j = 0; j < K; j++) {
                            if ((uint32_t)j < cn && pe[j] > pb[j]) {
                                const uint32_t b2 = X.PC[p] + pb[j], e2 = X.PC[p] + pe[j] - 1;
                                if (nn && b2 == last_e + 1) {
#pragma unroll
                                    for (int t = 0; t < K; t++)
                                        if ((uint32_t)t + 1 == nn) ne[t] = e2;
                                } else {
#pragma unroll
                                    for (int t = 0; t < K; t++)
                                        if ((uint32_t)t == nn) { nb[t] = b2; ne[t] = e2; }
                                    nn++;
                                }
                                last_e = e2;
                            }
                        }
                        n_steps += 2 * cn;
                        cn = nn;
#pragma unroll
                        for (int t = 0; t < K; t++) { cb[t] = nb[t]; ce[t] = ne[t]; }
                        d++;  // (and the loop's d++: both characters consumed)
                        continue;
                    }
                    pskip = true;
                }
            } else {
                pskip = false;
            }
            // ranks at both ends of every current interval: '#'-rows (link) and c (step)
            uint32_t sb[K], se[K], raw[K], rawk[EOFROW ? K : 1];  // rawk: a '#'-rank of raw's segment (its eofrow line)
            uint32_t rn = 0;
#pragma unroll
            for (int j = 0; j < K; j++) {
                sb[j] = se[j] = 0;
                raw[j] = 0;
                if constexpr (EOFROW) rawk[j] = 0;
            }
#pragma unroll
            for (int j = 0; j < K; j++) {
                if ((uint32_t)j < cn) {
                    uint32_t h0, h1;
                    n_blk += 2 - rank2_any(X, cb[j], ce[j] + 1, c, h0, sb[j], h1, se[j]);
                    n_hash += h1 - h0;
                    for (uint32_t k = h0; k < h1; k++) {  // dollars_in_interval (:607-625)
                        // the word's segment: from its link row (one line, the ranks come with it) or eof_seg
                        const uint32_t s = EOFROW ? X.eofrow[(size_t)k * 16 + 15] : X.eof_seg[k];
                        if (!s) continue;
                        // insert s into raw[0..rn) ascending, dropping duplicates
                        bool dup = false;
#pragma unroll
                        for (int t = 0; t < K; t++)
                            if ((uint32_t)t < rn && raw[t] == s) dup = true;
                        if (dup) continue;
                        if (rn == K) { over = true; break; }
                        uint32_t vv = s, vk = k;
#pragma unroll
                        for (int t = 0; t < K; t++) {
                            if ((uint32_t)t < rn) {
                                if (raw[t] > vv) {
                                    const uint32_t tmp = raw[t];
                                    raw[t] = vv;
                                    vv = tmp;
                                    if constexpr (EOFROW) {
                                        const uint32_t tk = rawk[t];
                                        rawk[t] = vk;
                                        vk = tk;
                                    }
                                }
                            } else if ((uint32_t)t == rn) {
                                raw[t] = vv;
                                if constexpr (EOFROW) rawk[t] = vk;
                            }
                        }
                        rn++;
                    }
                }
            }
            if (over) break;
            DEEP_CLK(t1);
            // step: [dollar runs (ascending), own intervals] by c, adjacent merged (:275-324)
            uint32_t nb[K], ne[K];
            uint32_t nn = 0, last_e = 0;
#pragma unroll
            for (int t = 0; t < K; t++) nb[t] = ne[t] = 0;
            auto push = [&](uint32_t b, uint32_t e) {
                if (nn && b == last_e + 1) {
#pragma unroll
                    for (int t = 0; t < K; t++)
                        if ((uint32_t)t + 1 == nn) ne[t] = e;
                    last_e = e;
                    return;
                }
                if (nn == K) { over = true; return; }
#pragma unroll
                for (int t = 0; t < K; t++)
                    if ((uint32_t)t == nn) { nb[t] = b; ne[t] = e; }
                nn++;
                last_e = e;
            };
            // a run [seg_lo[s_first], s_last - 1] of previous-segment words, stepped by c:
            // its c-ranks come precomputed from the segment table (one line per segment)
            uint32_t run_x = 0, run_y = 0, run_s = 0;
            bool have = false;
            auto close_run = [&]() {
                if (run_y > run_x) push(X.C[c] + run_x, X.C[c] + run_y - 1);
                n_steps++;
            };
#pragma unroll
            for (int t = 0; t < K; t++) {
                if ((uint32_t)t < rn) {
                    const uint32_t s = raw[t];
                    // the '#' row's link row was just read (a cache hit); else the segment's table row
                    const uint32_t* e = EOFROW ? X.eofrow + (size_t)rawk[EOFROW ? t : 0] * 16 : X.segtab + (size_t)s * X.seg_stride;
                    const uint32_t lo = e[0];
                    if (!EOFROW) n_blk++;
                    if (have && lo > run_s) { close_run(); have = false; }
                    if (!have) { run_x = e[1 + c]; have = true; }
                    run_y = e[X.seg_hi + c];
                    run_s = s;
                }
            }
            if (have) close_run();
            DEEP_CLK(t2);
#pragma unroll
            for (int j = 0; j < K; j++)
                if ((uint32_t)j < cn && se[j] > sb[j]) push(X.C[c] + sb[j], X.C[c] + se[j] - 1);
            n_steps += cn;
            if (over) break;
            cn = nn;
#pragma unroll
            for (int t = 0; t < K; t++) { cb[t] = nb[t]; ce[t] = ne[t]; }
            DEEP_CLK(t3);
            DEEP_CLK_ADD(c_rank, t1 - t0);
            DEEP_CLK_ADD(c_runs, t2 - t1);
            DEEP_CLK_ADD(c_rest, t3 - t2);
            DEEP_CLK_ADD(c_steps, 1);
            DEEP_CLK_ADD(c_hsteps, rn ? 1 : 0);
        }
        if (over) { flag_push(ovf, (uint32_t)i); continue; }
        if (posres) continue;
        // ascending rows (the input lists may be unordered sets)
#pragma unroll
        for (int a = 0; a < K; a++)
#pragma unroll
            for (int b2 = 0; b2 + 1 < K - a; b2++)
                if ((uint32_t)(b2 + 1) < cn && cb[b2] > cb[b2 + 1]) {
                    uint32_t t0 = cb[b2]; cb[b2] = cb[b2 + 1]; cb[b2 + 1] = t0;
                    t0 = ce[b2]; ce[b2] = ce[b2 + 1]; ce[b2 + 1] = t0;
                }
        const uint32_t o = (PACKED || q2) ? pi : perm[i];
        uint32_t occ = 0;
        const uint64_t at = abase + (uint64_t)i * K;
        if (cn == 1) {
            put_res(res, o, cb[0], 1u | kResRow, ce[0] - cb[0] + 1);
            cs.put(counts, o, ce[0] - cb[0] + 1);
            continue;
        }
#pragma unroll
        for (int t = 0; t < K; t++)
            if ((uint32_t)t < cn) {
                ab[at + t] = cb[t];
                ae[at + t] = ce[t];
                occ += ce[t] - cb[t] + 1;
            }
        put_res(res, o, at, cn, occ);
        cs.put(counts, o, occ);
    }
    __shared__ unsigned long long sh[4];
    stat_add(ctr, ST_DEEPQ_STEPS, n_steps.v, sh);
    stat_add(ctr, ST_DEEP_HASH, n_hash.v, sh);
    stat_add(ctr, ST_DEEPQ_BLOCKS, n_blk.v, sh);
    stat_add(ctr, ST_DEEPQ_PATS, n_q.v, sh);
    stat_add(ctr, ST_TEXT_CHARS, n_text.v, sh);
    stat_add(ctr, ST_TEXT_ROWS, n_trow.v, sh);
    cs.flush(counts, ctr, sh);
#ifdef EDSBWT_DEBUG_CHECKS
    stat_add(ctr, ST_DBG_QUEUE, dbg_q, sh);
    stat_add(ctr, ST_DBG_PACKED, dbg_p, sh);
    stat_add(ctr, ST_DBG_WIDE, dbg_w, sh);
    stat_add(ctr, ST_DBG_LIST, dbg_l, sh);
#endif
#ifdef EDSBWT_DEEP_CLOCKS
    stat_add(ctr, ST_CLK_RANK, c_rank, sh);
    stat_add(ctr, ST_CLK_RUNS, c_runs, sh);
    stat_add(ctr, ST_CLK_REST, c_rest, sh);
    stat_add(ctr, ST_CLK_STEPS, c_steps, sh);
    stat_add(ctr, ST_CLK_HASH_STEPS, c_hsteps, sh);
#endif
}

// Patterns k_deep<8> could not hold: the same walk with lists of up to KW intervals
// in private (scratch) arrays, one thread per flagged pattern.  Rare, so plain loops.
template <int KW>
__global__ void __launch_bounds__(256) k_deep_wide(uint64_t P, uint32_t D0, const uint32_t* __restrict__ todo, uint32_t ntodo,
                                                  const uint32_t* __restrict__ slen, const uint32_t* __restrict__ perm, uint32_t ind,
                                                  const uint64_t* __restrict__ off, const uint8_t* __restrict__ bytes,
                                                  const uint8_t* __restrict__ code_of, const uint32_t* __restrict__ nid,
                                                  const uint32_t* __restrict__ ioff, const uint32_t* __restrict__ iend,
                                                  const uint32_t* __restrict__ ib, const uint32_t* __restrict__ ie, KIdx X, uint64_t abase,
                                                  uint32_t* __restrict__ ab, uint32_t* __restrict__ ae, Res* __restrict__ res,
                                                  uint32_t* __restrict__ ovf2, const uint32_t* __restrict__ ntodo_dev) {
    (void)P;
    // ntodo_dev (deferred checks): the list's length lives on the device; ntodo is the grid's
    // capacity, and a longer list is caught by the caller's final check
    if (ntodo_dev) ntodo = min(ntodo, *ntodo_dev);
    GRID_STRIDE(j, ntodo) {
        const uint32_t i = todo[j];
        const uint32_t L = slen[ind ? perm[i] : i];
        const uint32_t u = nid[i];
        const uint32_t n0 = iend[u] - ioff[u];
        if (n0 > KW) { flag_push(ovf2, i); continue; }
        uint32_t cb[KW], ce[KW], nb[KW], ne[KW], sb[KW], se[KW], raw[KW];
        uint32_t cn = n0;
        for (uint32_t t = 0; t < cn; t++) { cb[t] = ib[ioff[u] + t]; ce[t] = ie[ioff[u] + t]; }
        const uint32_t a = perm[i];
        const uint8_t* pat = bytes + off[a];
        bool over = false;
        for (uint32_t d = D0; d < L && cn && !over; d++) {
            const uint32_t code = code_of[pat[L - 1 - d]];
            if (code >= X.sigma) { cn = 0; break; }
            const uint32_t c = code;
            uint32_t rn = 0;
            for (uint32_t q = 0; q < cn && !over; q++) {
                uint32_t h0, h1;
                rank2_any(X, cb[q], ce[q] + 1, c, h0, sb[q], h1, se[q]);
                for (uint32_t k = h0; k < h1; k++) {
                    const uint32_t s = X.eof_seg[k];
                    if (!s) continue;
                    uint32_t pos = 0;
                    while (pos < rn && raw[pos] < s) pos++;
                    if (pos < rn && raw[pos] == s) continue;
                    if (rn == KW) { over = true; break; }
                    for (uint32_t t = rn; t > pos; t--) raw[t] = raw[t - 1];
                    raw[pos] = s;
                    rn++;
                }
            }
            if (over) break;
            uint32_t nn = 0;
            auto push = [&](uint32_t b, uint32_t e) {
                if (nn && b == ne[nn - 1] + 1) { ne[nn - 1] = e; return; }
                if (nn == KW) { over = true; return; }
                nb[nn] = b; ne[nn] = e; nn++;
            };
            for (uint32_t t = 0; t < rn && !over;) {
                // a maximal run of [seg_lo[s], s-1] ranges (link(), :533-561)
                const uint32_t lo = X.seg_lo[raw[t]];
                uint32_t hi = raw[t];
                uint32_t t2 = t + 1;
                while (t2 < rn && X.seg_lo[raw[t2]] <= hi) { hi = raw[t2]; t2++; }
                uint32_t x0, x1, y0, y1;
                rank2_pair(X.occ, X.seg_start[lo], X.seg_start[hi], c, x0, x1, y0, y1);  // hi: one past the last word of segment hi-1
                if (y1 > x1) push(X.C[c] + x1, X.C[c] + y1 - 1);
                t = t2;
            }
            for (uint32_t q = 0; q < cn && !over; q++)
                if (se[q] > sb[q]) push(X.C[c] + sb[q], X.C[c] + se[q] - 1);
            if (over) break;
            cn = nn;
            for (uint32_t t = 0; t < cn; t++) { cb[t] = nb[t]; ce[t] = ne[t]; }
        }
        if (over) { flag_push(ovf2, i); continue; }
        for (uint32_t t = 1; t < cn; t++) {  // ascending rows
            const uint32_t xb = cb[t], xe = ce[t];
            uint32_t q = t;
            while (q && cb[q - 1] > xb) { cb[q] = cb[q - 1]; ce[q] = ce[q - 1]; q--; }
            cb[q] = xb; ce[q] = xe;
        }
        const uint32_t o = perm[i];
        uint32_t occ = 0;
        const uint64_t at = abase + (uint64_t)j * KW;
        if (cn == 1) {
            put_res(res, o, cb[0], 1u | kResRow, ce[0] - cb[0] + 1);
            continue;
        }
        for (uint32_t t = 0; t < cn; t++) { ab[at + t] = cb[t]; ae[at + t] = ce[t]; occ += ce[t] - cb[t] + 1; }
        put_res(res, o, at, cn, occ);
    }
}

// Wide lists, one wavefront per pattern (the patterns whose list outgrew k_deep's registers):
// lane t holds interval t of the list (at most 64) and steps it by the pattern's next character
// with one rank-entry load per end (updateSingleInterval, MOVE_EDSBWTSearch.cpp:424-510).  The
// link (:512-563): the '#' rows of every lane's interval are gathered in LDS, their segments
// sorted and deduplicated by the wave, cut into maximal runs of [seg_lo[s], s-1] ranges (a lane
// per run) and stepped from the occ blocks; the new list (runs and stepped intervals) is sorted
// by row and adjacent intervals merged (:309-324), so lists stay short and end sorted, as the
// finished list must be.  A list or a '#'-row set beyond the wave's LDS goes to the level path
// (ovf2), as it did for the lane-per-pattern k_deep_wide.
constexpr uint32_t kWaveHash = 512;  // '#' rows one step may gather
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, uint32_t lane, uint32_t& total) {
    uint32_t v = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(v, o, 64);
        if ((int)lane >= o) v += y;
    }
    total = __shfl(v, 63, 64);
    return v - x;
}
// the n (<= 128) intervals in lb/le, sorted by row into tb/te and adjacent ones merged; lane r
// receives the r-th merged interval.  Returns the merged count (> 64: the caller overflows).
__device__ __forceinline__ uint32_t wave_sort_merge(uint32_t n, uint32_t* lb, uint32_t* le, uint32_t* tb, uint32_t* te, uint32_t lane,
                                                    uint32_t& cb, uint32_t& ce) {
    for (uint32_t k = lane; k < n; k += 64) {  // rank sort: the rows of disjoint intervals are distinct
        const uint32_t v = lb[k];
        uint32_t r = 0;
        for (uint32_t q = 0; q < n; q++) r += lb[q] < v;
        tb[r] = v;
        te[r] = le[k];
    }
    __threadfence_block();
    uint32_t m = 0;
    cb = ce = 0;
    for (uint32_t base = 0; base < n; base += 64) {
        const uint32_t k = base + lane;
        const bool start = k < n && (k == 0 || tb[k] != te[k - 1] + 1u);
        const uint64_t sm = __ballot(start);
        // a run's end: one before the next start (or the list's end)
        if (start) {
            uint32_t e = k + 1;
            while (e < n && tb[e] == te[e - 1] + 1u) e++;
            const uint32_t r = m + lane_rank(sm, lane);
            if (r < 64) {  // park the merged interval at slot r of lb/le (read back below)
                lb[128 + r] = tb[k];
                le[128 + r] = te[e - 1];
            }
        }
        m += (uint32_t)__popcll(sm);
    }
    __threadfence_block();
    if (lane < m && m <= 64) { cb = lb[128 + lane]; ce = le[128 + lane]; }
    return m;
}
__global__ void __launch_bounds__(256) k_deep_wave(uint64_t P, uint32_t D0, const uint32_t* __restrict__ todo, uint32_t ntodo,
                                                  const uint32_t* __restrict__ slen, const uint32_t* __restrict__ perm, uint32_t ind,
                                                  const uint64_t* __restrict__ off, const uint8_t* __restrict__ bytes,
                                                  const uint8_t* __restrict__ code_of, const uint32_t* __restrict__ nid,
                                                  const uint32_t* __restrict__ ioff, const uint32_t* __restrict__ iend,
                                                  const uint32_t* __restrict__ ib, const uint32_t* __restrict__ ie, KIdx X, uint64_t abase,
                                                  uint32_t* __restrict__ ab, uint32_t* __restrict__ ae, Res* __restrict__ res,
                                                  uint32_t* __restrict__ ovf2, const uint32_t* __restrict__ ntodo_dev,
                                                  unsigned long long* __restrict__ ctr, uint32_t* __restrict__ counts) {
    (void)P;
    CountSums cs;  // (lane 0 of each wave puts its patterns' counts)
    __shared__ uint32_t s_seg[4][kWaveHash], s_tmp[4][kWaveHash];
    __shared__ uint32_t s_b[4][192], s_e[4][192];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t* seg = s_seg[wv];
    uint32_t* tmp = s_tmp[wv];
    uint32_t* lb = s_b[wv];
    uint32_t* le = s_e[wv];
    // ntodo_dev (deferred checks): the list's length lives on the device; ntodo is the grid's
    // capacity, and a longer list is caught by the caller's final check
    if (ntodo_dev) ntodo = min(ntodo, *ntodo_dev);
    unsigned long long n_blk = 0, n_steps = 0;
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t j = blockIdx.x * (blockDim.x >> 6) + wv; j < ntodo; j += nwaves) {  // wave-uniform
        const uint32_t i = todo[j];
        const uint32_t L = slen[ind ? perm[i] : i];
        const uint32_t u = nid[i];
        const uint32_t o0 = ioff[u];
        uint32_t cn = iend[u] - o0;
        if (cn > 64) {
            if (lane == 0) flag_push(ovf2, i);
            continue;
        }
        if (lane < cn) { lb[lane] = ib[o0 + lane]; le[lane] = ie[o0 + lane]; }
        __threadfence_block();
        uint32_t cb, ce;
        cn = wave_sort_merge(cn, lb, le, tmp, tmp + 256, lane, cb, ce);
        const uint8_t* pat = bytes + off[perm[i]];
        bool over = false;
        for (uint32_t d = D0; d < L && cn && !over; d++) {
            const uint32_t c = code_of[pat[L - 1 - d]];
            if (c >= X.sigma) { cn = 0; break; }
            // every interval stepped by c, and its '#' rows [h0, h1)
            uint32_t h0 = 0, h1 = 0, sb = 0, se = 0;
            if (lane < cn) {
                n_blk += 2 - rank2_any(X, cb, ce + 1, c, h0, sb, h1, se);
                n_steps++;
            }
            uint32_t H;
            const uint32_t hpre = wave_excl_scan(h1 - h0, lane, H);
            if (H > kWaveHash) { over = true; break; }
            for (uint32_t k = h0; k < h1; k++) seg[hpre + k - h0] = X.eof_seg[k];
            __threadfence_block();
            // keep the segments of words outside segment 1 (eof_seg 0: no previous segment)
            uint32_t R0 = 0;
            for (uint32_t base = 0; base < H; base += 64) {
                const uint32_t v = base + lane < H ? seg[base + lane] : 0u;
                const uint64_t km = __ballot(v != 0);
                __threadfence_block();
                if (v) tmp[R0 + lane_rank(km, lane)] = v;
                R0 += (uint32_t)__popcll(km);
            }
            __threadfence_block();
            // sorted (rank with ties broken by position) into seg, then the distinct ones into tmp
            for (uint32_t k = lane; k < R0; k += 64) {
                const uint32_t v = tmp[k];
                uint32_t r = 0;
                for (uint32_t q = 0; q < R0; q++) {
                    const uint32_t w = tmp[q];
                    r += (w < v) || (w == v && q < k);
                }
                seg[r] = v;
            }
            __threadfence_block();
            uint32_t R = 0;
            for (uint32_t base = 0; base < R0; base += 64) {
                const uint32_t k = base + lane;
                const bool f = k < R0 && (k == 0 || seg[k] != seg[k - 1]);
                const uint64_t fm = __ballot(f);
                if (f) tmp[R + lane_rank(fm, lane)] = seg[k];
                R += (uint32_t)__popcll(fm);
            }
            __threadfence_block();
            if (R > 64) { over = true; break; }
            // maximal runs (link(), :533-561): a run starts where seg_lo of the segment passes the
            // previous segment; lane r handles the run starting at distinct segment r
            const uint32_t sr = lane < R ? tmp[lane] : 0u;
            const uint32_t lor = lane < R ? X.seg_lo[sr] : 0u;
            const uint32_t prev = __shfl_up(sr, 1, 64);
            const bool rstart = lane < R && (lane == 0 || lor > prev);
            const uint64_t rm = __ballot(rstart);
            uint32_t nb_ = 0, ne_ = 0;
            bool rv = false;
            if (rstart) {
                const uint64_t later = lane == 63 ? 0ull : rm & ~((2ull << lane) - 1ull);  // starts after this lane
                const uint32_t end = later ? (uint32_t)(__ffsll((unsigned long long)later) - 1) - 1u : R - 1u;
                const uint32_t hi = tmp[end];
                uint32_t x0, x1, y0, y1;
                rank2_pair(X.occ, X.seg_start[lor], X.seg_start[hi], c, x0, x1, y0, y1);  // hi: one past the last word of segment hi-1
                n_blk += 2;
                if (y1 > x1) { rv = true; nb_ = X.C[c] + x1; ne_ = X.C[c] + y1 - 1; }
            }
            // the new list: runs, then stepped intervals, into lb/le; sorted and merged
            const uint64_t vm = __ballot(rv), sm = __ballot(lane < cn && se > sb);
            const uint32_t nr = (uint32_t)__popcll(vm), ns = (uint32_t)__popcll(sm);
            __threadfence_block();
            if (rv) { const uint32_t r = lane_rank(vm, lane); lb[r] = nb_; le[r] = ne_; }
            if (lane < cn && se > sb) { const uint32_t r = nr + lane_rank(sm, lane); lb[r] = X.C[c] + sb; le[r] = X.C[c] + se - 1; }
            __threadfence_block();
            cn = wave_sort_merge(nr + ns, lb, le, tmp, tmp + 256, lane, cb, ce);
            if (cn > 64) over = true;
        }
        if (over) {
            if (lane == 0) flag_push(ovf2, i);
            continue;
        }
        const uint32_t o = perm[i];
        const uint64_t at = abase + (uint64_t)j * 64;
        if (cn == 1) {
            if (lane == 0) {
                put_res(res, o, cb, 1u | kResRow, ce - cb + 1);
                cs.put(counts, o, ce - cb + 1);
            }
            continue;
        }
        uint32_t occ = lane < cn ? ce - cb + 1 : 0u;
#pragma unroll
        for (int q = 32; q >= 1; q >>= 1) occ += __shfl_xor(occ, q, 64);
        if (lane < cn) { ab[at + lane] = cb; ae[at + lane] = ce; }
        if (lane == 0) {
            put_res(res, o, at, cn, occ);
            cs.put(counts, o, occ);
        }
    }
    __shared__ unsigned long long ssum[4];
    stat_add(ctr, ST_DW_BLOCKS, n_blk, ssum);
    stat_add(ctr, ST_DW_STEPS, n_steps, ssum);
    cs.flush(counts, ctr, ssum);
}

__global__ void k_list_flagged(uint64_t P, const uint32_t* __restrict__ flag, const uint32_t* __restrict__ fscan, uint32_t* __restrict__ out) {
    GRID_STRIDE(i, P) if (flag[i]) out[fscan[i]] = (uint32_t)i;
}

// pattern-length histogram: per-block LDS bins, one global atomic per bin per block
__global__ void __launch_bounds__(256) k_len_hist(const uint32_t* __restrict__ len, uint64_t P, uint32_t Lmax,
                                                  unsigned long long* __restrict__ hist) {
    __shared__ unsigned int h[1024];
    const uint32_t nb = Lmax + 1 < 1024 ? Lmax + 1 : 1024;
    for (uint32_t t = threadIdx.x; t < nb; t += blockDim.x) h[t] = 0;
    __syncthreads();
    GRID_STRIDE(i, P) {
        const uint32_t l = len[i];
        if (l < nb) atomicAdd(&h[l], 1u);
        else atomicAdd(hist + (l < Lmax ? l : Lmax), 1ull);
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < nb; t += blockDim.x)
        if (h[t]) atomicAdd(hist + t, (unsigned long long)h[t]);
}

// overflowed patterns → a compact sub-batch (original ids kept in `map`)
// patterns the deep kernels could not hold (a flag_push list), flagged by input index
// path tags (EDSBWT_PATH_TAGS, tests): the patterns a kernel's queue or list held.  Queue:
// sharded (region s at s*qcap, count at qcnt[s*32]), entry .x = sorted pattern index.  List:
// list[0] = count, then sorted indices.  perm maps sorted -> batch index, map (grouped
// search) batch -> caller's index.
__global__ void k_tag_queue(const uint4* __restrict__ q, const uint32_t* __restrict__ qcnt, uint32_t qcap, const uint32_t* __restrict__ perm,
                            const uint32_t* __restrict__ map, uint8_t* __restrict__ tag, uint32_t bit) {
    GRID_STRIDE(j, (uint64_t)qcap * NSHARD) {
        const uint32_t sh = (uint32_t)(j / qcap), at = (uint32_t)(j % qcap);
        if (at < min(qcnt[sh * 32], qcap)) {
            uint32_t p = perm[q[j].x];
            if (map) p = map[p];
            tag[p] |= (uint8_t)bit;
        }
    }
}
__global__ void k_tag_list(const uint32_t* __restrict__ list, uint64_t cap, const uint32_t* __restrict__ perm,
                           const uint32_t* __restrict__ map, uint8_t* __restrict__ tag, uint32_t bit) {
    GRID_STRIDE(j, cap) {
        if (j < list[0]) {
            uint32_t p = perm[list[1 + j]];
            if (map) p = map[p];
            tag[p] |= (uint8_t)bit;
        }
    }
}
__global__ void k_tag_all(uint8_t* __restrict__ tag, uint64_t n, uint32_t bit) { GRID_STRIDE(i, n) tag[i] |= (uint8_t)bit; }
__global__ void k_ovf_mark(uint32_t n, const uint32_t* __restrict__ list, const uint32_t* __restrict__ perm, uint32_t* __restrict__ flag_orig) {
    GRID_STRIDE(j, n) flag_orig[perm[list[j]]] = 1;
}

__global__ void k_sub_build(uint64_t P, const uint32_t* __restrict__ flag, const uint32_t* __restrict__ fscan, const uint32_t* __restrict__ len,
                            uint32_t* __restrict__ map, uint64_t* __restrict__ sublen) {
    GRID_STRIDE(o, P) if (flag[o]) { map[fscan[o]] = (uint32_t)o; sublen[fscan[o]] = len[o]; }
}

__global__ void k_sub_bytes(uint64_t n, const uint32_t* __restrict__ map, const uint64_t* __restrict__ off, const uint64_t* __restrict__ suboff,
                            const uint8_t* __restrict__ bytes, uint8_t* __restrict__ subbytes) {
    GRID_STRIDE(j, n) {
        const uint64_t s = off[map[j]], d = suboff[j], l = suboff[j + 1] - d;
        for (uint64_t t = 0; t < l; t++) subbytes[d + t] = bytes[s + t];
    }
}

__global__ void k_sub_scatter(uint64_t n, const uint32_t* __restrict__ map, const Res* __restrict__ sr, Res* __restrict__ res) {
    GRID_STRIDE(j, n) res[map[j]] = sr[j];
}

// ------------------------------------------- order-free level step (default path)
// A node's interval list is kept as an unordered set of (node, b, e) items: merging
// adjacent intervals and the order of the list never change the rows locate emits
// (LF_c is monotone on each pile and the reference's lists are ascending and
// disjoint for patterns without '#'), so every level is one fused pass that reads
// each item's two occ-block lines and appends only the non-empty children.

// Children of node u, packed by k_child_info: child_info[u] = first child | symbol
// mask << 32.  Children are in trie order (ascending symbol code, a child for bytes
// outside the alphabet last), so the child with symbol c is first + popcount of the
// mask bits below c.  Mask bit 8 + c (node_first given): that child finishes a pattern
// (its first pattern, the shortest in trie order, has length D) — the count-only step
// sums its occurrences.
__global__ void k_child_info(uint32_t M, const uint32_t* __restrict__ node_parent, const uint8_t* __restrict__ node_char,
                             uint64_t* __restrict__ info, uint32_t D, const uint32_t* __restrict__ node_first,
                             const uint32_t* __restrict__ slen) {
    GRID_STRIDE(u, M) {
        const uint32_t p = node_parent[u];
        if (u == 0 || node_parent[u - 1] != p) {
            uint32_t mask = 0;
            for (size_t v = u; v < M && node_parent[v] == p; v++) {
                const uint32_t c = node_char[v];
                if (c < 8) {
                    mask |= 1u << c;
                    if (node_first && slen[node_first[v]] == D) mask |= 1u << (8 + c);
                }
            }
            info[p] = ((uint64_t)mask << 32) | (uint32_t)u;
        }
    }
}

// Count-only finishing fused into the level step: a finishing child's occurrences
// (e - b + 1 of each interval it receives, as k_fin_emit sums them) go to a block-wide
// LDS table (open addressing; a full probe run adds to memory directly), which goes to
// node_occ once at the end of the block.
constexpr uint32_t kFinH = 1024;
__device__ __forceinline__ void fin_add(uint32_t* hk, uint32_t* hv, uint32_t* __restrict__ node_occ, uint32_t key, uint32_t v) {
    uint32_t slot = (key * 2654435761u) >> 22;
    for (uint32_t q = 0; q < 16; q++, slot = (slot + 1) & (kFinH - 1)) {
        const uint32_t seen = hk[slot];
        if (seen == key) { atomicAdd(&hv[slot], v); return; }
        if (seen == 0xffffffffu) {
            const uint32_t old = atomicCAS(&hk[slot], 0xffffffffu, key);
            if (old == 0xffffffffu || old == key) { atomicAdd(&hv[slot], v); return; }
        }
    }
    atomicAdd(node_occ + key, v);
}
__device__ __forceinline__ void fin_init(uint32_t* hk, uint32_t* hv) {
    for (uint32_t t = threadIdx.x; t < kFinH; t += blockDim.x) { hk[t] = 0xffffffffu; hv[t] = 0; }
}
__device__ __forceinline__ void fin_flush(const uint32_t* hk, const uint32_t* hv, uint32_t* __restrict__ node_occ) {
    for (uint32_t t = threadIdx.x; t < kFinH; t += blockDim.x)
        if (hv[t]) atomicAdd(node_occ + hk[t], hv[t]);
}

// one interval (node u, rows b..e1-1) stepped by every live child symbol: appends the
// non-empty children.  The rank loads do not wait for the node's child word.
#define LVL_STEP_LOAD(u, b, e1)                                                         \
    {                                                                                   \
        const uint64_t ci = child_info[u];                                              \
        n_blk += 2 - rank_all_pair_any(X, b, e1, rb, re);                               \
        cf = (uint32_t)ci;                                                              \
        mask = (uint32_t)(ci >> 32);                                                    \
    }

__device__ __forceinline__ void lvl_emit(uint32_t mask, uint32_t emit, uint32_t cf, const uint32_t* rb, const uint32_t* re, const KIdx& X,
                                         uint32_t at, uint32_t cap, uint32_t* __restrict__ nu, uint32_t* __restrict__ nb,
                                         uint32_t* __restrict__ ne, uint32_t* hk, uint32_t* hv, uint32_t* __restrict__ node_occ,
                                         uint32_t tmask = 0, const uint2* tform = nullptr) {
    // tmask bit c: child c's one row goes on as the text item tform[c] (k_lvl_dollar, KIdx::segtext)
#pragma unroll
    for (uint32_t c = 0; c < 8; c++)
        if ((emit >> c) & 1) {
            const uint32_t child = cf + (uint32_t)__popc(mask & ((1u << c) - 1u));
            if (at < cap) {
                nu[at] = child;
                const bool t = (tmask >> c) & 1u;
                nb[at] = t ? tform[c].x : X.C[c] + rb[c];
                ne[at] = t ? tform[c].y : X.C[c] + re[c] - 1;
            }
            at++;
            // (counted whether or not the append fits: a relaunch after a regrow passes no node_occ)
            if (node_occ && ((mask >> (8 + c)) & 1)) fin_add(hk, hv, node_occ, child, re[c] - rb[c]);
        }
}

// Text items (count-only level walk): a single row whose suffix starts r <= 16
// characters after its word's start is one text position, so its next r backward steps are the
// r text characters before it and its '#' comes right after them.  Its first step reads the row's
// srow line (sample + text window) instead of a rank entry, and its child becomes a text item
// (node, kTextItem | r << 27 | segment, the next 16 characters, 2 bits each): every further step
// takes its character from the item itself and needs only the node's child word; at r = 0 it
// leaves the link key of its word's segment, as the row's '#' would.  Items carry no row, so
// they exist only when the walk counts (fused finish) and never reach the deep cutover.
constexpr uint32_t kTextItem = 0x80000000u, kTextSeg = 0x07ffffffu;

template <bool LINK, int MINW = 1>  // MINW 8: 8 waves per SIMD (the kernel arguments then spill to VGPR lanes)
__global__ void __launch_bounds__(256, MINW) k_lvl_items(uint32_t n, const uint32_t* __restrict__ iu, const uint32_t* __restrict__ ib,
                                                   const uint32_t* __restrict__ ie, const uint64_t* __restrict__ child_info, KIdx X,
                                                   uint32_t* __restrict__ nu, uint32_t* __restrict__ nb, uint32_t* __restrict__ ne,
                                                   uint32_t cap_next, uint32_t* __restrict__ cnt_all, uint64_t* __restrict__ keys,
                                                   uint32_t cap_keys, uint32_t* __restrict__ ck_u, uint32_t* __restrict__ ck_k,
                                                   uint32_t* __restrict__ ck_e, uint32_t cap_chunks, unsigned long long* __restrict__ stats,
                                                   const uint32_t* __restrict__ ipre, uint32_t icap, uint32_t* __restrict__ node_occ,
                                                   uint32_t text_mode) {
    // ipre != nullptr: the input items are still in the previous depth's NSHARD regions
    // (region s at s*icap, ipre = their prefix sums), read in place instead of packed;
    // node_occ != nullptr (count only): finishing children's occurrences are summed here;
    // text_mode bit 0: step text items (rows < 2^31), bit 1: also turn single rows into them
    __shared__ uint32_t spre[NSHARD + 1];
    __shared__ uint32_t hk[kFinH], hv[kFinH];
    if (node_occ) fin_init(hk, hv);
    if (ipre)
        for (uint32_t t = threadIdx.x; t <= NSHARD; t += blockDim.x) spre[t] = ipre[t];
    if (ipre || node_occ) __syncthreads();
    const uint32_t sh = blockIdx.x % NSHARD;
    unsigned long long n_blk = 0, n_single = 0;  // occ blocks read, single-row items
    uint32_t* cnt = cnt_all + sh * 32;
    nu += (size_t)sh * cap_next; nb += (size_t)sh * cap_next; ne += (size_t)sh * cap_next;
    keys += (size_t)sh * cap_keys;
    ck_u += (size_t)sh * cap_chunks; ck_k += (size_t)sh * cap_chunks; ck_e += (size_t)sh * cap_chunks;
    UNIFORM_STRIDE(i, valid, n) {
        uint32_t u = 0, cf = 0, mask = 0;
        uint32_t rb[8], re[8];
#pragma unroll
        for (int t = 0; t < 8; t++) rb[t] = re[t] = 0;
        bool tx = false;  // a text item (or a single row turned into one): r, segment, window,
        uint32_t t_r = 0, t_seg = 0, t_win = 0, t_ch = 0;  // and the segment's chain bit (seg_lo != s - 1)
        if (valid) {
            size_t src = i;
            if (ipre) {
                uint32_t lo = 0, hi = NSHARD;
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (spre[mid] <= (uint32_t)i) lo = mid; else hi = mid;
                }
                src = (size_t)lo * icap + ((uint32_t)i - spre[lo]);
            }
            u = iu[src];
            const uint32_t b0 = ib[src], e0 = ie[src];
            n_single += b0 == e0;
            if (text_mode && (b0 & kTextItem)) {
                const uint64_t ci = child_info[u];
                cf = (uint32_t)ci;
                mask = (uint32_t)(ci >> 32);
                tx = true;
                t_r = (b0 >> 27) & 15u;
                t_seg = b0 & kTextSeg;
                t_win = e0 & 0x7fffffffu;
                t_ch = e0 >> 31;
            } else if ((text_mode & 2u) && b0 == e0) {
                const uint64_t ci = child_info[u];
                const uint4 s0 = X.srow[2 * (size_t)b0];  // (word, offset, segment, word in segment)
                const uint4 s1 = X.srow[2 * (size_t)b0 + 1];  // {text position, 0, window}
                n_blk += 1;
                cf = (uint32_t)ci;
                mask = (uint32_t)(ci >> 32);
                if (s0.y <= 16) {
                    tx = true;
                    t_r = s0.y;
                    t_seg = s0.z;
                    t_win = s1.z;
                    t_ch = s1.y & 1u;
                } else {  // a suffix deeper in a long word: the rank step
                    n_blk += 2 - rank_all_pair_any(X, b0, e0 + 1, rb, re);
                }
            } else {
                LVL_STEP_LOAD(u, b0, e0 + 1)
            }
        }
        // backward step of every child symbol (updateSingleInterval, :424-510)
        uint32_t emit = 0;
#pragma unroll
        for (uint32_t c = 0; c < 8; c++)
            if (((mask >> c) & 1) && re[c] > rb[c]) emit |= 1u << c;
        // a text item steps by its next character only (r > 0), or meets its word's '#' (r = 0)
        uint32_t t_c = 0;
        bool t_child = false, t_key = false;
        if (tx) {
            if (t_r == 0) {
                t_key = LINK && (mask & 0xffu) && t_seg >= 2;
            } else {
                t_c = 1u + (t_win & 3u);
                t_child = (mask >> t_c) & 1u;
            }
        }
        const uint32_t nk = (uint32_t)__popc(emit) + (t_child ? 1u : 0u);
        // '#' rows of the item (dollars_in_interval, :607-625): short ranges inline,
        // long ones as chunks of 256 rows for k_lvl_chunks
        const uint32_t h = (LINK && mask) ? re[0] - rb[0] : 0u;
        const uint32_t nc = h > 16 ? (h + 255) / 256 : 0u;
        uint32_t nz = t_key ? 1u : 0u;
        if (LINK && h && h <= 16)
            for (uint32_t k = rb[0]; k < re[0]; k++) nz += X.link_seg[k] != 0;
        uint32_t at, kat, cat;
        wave_append3(cnt, nk, nz, nc, at, kat, cat);  // one atomic round trip for the three lists
        lvl_emit(mask, emit, cf, rb, re, X, at, cap_next, nu, nb, ne, hk, hv, node_occ);
        if (text_mode) {
            if (t_child) {
                const uint32_t child = cf + (uint32_t)__popc(mask & ((1u << t_c) - 1u));
                if (at < cap_next) {
                    nu[at] = child;
                    nb[at] = kTextItem | ((t_r - 1u) << 27) | t_seg;
                    ne[at] = (t_win >> 2) | (t_ch << 31);
                }
                if (node_occ && ((mask >> (8 + t_c)) & 1u)) fin_add(hk, hv, node_occ, child, 1u);
            }
            const uint64_t tb = __ballot(t_child);  // text items handed to the next depth (the deep cutover waits for none)
            if ((threadIdx.x & 63) == 0 && tb) atomicAdd(cnt + 5, (uint32_t)__popcll(tb));
        }
        if (LINK) {
            if (t_key) {
                if (kat < cap_keys) keys[kat] = ((uint64_t)u << (X.segbits + X.link_cb)) | (X.link_cb ? t_seg << 1 | t_ch : t_seg);
                kat++;
            }
            if (nz)
                for (uint32_t k = rb[0]; k < re[0]; k++) {
                    const uint32_t s = X.link_seg[k];
                    if (s) {
                        if (kat < cap_keys) keys[kat] = ((uint64_t)u << (X.segbits + X.link_cb)) | s;
                        kat++;
                    }
                }
            // chunk records: a lane writes a few itself; the wave writes long runs together
            // (the root's items hold every '#' row: thousands of chunks each)
            if (nc && nc <= 8)
                for (uint32_t q = 0; q < nc; q++)
                    if (cat + q < cap_chunks) {
                        ck_u[cat + q] = u;
                        ck_k[cat + q] = rb[0] + 256 * q;
                        ck_e[cat + q] = min(rb[0] + 256 * (q + 1), re[0]);
                    }
            uint64_t big = __ballot(nc > 8);
            const uint32_t lane = threadIdx.x & 63;
            while (big) {
                const int l = __ffsll((unsigned long long)big) - 1;
                big &= big - 1;
                const uint32_t lu = __shfl(u, l, 64), lb = __shfl(rb[0], l, 64), le = __shfl(re[0], l, 64);
                const uint32_t lc = __shfl(cat, l, 64), ln = __shfl(nc, l, 64);
                for (uint32_t q = lane; q < ln; q += 64)
                    if (lc + q < cap_chunks) {
                        ck_u[lc + q] = lu;
                        ck_k[lc + q] = lb + 256 * q;
                        ck_e[lc + q] = min(lb + 256 * (q + 1), le);
                    }
            }
        }
    }
    if (node_occ) {
        __syncthreads();
        fin_flush(hk, hv, node_occ);
    }
    __shared__ unsigned long long ssum[4];
    stat_add(stats, ST_STEP_BLOCKS, n_blk, ssum);
    stat_add(stats, ST_LVL_SINGLE, n_single, ssum);
}

// long '#'-row ranges: one wave per chunk (<= 256 rows, clipped to the item's end);
// lanes read 4 rows each (coalesced), one atomic per wave
__global__ void __launch_bounds__(256) k_lvl_chunks(uint32_t n, const uint32_t* __restrict__ ck_u, const uint32_t* __restrict__ ck_k,
                                                    const uint32_t* __restrict__ ck_end, KIdx X, uint32_t* __restrict__ cnt_all,
                                                    uint64_t* __restrict__ keys, uint32_t cap_keys) {
    const uint32_t sh = blockIdx.x % NSHARD;
    uint32_t* cnt = cnt_all + sh * 32;
    keys += (size_t)sh * cap_keys;
    const uint32_t lane = threadIdx.x & 63, wib = threadIdx.x >> 6, wpb = blockDim.x >> 6;
    for (size_t w = (size_t)blockIdx.x * wpb + wib; w < n; w += (size_t)gridDim.x * wpb) {  // wave-uniform
        const uint32_t u = ck_u[w], k0 = ck_k[w], k1 = ck_end[w];
        uint32_t s[4], nz = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t k = k0 + lane + 64 * q;
            s[q] = k < k1 ? X.link_seg[k] : 0u;
            nz += s[q] != 0;
        }
        uint32_t at = wave_append(cnt + 1, nz);
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (s[q]) {
                if (at < cap_keys) keys[at] = ((uint64_t)u << (X.segbits + X.link_cb)) | s[q];
                at++;
            }
    }
}

// dollar items (previous-segment word ranges of a node) stepped by each child
template <int MINW = 1>
__global__ void __launch_bounds__(256, MINW) k_lvl_dollar(const uint32_t* __restrict__ dn, const uint32_t* __restrict__ du, const uint32_t* __restrict__ db,
                                                    const uint32_t* __restrict__ de, const uint64_t* __restrict__ child_info, KIdx X,
                                                    uint32_t* __restrict__ nu, uint32_t* __restrict__ nb, uint32_t* __restrict__ ne,
                                                    uint32_t cap_next, uint32_t* __restrict__ cnt_all, unsigned long long* __restrict__ stats,
                                                    uint32_t* __restrict__ node_occ, uint32_t text_mode) {
    // text_mode bit 1 (text items made at this depth) with KIdx::segtext: a single-key run's child
    // interval of ONE row goes on as that row's text item, read from the run's own segment row
    const uint32_t n = *dn;  // link runs, counted on the device by k_run_build
    unsigned long long n_blk = 0;  // occ blocks read
    // node_occ != nullptr (count only): finishing children's occurrences are summed here
    __shared__ uint32_t hk[kFinH], hv[kFinH];
    if (node_occ) {
        fin_init(hk, hv);
        __syncthreads();
    }
    const uint32_t sh = blockIdx.x % NSHARD;
    uint32_t* cnt = cnt_all + sh * 32;
    nu += (size_t)sh * cap_next; nb += (size_t)sh * cap_next; ne += (size_t)sh * cap_next;
    UNIFORM_STRIDE(i, valid, n) {
        uint32_t cf = 0, mask = 0;
        uint32_t rb[8], re[8];
#pragma unroll
        for (int t = 0; t < 8; t++) rb[t] = re[t] = 0;
        uint2 tform[8];
        bool one_seg = false;
        const uint32_t* e0 = nullptr;
        if (valid) {
            const uint32_t u = du[i];
            const uint64_t ci = child_info[u];
            const uint32_t s0 = db[i], s1 = de[i];
            one_seg = s0 == s1;
            e0 = X.segtab + (size_t)s0 * X.seg_stride;  // s_first: ranks at the run's first word
            const uint32_t* e1 = X.segtab + (size_t)s1 * X.seg_stride;  // s_last: ranks one past its last word
            if (X.seg_stride >= 16 && X.seg_hi == 8) {  // sigma <= 7: [lo, lo-ranks 1..7 | hi-ranks 8..14, pad] as 16-B vectors
                const uint4 a0 = reinterpret_cast<const uint4*>(e0)[0], a1 = reinterpret_cast<const uint4*>(e0)[1];
                const uint4 b0 = reinterpret_cast<const uint4*>(e1)[2], b1 = reinterpret_cast<const uint4*>(e1)[3];
                rb[0] = a0.y; rb[1] = a0.z; rb[2] = a0.w; rb[3] = a1.x; rb[4] = a1.y; rb[5] = a1.z; rb[6] = a1.w;
                re[0] = b0.x; re[1] = b0.y; re[2] = b0.z; re[3] = b0.w; re[4] = b1.x; re[5] = b1.y; re[6] = b1.z;
            } else {
#pragma unroll
                for (uint32_t c = 0; c < 8; c++)
                    if (c < X.sigma) { rb[c] = e0[1 + c]; re[c] = e1[X.seg_hi + c]; }
            }
            n_blk += 2;
            cf = (uint32_t)ci;
            mask = (uint32_t)(ci >> 32);
        }
        uint32_t emit = 0;
#pragma unroll
        for (uint32_t c = 0; c < 8; c++)
            if (((mask >> c) & 1) && re[c] > rb[c]) emit |= 1u << c;
        uint32_t tmask = 0;
        if ((text_mode & 2u) && X.segtext && one_seg) {
            // single rows of a one-key run: the word's text item from the run segment's row (same line)
#pragma unroll
            for (uint32_t c = 1; c <= 4; c++)
                if (((emit >> c) & 1) && re[c] - rb[c] == 1) {
                    tform[c] = reinterpret_cast<const uint2*>(e0 + 16)[c - 1];
                    if (tform[c].x & kTextItem) tmask |= 1u << c;
                }
        }
        const uint32_t at = wave_append(cnt + 0, (uint32_t)__popc(emit));
        lvl_emit(mask, emit, cf, rb, re, X, at, cap_next, nu, nb, ne, hk, hv, node_occ, tmask, tform);
        if (text_mode) {  // text items handed to the next depth (the deep cutover waits for none)
            const uint64_t tb = __ballot(tmask != 0);
            const uint32_t nt = (uint32_t)__popc(tmask);
            uint32_t wsum = nt;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) wsum += __shfl_xor(wsum, o, 64);
            if ((threadIdx.x & 63) == 0 && tb) atomicAdd(cnt + 5, wsum);
        }
    }
    if (node_occ) {
        __syncthreads();
        fin_flush(hk, hv, node_occ);
    }
    __shared__ unsigned long long ssum[4];
    stat_add(stats, ST_STEP_BLOCKS, n_blk, ssum);
}

// finishing nodes (patterns of length D): (node << rowbits | b, e) pairs, sorted later
__global__ void __launch_bounds__(256) k_fin_emit(uint32_t n, const uint32_t* __restrict__ nu, const uint32_t* __restrict__ nb,
                                                  const uint32_t* __restrict__ ne, const uint8_t* __restrict__ fin, uint32_t* __restrict__ cnt_all,
                                                  uint64_t* __restrict__ fk, uint32_t* __restrict__ fv, uint32_t cap,
                                                  uint32_t* __restrict__ node_occ, uint32_t rowbits, const uint32_t* __restrict__ ipre,
                                                  uint32_t icap) {
    // ipre != nullptr: the items are still in the step's NSHARD regions (as k_lvl_items reads them)
    __shared__ uint32_t spre[NSHARD + 1];
    // the block's occurrence sums per finishing node (open addressing; full: global atomics)
    constexpr uint32_t kH = 1024;
    __shared__ uint32_t hk[kH], hv[kH];
    for (uint32_t t = threadIdx.x; t < kH; t += blockDim.x) { hk[t] = 0xffffffffu; hv[t] = 0; }
    if (ipre)
        for (uint32_t t = threadIdx.x; t <= NSHARD; t += blockDim.x) spre[t] = ipre[t];
    __syncthreads();
    const uint32_t sh = blockIdx.x % NSHARD;
    uint32_t* cnt = cnt_all + sh * 32;
    if (fk) { fk += (size_t)sh * cap; fv += (size_t)sh * cap; }
    UNIFORM_STRIDE(i, valid, n) {
        uint32_t f = 0, u = 0;
        size_t src = i;
        if (valid) {
            if (ipre) {
                uint32_t lo = 0, hi = NSHARD;
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (spre[mid] <= (uint32_t)i) lo = mid; else hi = mid;
                }
                src = (size_t)lo * icap + ((uint32_t)i - spre[lo]);
            }
            u = nu[src];
            f = fin[u];
        }
        // fk == nullptr (count only): the occurrence sums are all that is kept
        uint32_t at = wave_append(cnt + 4, fk ? f : 0u);
        uint32_t v = 0;
        if (f) {
            const uint32_t b = nb[src], e = ne[src];
            if (fk && at < cap) {
                fk[at] = ((uint64_t)u << rowbits) | b;
                fv[at] = e;
            }
            v = e - b + 1;
        }
        // a few finishing nodes can hold millions of items each (C5: a group's depth-8 nodes):
        // per-item atomics on one address serialise in L2.  The wave sums each distinct node
        // first (up to 8 of them; lanes left over add their own) into the block's LDS table,
        // which goes to memory once at the end.
        const int lane = threadIdx.x & 63;
        const uint32_t key = f ? u : 0xffffffffu;
        uint64_t todo = __ballot(key != 0xffffffffu && v != 0);
        for (int it = 0; it < 8 && todo; it++) {
            const int l = __ffsll((unsigned long long)todo) - 1;
            const uint32_t kl = __shfl(key, l, 64);
            const bool m = key == kl;
            uint32_t sum = m ? v : 0u;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 64);
            if (lane == l) {
                uint32_t slot = (kl * 2654435761u) >> 22, q = 0;
                for (; q < 16; q++, slot = (slot + 1) & (kH - 1)) {
                    const uint32_t old = atomicCAS(&hk[slot], 0xffffffffu, kl);
                    if (old == 0xffffffffu || old == kl) { atomicAdd(&hv[slot], sum); break; }
                }
                if (q == 16) atomicAdd(node_occ + kl, sum);
            }
            todo &= ~__ballot(m);
        }
        if ((todo >> lane) & 1) atomicAdd(node_occ + u, v);
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < kH; t += blockDim.x)
        if (hv[t]) atomicAdd(node_occ + hk[t], hv[t]);
}

// pack shard regions: item t of the packed array lives in shard s = last with
// pre[s] <= t, at s*cap + (t - pre[s])
template <typename A, typename B, typename C3>
__global__ void k_unshard(uint32_t total, const uint32_t* __restrict__ pre, uint32_t cap, const A* __restrict__ a, const B* __restrict__ b,
                          const C3* __restrict__ c, A* __restrict__ oa, B* __restrict__ ob, C3* __restrict__ oc) {
    __shared__ uint32_t sp[NSHARD + 1];
    for (uint32_t t = threadIdx.x; t <= NSHARD; t += blockDim.x) sp[t] = pre[t];
    __syncthreads();
    GRID_STRIDE(t, total) {
        uint32_t lo = 0, hi = NSHARD;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (sp[mid] <= (uint32_t)t) lo = mid; else hi = mid;
        }
        const size_t src = (size_t)lo * cap + ((uint32_t)t - sp[lo]);
        oa[t] = a[src];
        if (ob) ob[t] = b[src];
        if (oc) oc[t] = c[src];
    }
}

__global__ void k_fin_flags(uint32_t M, uint32_t D, const uint32_t* __restrict__ node_first, const uint32_t* __restrict__ slen,
                            uint8_t* __restrict__ fin) {
    GRID_STRIDE(u, M) fin[u] = slen[node_first[u]] == D;
}

// finishers at the level table's start (patterns of length L, engine.hip levels2): a node's items are
// [kt_pos[u], + kt_cnt[u]) as k_ltab_emit wrote them, already sorted by row (the table's order), so
// its archive range is those items as they are.  k_fin_lt_cnt: the finishing nodes' item counts
// (others 0), whose exclusive scan (foff) places each finishing node's list in the archive;
// k_fin_lt copies the finishing lists there and sums their occurrences — one wave per node, no emit,
// sort or bounds pass, and the lists of nodes that do not finish (only longer patterns pass them)
// never reach the archive
__global__ void k_fin_lt_cnt(uint32_t M, uint32_t D, const uint32_t* __restrict__ node_first, const uint32_t* __restrict__ slen,
                             const uint32_t* __restrict__ kt_cnt, uint8_t* __restrict__ fin, uint32_t* __restrict__ fc) {
    GRID_STRIDE(u, M) {
        const bool f = slen[node_first[u]] == D;
        fin[u] = f;
        fc[u] = f ? kt_cnt[u] : 0u;
    }
}
__global__ void __launch_bounds__(256) k_fin_lt(uint32_t M, const uint8_t* __restrict__ fin, const uint32_t* __restrict__ kt_pos,
                                                const uint32_t* __restrict__ kt_cnt, const uint32_t* __restrict__ ib,
                                                const uint32_t* __restrict__ ie, const uint32_t* __restrict__ foff, uint32_t* __restrict__ fend,
                                                uint32_t* __restrict__ node_occ, uint64_t abase, uint32_t* __restrict__ ab,
                                                uint32_t* __restrict__ ae) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t u = w0; u < M; u += nw) {  // (wave-uniform)
        if (!fin[u]) continue;
        const uint32_t a = kt_pos[u], n = kt_cnt[u], o = foff[u];
        uint32_t* db = ab + abase + o;
        uint32_t* de = ae + abase + o;
        unsigned long long s = 0;
        for (uint32_t t = lane; t < n; t += 64) {
            const uint32_t b = ib[a + t], e = ie[a + t];
            db[t] = b;
            de[t] = e;
            s += (unsigned long long)(e - b) + 1;
        }
        s = wave_sum(s);
        if (lane == 0) {
            fend[u] = o + n;
            node_occ[u] = (uint32_t)s;
        }
    }
}

// per node [off, end) in the sorted finisher keys
__global__ void k_fin_bounds(uint32_t F, const uint64_t* __restrict__ fk, uint32_t rowbits, uint32_t* __restrict__ foff,
                             uint32_t* __restrict__ fend) {
    GRID_STRIDE(t, F) {
        const uint32_t u = (uint32_t)(fk[t] >> rowbits);
        if (t == 0 || (uint32_t)(fk[t - 1] >> rowbits) != u) foff[u] = (uint32_t)t;
        if (t + 1 == F || (uint32_t)(fk[t + 1] >> rowbits) != u) fend[u] = (uint32_t)t + 1;
    }
}

__global__ void k_fin_archive(uint32_t F, const uint64_t* __restrict__ fk, const uint32_t* __restrict__ fv, uint64_t abase, uint32_t rowbits,
                              uint32_t* __restrict__ ab, uint32_t* __restrict__ ae) {
    GRID_STRIDE(t, F) {
        ab[abase + t] = (uint32_t)(fk[t] & ((1ull << rowbits) - 1));
        ae[abase + t] = fv[t];
    }
}

__global__ void k_finish2(uint64_t P, uint32_t D, const uint32_t* __restrict__ slen, const uint32_t* __restrict__ nid,
                          const uint32_t* __restrict__ perm, const uint32_t* __restrict__ foff, const uint32_t* __restrict__ fend,
                          const uint32_t* __restrict__ node_occ, uint64_t abase, Res* __restrict__ res) {
    GRID_STRIDE(i, P) {
        if (slen[i] != D) continue;
        const uint32_t u = nid[i];
        const uint32_t o = perm[i];
        put_res(res, o, abase + foff[u], fend[u] - foff[u], node_occ[u]);
    }
}

// group unordered items by node (deep cut-over): count, scan, scatter
__global__ void k_group_count(uint32_t n, const uint32_t* __restrict__ iu, uint32_t* __restrict__ gcnt) {
    GRID_STRIDE(i, n) atomicAdd(gcnt + iu[i], 1u);
}
__global__ void k_group_scatter(uint32_t n, const uint32_t* __restrict__ iu, const uint32_t* __restrict__ ib, const uint32_t* __restrict__ ie,
                                const uint32_t* __restrict__ goff, uint32_t* __restrict__ gfill, uint32_t* __restrict__ ob,
                                uint32_t* __restrict__ oe) {
    GRID_STRIDE(i, n) {
        const uint32_t u = iu[i];
        const uint32_t at = goff[u] + atomicAdd(gfill + u, 1u);
        ob[at] = ib[i];
        oe[at] = ie[i];
    }
}
__global__ void k_group_end(uint32_t M, const uint32_t* __restrict__ goff, const uint32_t* __restrict__ gcnt, uint32_t* __restrict__ gend) {
    GRID_STRIDE(u, M) gend[u] = goff[u] + gcnt[u];
}

// patterns holding the end-marker byte take the ordered (reference list) path
__global__ void k_has_term(uint64_t P, const uint64_t* __restrict__ off, const uint8_t* __restrict__ bytes, uint32_t* __restrict__ flag,
                           uint32_t* __restrict__ count) {
    GRID_STRIDE(i, P) {
        uint32_t f = 0;
        for (uint64_t t = off[i]; t < off[i + 1]; t++) f |= bytes[t] == '#';
        flag[i] = f;
        if (f) atomicAdd(count, 1u);
    }
}

// ------------------------------------------------------------- finishing
__global__ void k_fin_counts(uint32_t M, uint32_t D, const uint32_t* __restrict__ node_first, const uint32_t* __restrict__ slen,
                             const uint32_t* __restrict__ ioff, const uint32_t* __restrict__ iend, uint32_t* __restrict__ fcnt) {
    GRID_STRIDE(u, M) fcnt[u] = (slen[node_first[u]] == D) ? iend[u] - ioff[u] : 0u;
}

__global__ void k_archive(uint64_t n, const uint32_t* __restrict__ nu, const uint32_t* __restrict__ nb, const uint32_t* __restrict__ ne,
                          const uint32_t* __restrict__ ioff, const uint32_t* __restrict__ fcnt, const uint32_t* __restrict__ foff,
                          uint64_t abase, uint32_t* __restrict__ ab, uint32_t* __restrict__ ae, uint32_t* __restrict__ node_occ) {
    GRID_STRIDE(r, n) {
        const uint32_t u = nu[r];
        if (fcnt[u]) {
            const uint64_t d = abase + foff[u] + (r - ioff[u]);
            ab[d] = nb[r];
            ae[d] = ne[r];
            atomicAdd(node_occ + u, ne[r] - nb[r] + 1);
        }
    }
}

__global__ void k_finish(uint64_t P, uint32_t D, const uint32_t* __restrict__ slen, const uint32_t* __restrict__ nid,
                         const uint32_t* __restrict__ perm, const uint32_t* __restrict__ foff, const uint32_t* __restrict__ fcnt,
                         const uint32_t* __restrict__ node_occ, uint64_t abase,
                         Res* __restrict__ res) {
    GRID_STRIDE(i, P) {
        if (slen[i] != D) continue;
        const uint32_t u = nid[i];
        const uint32_t o = perm[i];
        put_res(res, o, abase + foff[u], fcnt[u], node_occ[u]);
    }
}

// --------------------------------------------------------------- locate
__global__ void k_u32_to_u64(const uint32_t* __restrict__ a, uint64_t n, uint64_t* __restrict__ b) { GRID_STRIDE(i, n) b[i] = a[i]; }
__global__ void k_u32_of_u64(const uint64_t* __restrict__ a, uint64_t n, uint32_t* __restrict__ b) { GRID_STRIDE(i, n) b[i] = (uint32_t)a[i]; }
// scan inputs of locate: occurrences and intervals per pattern
__global__ void k_res_scan_in(const Res* __restrict__ res, uint64_t n, uint64_t* __restrict__ occ, uint64_t* __restrict__ cnt) {
    GRID_STRIDE(i, n) {
        const Res r = res[i];
        if (cnt) {
            occ[i] = res_occ(r);
            cnt[i] = res_cnt(r);
        } else {  // one scan of both (the batch's totals stay below 2^32)
            occ[i] = (uint64_t)res_occ(r) << 32 | res_cnt(r);
        }
    }
}

// one task per finished interval: its first row, first output record and pattern; and,
// per run of kLocRun records, the task holding the run's first record (blk_first), so
// k_locate finds a record's task in LDS instead of searching all tasks
constexpr uint32_t kLocRun = 256;
__global__ void k_tasks(uint64_t P, const Res* __restrict__ res,
                        const uint64_t* __restrict__ tscan, const uint64_t* __restrict__ oscan,
                        const uint32_t* __restrict__ ab, const uint32_t* __restrict__ ae,
                        uint32_t* __restrict__ trow, uint64_t* __restrict__ tout, uint32_t* __restrict__ tpat,
                        uint64_t* __restrict__ blk_first, uint64_t occ_cap, uint64_t task_cap, uint32_t* __restrict__ oflow) {
    GRID_STRIDE(i, P) {
        // tscan null: oscan holds the packed scan (occurrences << 32 | tasks)
        const uint64_t ps = oscan[i];
        uint64_t base = tscan ? ps : ps >> 32;
        const uint64_t t0 = tscan ? tscan[i] : (ps & 0xffffffffull);
        const Res r = res[i];
        // buffers sized before the totals were read (deferred checks): a pattern whose tasks or
        // records pass them flags the batch, and the caller searches it again with exact sizes
        if (t0 + res_cnt(r) > task_cap || base + res_occ(r) > occ_cap) { atomicOr(oflow, 1u); continue; }
        const bool direct_row = (r.cnt & kResRow) != 0;
        const uint32_t n = res_cnt(r);
        for (uint32_t q = 0; q < n; q++) {
            const uint64_t a = r.off + q;
            // a text-position result has no row: k_locate takes (word, offset) from res
            const uint32_t row = (r.cnt & kResPos) ? ~0u : direct_row ? (uint32_t)r.off : ab[a];
            const uint64_t len = direct_row ? (uint64_t)res_occ(r) : (uint64_t)(ae[a] - row) + 1;
            trow[t0 + q] = row;
            tout[t0 + q] = base;
            tpat[t0 + q] = (uint32_t)i;
            for (uint64_t k = (base + kLocRun - 1) / kLocRun; k * kLocRun < base + len; k++) blk_first[k] = t0 + q;
            base += len;
        }
    }
}

// The same tasks for batches whose patterns hold long lists (C5's 8-mers: ~1.5e5 intervals each,
// which k_tasks walks one lane per pattern): one wave per pattern, its lanes striding over the
// pattern's intervals — each task's row, pattern and length; the record offsets are then one scan
// of the lengths (records follow the tasks in order) and k_blk_first finds each record block's
// first task, so no lane walks a whole list
__global__ void __launch_bounds__(256) k_tasks_wave(uint64_t P, const Res* __restrict__ res, const uint64_t* __restrict__ tscan,
                                                    const uint64_t* __restrict__ oscan, const uint32_t* __restrict__ ab,
                                                    const uint32_t* __restrict__ ae, uint32_t* __restrict__ trow,
                                                    uint64_t* __restrict__ tlen, uint32_t* __restrict__ tpat) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t i = w0; i < P; i += nw) {  // (wave-uniform)
        const uint64_t t0 = tscan ? tscan[i] : (oscan[i] & 0xffffffffull);
        const Res r = res[i];
        const uint32_t n = res_cnt(r);
        const bool direct_row = (r.cnt & kResRow) != 0;
        for (uint32_t q = lane; q < n; q += 64) {
            const uint64_t a = r.off + q;
            const uint32_t row = (r.cnt & kResPos) ? ~0u : direct_row ? (uint32_t)r.off : ab[a];
            trow[t0 + q] = row;
            tlen[t0 + q] = direct_row ? (uint64_t)res_occ(r) : (uint64_t)(ae[a] - row) + 1;
            tpat[t0 + q] = (uint32_t)i;
        }
    }
}
// blk_first[k] = the task holding record k * kLocRun (tout: the tasks' first records, ascending)
__global__ void k_blk_first(uint64_t nblk, const uint64_t* __restrict__ tout, uint64_t TT, uint64_t* __restrict__ blk_first) {
    GRID_STRIDE(k, nblk) {
        const uint64_t o = k * kLocRun;
        uint64_t lo = 0, hi = TT;  // last task with tout <= o
        while (hi - lo > 1) {
            const uint64_t mid = (lo + hi) >> 1;
            if (tout[mid] <= o) lo = mid; else hi = mid;
        }
        blk_first[k] = lo;
    }
}

// the #Pat a record reports for batch pattern i: first_id + i, or ids[i] when the caller's batch
// is a subset of its pattern file in another order (edsbwt_search_device_ids)
__device__ __forceinline__ uint32_t pat_id(const uint32_t* __restrict__ ids, uint32_t first_id, uint64_t i) {
    return ids ? ids[i] : first_id + (uint32_t)i;
}

// locate (:328-369): walk LF until L = '#'; the walk length is the offset in the
// word, the '#'-rank gives EOF_ID, the segment bitvector gives (D, S_j).
// mode 0: the reference's full walk; 1: per-row (word, offset) table; 2: walk until
// the first sampled row (offset a multiple of the sample rate) and add its stored
// (word, offset) — '#' rows have offset 0 and are always sampled.
// launched with 256-thread blocks: a block's pass covers records [o0, o0 + kLocRun), whose
// tasks (at most kLocRun + 1, from blk_first) are staged in LDS
__global__ void __launch_bounds__(256) k_locate(uint64_t OCC, uint64_t TT, const uint64_t* __restrict__ tout, const uint32_t* __restrict__ trow,
                                                const uint32_t* __restrict__ tpat, const uint64_t* __restrict__ blk_first, uint32_t first_id,
                                                const uint32_t* __restrict__ ids, KIdx X, int mode, edsbwt_occ* __restrict__ rec,
                                                unsigned long long* __restrict__ stats, const Res* __restrict__ res,
                                                const unsigned long long* __restrict__ tot_dev, const uint32_t* __restrict__ oflow) {
    // tot_dev (deferred checks): OCC and TT are the batch's totals on the device, the launch
    // arguments the buffers' capacities; nothing runs when k_tasks found them too small
    if (tot_dev) {
        if (*oflow) return;
        OCC = min(OCC, (uint64_t)tot_dev[0]);
        TT = min(TT, (uint64_t)tot_dev[1]);
    }
    unsigned long long my_steps = 0, my_off = 0;
    __shared__ uint64_t s_out[kLocRun + 1];
    __shared__ uint32_t s_row[kLocRun + 1], s_pat[kLocRun + 1];
    // the pass's kLocRun records are one contiguous 5 KB of the output (o0 is a multiple of kLocRun,
    // so its start is 16-B aligned): staged here and written as 16-B stores instead of five strided
    // 4-B stores per record from every lane
    __shared__ uint32_t s_rec[kLocRun * 5];
    uint32_t* recw = reinterpret_cast<uint32_t*>(rec);
    for (uint64_t o0 = (uint64_t)blockIdx.x * kLocRun; o0 < OCC; o0 += (uint64_t)gridDim.x * kLocRun) {  // block-uniform
        const uint64_t t0 = blk_first[o0 / kLocRun];
        if (t0 >= TT) continue;  // (block-uniform) only a batch that fails its deferred checks gets here
        const uint32_t nt = (uint32_t)min((uint64_t)kLocRun + 1, TT - t0);
        __syncthreads();  // the previous pass is done with the staged tasks and records
        for (uint32_t j = threadIdx.x; j < nt; j += blockDim.x) {
            s_out[j] = tout[t0 + j];
            s_row[j] = trow[t0 + j];
            s_pat[j] = tpat[t0 + j];
        }
        __syncthreads();
        const uint64_t o = o0 + threadIdx.x;
        // (pat, word, segment, word in segment, offset) of record o; zeros where no valid task holds it
        uint32_t q0 = 0, q1 = 0, q2 = 0, q3 = 0, q4 = 0;
        if (o < OCC) {
            uint32_t lo = 0, hi = nt;  // last staged task with s_out <= o
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_out[mid] <= o) lo = mid; else hi = mid;
            }
            const uint32_t pat = s_pat[lo];
            q0 = pat_id(ids, first_id, pat);
            if (s_row[lo] == ~0u) {  // text-position result (kResPos): (word, offset) from the pattern's result
                const Res rr = res[pat];
                q1 = (uint32_t)rr.off;
                q2 = rr.occ;
                q3 = rr.cnt & kResCnt;
                q4 = (uint32_t)(rr.off >> 32);
                my_off += q4;
            } else {
                uint32_t x = s_row[lo] + (uint32_t)(o - s_out[lo]);
                if (x >= X.N) {
                    q0 = 0;  // as above: rows of a valid task are < N
                } else if (mode == 2 && X.samp_dense) {  // every row sampled: the record straight from row x's sample
                    const uint4 s = X.samples[x];
                    q1 = s.x; q2 = s.z; q3 = s.w; q4 = s.y;
                    my_off += s.y;
                } else {
                    uint32_t word = ~0u, off = 0;
                    bool done = false;  // the record came from a sample met on the walk
                    if (mode == 1) {
                        word = X.da[x];
                        off = X.offt[x];
                    } else {
                        for (;;) {
#if EDSBWT_OCC_ROWS == 64
                            const OccV v = load_block(X.occ, x >> 6);
                            const uint32_t bit = x & 63u;
                            const uint64_t m = (1ull << bit) - 1ull;
                            if (mode == 2 && ((v.samp >> bit) & 1)) {  // (word, offset, segment, word in segment)
                                const uint4 s = X.samples[v.cnt[7] + (uint32_t)__popcll(v.samp & m)];
                                my_steps += off;
                                q1 = s.x; q2 = s.z; q3 = s.w; q4 = off + s.y;
                                done = true;
                                break;
                            }
                            const uint32_t c = (uint32_t)((v.p0 >> bit) & 1) | (uint32_t)(((v.p1 >> bit) & 1) << 1) | (uint32_t)(((v.p2 >> bit) & 1) << 2);
                            uint32_t acc = 0;
#pragma unroll
                            for (uint32_t cc = 0; cc < 8; cc++)
                                if (cc == c) acc = v.cnt[cc];
                            const uint64_t e = ((c & 1) ? v.p0 : ~v.p0) & ((c & 2) ? v.p1 : ~v.p1) & ((c & 4) ? v.p2 : ~v.p2);
                            const uint32_t rk = acc + (uint32_t)__popcll(e & m);
#else
                            uint32_t rk;
                            const uint32_t c = sym_rank(X.occ, x, &rk);
#endif
                            if (c == 0) { word = X.eof_word[rk]; my_steps += off; break; }
                            x = X.C[c] + rk;
                            off++;
                        }
                    }
                    if (!done) {
                        const uint32_t seg = X.seg_of_word[word];
                        q1 = word; q2 = seg; q3 = word - X.seg_start[seg]; q4 = off;
                    }
                    my_off += q4;
                }
            }
        }
        uint32_t* d = s_rec + threadIdx.x * 5;
        d[0] = q0; d[1] = q1; d[2] = q2; d[3] = q3; d[4] = q4;
        __syncthreads();
        // words [o0*5, (o0 + n)*5) of the output, n = the pass's records: 16-B stores and a 4-B tail
        const uint32_t n = (uint32_t)min((uint64_t)kLocRun, OCC - o0);
        const uint32_t nw = n * 5, nq = nw / 4;
        uint4* dst = reinterpret_cast<uint4*>(recw + o0 * 5);
        for (uint32_t k = threadIdx.x; k < nq; k += blockDim.x) {
            const uint32_t* s4 = s_rec + 4 * k;
            dst[k] = make_uint4(s4[0], s4[1], s4[2], s4[3]);
        }
        if (threadIdx.x < nw - nq * 4) recw[o0 * 5 + nq * 4 + threadIdx.x] = s_rec[nq * 4 + threadIdx.x];
    }
    __shared__ unsigned long long sh[4];
    stat_add(stats, ST_LOC_STEPS, my_steps, sh);
    stat_add(stats, ST_LOC_OFFSETS, my_off, sh);
}

// Locate for dense samples without tasks (the deferred direct start's results: single
// intervals, text positions, or at most kDeepWide archived intervals per pattern): one lane per
// pattern writes its records from oscan's offset; a pattern with more than kLocBig records is
// listed for k_locate_big instead (a block per pattern), so no lane walks a long run alone.
constexpr uint32_t kLocBig = 64;
__device__ __forceinline__ void put_rec(edsbwt_occ* __restrict__ rec, uint64_t o, uint32_t pat, uint32_t word, uint32_t seg, uint32_t wis,
                                        uint32_t off) {
    edsbwt_occ r;
    r.pat = pat;
    r.word = word;
    r.seg = seg;
    r.word_in_seg = wis;
    r.offset = off;
    rec[o] = r;
}
// Dense samples, the level walk's results (C5's 8-mer lists: ~1.5e5 intervals each, nearly all one row
// wide): one wave per pattern, its lanes taking 64 of the pattern's intervals at a time; a wave scan of
// their widths places each interval's records after the pattern's offset (oscan: exclusive, packed =
// occurrences << 32 | tasks or the occurrences alone), and each row's record comes straight from its
// sample — no task arrays (k_tasks / k_tasks_wave), no scan over the tasks, no per-record task search
// (k_locate).  Same records in the same order as k_tasks + k_locate.
constexpr uint32_t kLocU = 4;
__global__ void __launch_bounds__(256) k_locate_lists(uint64_t P, const Res* __restrict__ res, const uint64_t* __restrict__ oscan,
                                                      uint32_t packed, uint32_t first_id, const uint32_t* __restrict__ ids, KIdx X,
                                                      const uint32_t* __restrict__ ab, const uint32_t* __restrict__ ae,
                                                      edsbwt_occ* __restrict__ rec, unsigned long long* __restrict__ stats) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    unsigned long long my_off = 0;
    for (uint64_t i = w0; i < P; i += nw) {  // (wave-uniform)
        const Res r = res[i];
        const uint32_t occ = res_occ(r);
        if (!occ) continue;
        const uint64_t ps = oscan[i];
        uint64_t base = packed ? ps >> 32 : ps;
        const uint32_t pat = pat_id(ids, first_id, i);
        if (r.cnt & kResPos) {  // the text position itself
            if (lane == 0) {
                const uint32_t off = (uint32_t)(r.off >> 32);
                put_rec(rec, base, pat, (uint32_t)r.off, r.occ, r.cnt & kResCnt, off);
                my_off += off;
            }
            continue;
        }
        if (r.cnt & kResRow) {  // one interval [off, off + occ), not in the archive
            for (uint32_t q = lane; q < occ; q += 64) {
                const uint4 sm = X.samples[(uint32_t)r.off + q];
                put_rec(rec, base + q, pat, sm.x, sm.z, sm.w, sm.y);
                my_off += sm.y;
            }
            continue;
        }
        // kLocU rounds of 64 intervals at once (interval c0 + 64 j + lane in lane's slot j, so each load
        // instruction reads 64 neighbouring intervals, as one round would): the kLocU sample reads of a
        // lane are issued together, before any record store, and each slot's records are placed by a
        // wave scan of its widths after the previous slot's
        const uint32_t n = r.cnt & kResCnt;
        for (uint32_t c0 = 0; c0 < n; c0 += 64 * kLocU) {
            uint32_t b[kLocU], wd[kLocU];
#pragma unroll
            for (uint32_t j = 0; j < kLocU; j++) {
                const uint32_t t = c0 + 64 * j + lane;
                b[j] = 0;
                wd[j] = 0;
                if (t < n) {
                    b[j] = ab[r.off + t];
                    wd[j] = ae[r.off + t] - b[j] + 1;
                }
            }
            uint4 s0[kLocU];  // each interval's first row's sample (nearly every interval of a long list is one row wide)
#pragma unroll
            for (uint32_t j = 0; j < kLocU; j++) s0[j] = wd[j] ? X.samples[b[j]] : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (uint32_t j = 0; j < kLocU; j++) {
                uint32_t tot;
                const uint64_t o = base + wave_excl_scan(wd[j], lane, tot);
                if (wd[j]) {
                    put_rec(rec, o, pat, s0[j].x, s0[j].z, s0[j].w, s0[j].y);
                    my_off += s0[j].y;
                }
                for (uint32_t k = 1; k < wd[j]; k++) {
                    const uint4 sm = X.samples[b[j] + k];
                    put_rec(rec, o + k, pat, sm.x, sm.z, sm.w, sm.y);
                    my_off += sm.y;
                }
                base += tot;
            }
        }
    }
    __shared__ unsigned long long sh[4];
    stat_add(stats, ST_LOC_OFFSETS, my_off, sh);
}

// records of one block's 256 patterns are one contiguous range of the output: staged in LDS
// (up to kLocStage records) and written out as 16-B stores, instead of five strided 4-B stores
// per record from every lane (records of patterns left to k_locate_big, which runs next on the
// stream, are written over by it)
constexpr uint32_t kLocStage = 1024;
template <uint32_t STAGE = kLocStage, int PPT = 1>  // records staged per block (STAGE x 20 B of LDS: 1024 -> 7 blocks per CU)
__global__ void __launch_bounds__(256) k_locate_pp(uint64_t P, const Res* __restrict__ res, uint32_t* __restrict__ oscan, uint32_t first_id,
                                                   const uint32_t* __restrict__ ids, KIdx X, const uint32_t* __restrict__ ab, const uint32_t* __restrict__ ae,
                                                   edsbwt_occ* __restrict__ rec, uint64_t occ_cap, uint32_t* __restrict__ big,
                                                   uint32_t* __restrict__ oflow, unsigned long long* __restrict__ stats,
                                                   uint32_t* __restrict__ counts, const unsigned long long* __restrict__ tile_pre) {
    // counts != nullptr (the deferred per-pattern locate): each pattern's count is written here and
    // found / occurrences summed (fused counts), the scan having read the results directly.
    // tile_pre != nullptr: each 64-pattern tile's first record (k_count_tiles + a scan over tiles);
    // the offsets inside a tile come from a wave scan here, and oscan is written only for the
    // patterns k_locate_big takes
    CountSums cs;
    __shared__ uint32_t sw[STAGE * 5];
    __shared__ uint64_t s_lo, s_hi;
    __shared__ unsigned long long sh[4];
    unsigned long long my_off = 0;
    uint32_t* recw = reinterpret_cast<uint32_t*>(rec);
    // PPT patterns per thread and block-round (p0 + h * 256 + thread): their loads issued together,
    // so a round's chain of dependent loads (result, then samples) serves PPT x 256 patterns
    const uint64_t span = (uint64_t)blockDim.x * PPT;
    for (uint64_t p0 = (uint64_t)blockIdx.x * span; p0 < P; p0 += (uint64_t)gridDim.x * span) {  // block-uniform
        const uint64_t plast = min(P, p0 + span) - 1;
        Res r[PPT];
        uint32_t occ[PPT];
        uint64_t base[PPT];
#pragma unroll
        for (int h = 0; h < PPT; h++) {
            const uint64_t i = p0 + (uint64_t)h * blockDim.x + threadIdx.x;
            r[h] = Res{};
            occ[h] = 0;
            base[h] = 0;
            if (i < P) {
                r[h] = res[i];
                occ[h] = res_occ(r[h]);
                if (!tile_pre) base[h] = oscan[i];  // exclusive scan of the counts
                cs.put(counts, i, occ[h]);
            }
        }
        if (tile_pre) {  // (a uniform branch) each wave's tile: its first record + the offsets inside it
#pragma unroll
            for (int h = 0; h < PPT; h++) {
                const uint64_t w0 = p0 + (uint64_t)h * blockDim.x + (threadIdx.x & ~63u);
                const unsigned long long inw = wave_excl_scan(occ[h]);
                if (w0 < P) base[h] = tile_pre[w0 >> 6] + inw;
            }
        }
        if (threadIdx.x == 0) s_lo = base[0];
#pragma unroll
        for (int h = 0; h < PPT; h++)
            if (p0 + (uint64_t)h * blockDim.x + threadIdx.x == plast) s_hi = base[h] + occ[h];
        __syncthreads();
        const uint64_t lo = s_lo, hi = min(s_hi, occ_cap);
        const bool stage = hi >= lo && hi - lo <= STAGE;
        auto emit = [&](uint64_t o, uint32_t pat, uint32_t word, uint32_t seg, uint32_t wis, uint32_t off) {
            if (stage) {
                uint32_t* d = sw + (o - lo) * 5;
                d[0] = pat; d[1] = word; d[2] = seg; d[3] = wis; d[4] = off;
            } else {
                put_rec(rec, o, pat, word, seg, wis, off);
            }
        };
#pragma unroll
        for (int h = 0; h < PPT; h++) {
            const uint64_t i = p0 + (uint64_t)h * blockDim.x + threadIdx.x;
            if (i < P && occ[h]) {
                const uint32_t pat = pat_id(ids, first_id, i);
                if (base[h] + occ[h] > occ_cap) {
                    atomicOr(oflow, 1u);
                } else if (r[h].cnt & kResPos) {
                    const uint32_t off = (uint32_t)(r[h].off >> 32);
                    emit(base[h], pat, (uint32_t)r[h].off, r[h].occ, r[h].cnt & kResCnt, off);
                    my_off += off;
                } else if (occ[h] > kLocBig) {
                    if (tile_pre) oscan[i] = (uint32_t)base[h];  // (< occ_cap < 2^32) k_locate_big's offset
                    flag_push(big, (uint32_t)i);
                } else {
                    uint64_t o = base[h];
                    const uint32_t n = (r[h].cnt & kResRow) ? 1u : (r[h].cnt & kResCnt);
                    for (uint32_t t = 0; t < n; t++) {
                        const uint32_t b = (r[h].cnt & kResRow) ? (uint32_t)r[h].off : ab[r[h].off + t];
                        const uint32_t e = (r[h].cnt & kResRow) ? (uint32_t)r[h].off + occ[h] - 1 : ae[r[h].off + t];
                        for (uint32_t x = b; x <= e; x++, o++) {
                            const uint4 sm = X.samples[x];
                            emit(o, pat, sm.x, sm.z, sm.w, sm.y);
                            my_off += sm.y;
                        }
                    }
                }
            }
        }
        __syncthreads();
        if (stage && hi > lo) {
            // words [lo*5, hi*5) of the output: 4-B stores up to a 16-B boundary, 16-B stores, 4-B tail
            const uint64_t g0 = lo * 5, nw = (hi - lo) * 5;
            const uint32_t head = (uint32_t)min<uint64_t>(nw, (4u - (uint32_t)(g0 & 3u)) & 3u);
            const uint64_t nq = (nw - head) / 4;
            if (threadIdx.x < head) recw[g0 + threadIdx.x] = sw[threadIdx.x];
            uint4* dst = reinterpret_cast<uint4*>(recw + g0 + head);
            for (uint64_t q = threadIdx.x; q < nq; q += blockDim.x) {
                const uint32_t* s4 = sw + head + 4 * q;
                dst[q] = make_uint4(s4[0], s4[1], s4[2], s4[3]);
            }
            const uint64_t t0 = head + nq * 4;
            if (threadIdx.x < nw - t0) recw[g0 + t0 + threadIdx.x] = sw[t0 + threadIdx.x];
        }
        __syncthreads();
    }
    stat_add(stats, ST_LOC_OFFSETS, my_off, sh);
    cs.flush(counts, stats, sh);
}
__global__ void __launch_bounds__(256) k_locate_big(const uint32_t* __restrict__ big, const Res* __restrict__ res,
                                                    const uint32_t* __restrict__ oscan, uint32_t first_id, const uint32_t* __restrict__ ids,
                                                    KIdx X, const uint32_t* __restrict__ ab, const uint32_t* __restrict__ ae,
                                                    edsbwt_occ* __restrict__ rec, unsigned long long* __restrict__ stats) {
    unsigned long long my_off = 0;
    const uint32_t nbig = big[0];
    for (uint32_t j = blockIdx.x; j < nbig; j += gridDim.x) {  // block-uniform
        const uint32_t i = big[1 + j];
        const Res r = res[i];
        const uint32_t occ = res_occ(r), pat = pat_id(ids, first_id, i);
        const uint64_t base = oscan[i];
        const uint32_t n = (r.cnt & kResRow) ? 1u : (r.cnt & kResCnt);
        uint64_t start = 0;
        for (uint32_t t = 0; t < n; t++) {
            const uint32_t b = (r.cnt & kResRow) ? (uint32_t)r.off : ab[r.off + t];
            const uint32_t e = (r.cnt & kResRow) ? (uint32_t)r.off + occ - 1 : ae[r.off + t];
            for (uint32_t q = threadIdx.x; q <= e - b; q += blockDim.x) {
                const uint4 sm = X.samples[b + q];
                put_rec(rec, base + start + q, pat, sm.x, sm.z, sm.w, sm.y);
                my_off += sm.y;
            }
            start += (uint64_t)(e - b) + 1;
        }
    }
    __shared__ unsigned long long sh[4];
    stat_add(stats, ST_LOC_OFFSETS, my_off, sh);
}

// ---------------------------------------------- locate samples (index open)
#if EDSBWT_OCC_ROWS == 64
// per 64-row block: the sampled-row plane (offset % 2^shift == 0) and its count
__global__ void k_samp_blocks(uint64_t nblk, uint32_t N, const uint32_t* __restrict__ offt, uint32_t shift, OccBlock* __restrict__ occ,
                              uint32_t* __restrict__ bcnt) {
    GRID_STRIDE(b, nblk) {
        uint64_t p = 0;
        for (uint32_t r = 0; r < 64; r++) {
            const uint64_t x = b * 64 + r;
            if (x < N && (offt[x] & ((1u << shift) - 1)) == 0) p |= 1ull << r;
        }
        occ[b].samp = p;
        bcnt[b] = (uint32_t)__popcll(p);
    }
}

__global__ void k_samp_fill(uint64_t nblk, uint32_t N, const uint32_t* __restrict__ da, const uint32_t* __restrict__ offt,
                            const uint32_t* __restrict__ bbase, const uint32_t* __restrict__ seg_of_word,
                            const uint32_t* __restrict__ seg_start, OccBlock* __restrict__ occ, uint4* __restrict__ samples) {
    GRID_STRIDE(b, nblk) {
        uint32_t at = bbase[b];
        occ[b].cnt[7] = at;
        const uint64_t p = occ[b].samp;
        for (uint32_t r = 0; r < 64; r++)
            if ((p >> r) & 1) {
                const uint64_t x = b * 64 + r;
                const uint32_t w = da[x], sg = seg_of_word[w];
                samples[at++] = make_uint4(w, offt[x], sg, w - seg_start[sg]);
            }
    }
}
#endif

// Legacy output order (findMultipleDollarsBackward, EDSBWTsearch.cpp:300-610): for one
// pattern, round r outputs the '#' rows reached after r LF steps, rounds ascending, and
// inside a round the intervals are sorted by row, so a record's position is (offset,
// '#'-row rank of its word).  Records arrive pattern-major: a stable sort by that key
// then a stable sort by pattern gives the order.
__global__ void k_legacy_keys(uint64_t n, const edsbwt_occ* __restrict__ rec, const uint32_t* __restrict__ kpos, uint32_t kbits,
                              uint64_t* __restrict__ key, uint32_t* __restrict__ pat, uint32_t* __restrict__ idx) {
    GRID_STRIDE(i, n) {
        const edsbwt_occ r = rec[i];
        key[i] = ((uint64_t)r.offset << kbits) | kpos[r.word];
        pat[i] = r.pat;
        idx[i] = (uint32_t)i;
    }
}

__global__ void k_gather_u32(const uint32_t* __restrict__ src, const uint32_t* __restrict__ idx, uint64_t n, uint32_t* __restrict__ out) {
    GRID_STRIDE(i, n) out[i] = src[idx[i]];
}

__global__ void k_gather_rec(uint64_t n, const uint32_t* __restrict__ idx, const edsbwt_occ* __restrict__ in, edsbwt_occ* __restrict__ out) {
    GRID_STRIDE(i, n) out[i] = in[idx[i]];
}

// ------------------------------------------------- DA/OFF table (index open)
// ------------------------------------------------------------ pair blocks (index open)
// pair code of every row (kernels.h rank entries); 31 for the padding rows past N
__global__ void k_pair_codes(uint64_t nrows, KIdx X, uint8_t* __restrict__ code) {
    GRID_STRIDE(x, nrows) {
        uint32_t k = 31;
        if (x < X.N) {
            uint32_t r;
            const uint32_t c1 = sym_rank(X.occ, (uint32_t)x, &r);
            if (c1 == 0) {
                k = 0;
            } else {
                uint32_t r2;
                const uint32_t c2 = sym_rank(X.occ, X.C[c1] + r, &r2);  // L[LF(x)]
                k = 1 + (c1 - 1) * X.sigma + c2;
            }
        }
        code[x] = (uint8_t)k;
    }
}

// rank of every symbol at every pile start: out[c1 * sigma + c2] = rank_c2(L, C[c1])
__global__ void k_pile_ranks(KIdx X, uint32_t* __restrict__ out) {
    if (blockIdx.x == 0 && threadIdx.x == 0)
        for (uint32_t c1 = 0; c1 < X.sigma; c1++) {
            uint32_t r[8];
            rank_all(X.occ, X.C[c1], X.sigma, r);
            for (uint32_t c2 = 0; c2 < X.sigma; c2++) out[c1 * X.sigma + c2] = r[c2];
        }
}

// one wave per 64-row block: rows of each code, code-major ([k * nblk + blk])
__global__ void k_pair_counts(uint64_t nblk, const uint8_t* __restrict__ code, uint32_t nc, uint32_t* __restrict__ cnt) {
    GRID_STRIDE(t, nblk * 64) {  // wave-uniform: nblk * 64 and the stride are multiples of 64
        const uint64_t blk = t >> 6;
        const uint32_t lane = (uint32_t)(t & 63), k = code[t];
        for (uint32_t j = 0; j < nc; j++) {
            const uint32_t n = (uint32_t)__popcll(__ballot(k == j));
            if (lane == (j & 63u)) cnt[(size_t)j * nblk + blk] = n;
        }
    }
}

// rank entries over 32-row blocks (kernels.h): one thread per block
__global__ void k_rent1(uint64_t nb32, KIdx X, uint4* __restrict__ rent1) {
    GRID_STRIDE(k, nb32) {
        const uint32_t x0 = (uint32_t)(k * 32);
        uint32_t r[8];
        rank_all(X.occ, x0, X.sigma, r);
        const OccV v = load_block(X.occ, x0 >> 6);
        const uint32_t sh = (uint32_t)(k & 1) * 32;
        uint32_t m[8];
#pragma unroll
        for (uint32_t c = 0; c < 8; c++)
            m[c] = (uint32_t)((((c & 1) ? v.p0 : ~v.p0) & ((c & 2) ? v.p1 : ~v.p1) & ((c & 4) ? v.p2 : ~v.p2)) >> sh);
        for (uint32_t c = 0; c < X.sigma; c++) {
            uint32_t rc = 0, mc = 0;
#pragma unroll
            for (uint32_t t = 0; t < 8; t++)
                if (t == c) { rc = r[t]; mc = m[t]; }
            rent1[k * X.sigma + c] = make_uint4(rc, mc, r[0], m[0]);
        }
    }
}

// rows of pair code j in the 32 codes w[0..3] (8 per word) as a bit mask
__device__ __forceinline__ uint32_t code_mask32(const uint64_t* w, uint32_t j) {
    uint32_t m = 0;
#pragma unroll
    for (uint32_t t = 0; t < 32; t++) m |= (uint32_t)(((w[t >> 3] >> (8 * (t & 7))) & 0xffu) == j) << t;
    return m;
}
// scan = scan_u32 of k_pair_counts' code-major 64-row counts (scan[0] = 0)
__global__ void k_rent2(uint64_t nb32, uint64_t nblk, const uint8_t* __restrict__ code, uint32_t nc, uint32_t sigma,
                        const uint32_t* __restrict__ scan, uint4* __restrict__ rent2) {
    GRID_STRIDE(k, nb32) {
        const uint64_t blk = k >> 1;
        const bool odd = (k & 1) != 0;
        const uint64_t* cw = reinterpret_cast<const uint64_t*>(code + blk * 64);
        uint64_t lo[4], hi[4];
#pragma unroll
        for (int t = 0; t < 4; t++) { lo[t] = cw[t]; hi[t] = cw[4 + t]; }
        const uint64_t* w = odd ? hi : lo;
        auto rank_at = [&](uint32_t j) -> uint32_t {
            uint32_t r = scan[(size_t)j * nblk + blk] - scan[(size_t)j * nblk];
            if (odd) r += (uint32_t)__popc(code_mask32(lo, j));
            return r;
        };
        const uint32_t r0 = rank_at(0), m0 = code_mask32(w, 0);
        for (uint32_t c1 = 1; c1 < sigma; c1++) {
            const uint32_t q = 1 + (c1 - 1) * sigma;
            const uint32_t rh = r0 + rank_at(q), mh = m0 | code_mask32(w, q);
            for (uint32_t c2 = 0; c2 < sigma; c2++) {
                const uint32_t p = q + c2;
                rent2[k * (nc - 1) + p - 1] = make_uint4(rank_at(p), code_mask32(w, p), rh, mh);
            }
        }
    }
}

// triple code of every row: 0 for '#'; else 1 + (c1-1)*sigma^2 + c2*sigma + c3 with c1 = L[x],
// c2 = L[LF(x)], c3 = L[LF^2(x)] (c3 = 0 when c2 = '#'); 255 for the padding rows past N
__global__ void k_triple_codes(uint64_t nrows, KIdx X, uint8_t* __restrict__ code) {
    GRID_STRIDE(x, nrows) {
        uint32_t k = 255;
        if (x < X.N) {
            uint32_t r;
            const uint32_t c1 = sym_rank(X.occ, (uint32_t)x, &r);
            if (c1 == 0) {
                k = 0;
            } else {
                uint32_t r2, r3;
                const uint32_t c2 = sym_rank(X.occ, X.C[c1] + r, &r2);
                const uint32_t c3 = c2 == 0 ? 0u : sym_rank(X.occ, X.C[c2] + r2, &r3);
                k = 1 + (c1 - 1) * X.sigma * X.sigma + c2 * X.sigma + c3;
            }
        }
        code[x] = (uint8_t)k;
    }
}

// rank of every symbol at n given rows: out[i * sigma + c]
__global__ void k_ranks_at(uint32_t n, const uint32_t* __restrict__ rows, KIdx X, uint32_t* __restrict__ out) {
    GRID_STRIDE(i, n) {
        uint32_t r[8];
        rank_all(X.occ, rows[i], X.sigma, r);
        for (uint32_t c = 0; c < X.sigma; c++) out[i * X.sigma + c] = r[c];
    }
}

// three-step rank entries (kernels.h rent3) from k_triple_codes' scanned 64-row counts
__global__ void k_rent3(uint64_t nb32, uint64_t nblk, const uint8_t* __restrict__ code, uint32_t sigma, const uint32_t* __restrict__ scan,
                        uint4* __restrict__ rent3) {
    GRID_STRIDE(k, nb32) {
        const uint64_t blk = k >> 1;
        const bool odd = (k & 1) != 0;
        const uint64_t* cw = reinterpret_cast<const uint64_t*>(code + blk * 64);
        uint64_t lo[4], hi[4];
#pragma unroll
        for (int t = 0; t < 4; t++) { lo[t] = cw[t]; hi[t] = cw[4 + t]; }
        const uint64_t* w = odd ? hi : lo;
        auto rank_at = [&](uint32_t j) -> uint32_t {
            uint32_t r = scan[(size_t)j * nblk + blk] - scan[(size_t)j * nblk];
            if (odd) r += (uint32_t)__popc(code_mask32(lo, j));
            return r;
        };
        const uint32_t B = sigma - 1, s2 = sigma * sigma;
        const uint32_t r0 = rank_at(0), m0 = code_mask32(w, 0);
        for (uint32_t c1 = 1; c1 < sigma; c1++) {
            const uint32_t s1 = 1 + (c1 - 1) * s2;  // (c1, '#')
            const uint32_t ra = r0 + rank_at(s1), ma = m0 | code_mask32(w, s1);
            for (uint32_t c2 = 1; c2 < sigma; c2++) {
                const uint32_t sc = s1 + c2 * sigma;  // (c1, c2, '#')
                const uint32_t rs = ra + rank_at(sc), ms = ma | code_mask32(w, sc);
                for (uint32_t c3 = 1; c3 < sigma; c3++) {
                    const uint32_t p = sc + c3;
                    rent3[k * B * B * B + ((c1 - 1) * B + (c2 - 1)) * B + (c3 - 1)] = make_uint4(rank_at(p), code_mask32(w, p), rs, ms);
                }
            }
        }
    }
}


// For every word w, walk LF from row w (its '#'-suffix) to the row with L='#'
// (position 0): rows visited get DA = w and their distance from the word end.
// segment link table (index open): for s >= 2 the c-ranks at both ends of the words of
// segments [seg_lo[s], s-1] (the range link() adds for a word of s, :533-561, :620)
// all-symbol rank entries (kernels.h rk16), from the 64-row occ blocks: entry k = rows 16k..16k+15
// of block k >> 2; its counts relative to the superblock start (block (k >> 12) << 10)
__device__ __forceinline__ uint64_t occ_match(const OccV& v, uint32_t c) {
    return ((c & 1) ? v.p0 : ~v.p0) & ((c & 2) ? v.p1 : ~v.p1) & ((c & 4) ? v.p2 : ~v.p2);
}
__global__ void k_rk16(uint64_t n16, KIdx X, uint4* __restrict__ out) {
    GRID_STRIDE(k, n16) {
        const OccV v = load_block(X.occ, (uint32_t)(k >> 2));
        const OccV s = load_block(X.occ, (uint32_t)((k >> 12) << 10));
        const uint32_t sh = (uint32_t)(k & 3) * 16u;
        const uint64_t below = sh ? (1ull << sh) - 1ull : 0ull;
        uint32_t c[5];
#pragma unroll
        for (uint32_t q = 1; q <= 4; q++) c[q] = v.cnt[q] + (uint32_t)__popcll(occ_match(v, q) & below) - s.cnt[q];
        out[k] = make_uint4(c[1] | (c[2] << 16), c[3] | (c[4] << 16),
                            (uint32_t)((v.p0 >> sh) & 0xFFFFu) | ((uint32_t)((v.p1 >> sh) & 0xFFFFu) << 16),
                            (uint32_t)((v.p2 >> sh) & 0xFFFFu));
    }
}
__global__ void k_rk16_sup(uint64_t nsup, KIdx X, uint4* __restrict__ out) {
    GRID_STRIDE(s, nsup) {
        const OccV v = load_block(X.occ, (uint32_t)(s << 10));
        out[s] = make_uint4(v.cnt[1], v.cnt[2], v.cnt[3], v.cnt[4]);
    }
}

__global__ void k_segtab(uint32_t S, KIdx X, uint32_t* __restrict__ tab) {
    GRID_STRIDE(s, (size_t)S + 2) {
        uint32_t* e = tab + s * X.seg_stride;
        uint32_t r0[8], r1[8];
        const uint32_t lo = X.seg_lo[s];
        if (s >= 2) {
            rank_all(X.occ, X.seg_start[lo], X.sigma, r0);
            rank_all(X.occ, X.seg_start[s], X.sigma, r1);
        } else {
#pragma unroll
            for (int c = 0; c < 8; c++) r0[c] = r1[c] = 0;
        }
        e[0] = lo;
        for (uint32_t c = 0; c < X.sigma; c++) {
            e[1 + c] = r0[c];
            e[X.seg_hi + c] = r1[c];
        }
    }
}

// KIdx::seglink (k_deep_direct's links): per segment s and c = 1..4, the segment link table's ranks
// and, when they give one row, that row's srow entry (sample, and the 32 reversed-text characters
// before its suffix); one 128-B line per segment
__global__ void k_seglink(uint32_t S, KIdx X, uint4* __restrict__ out) {
    GRID_STRIDE(t, ((size_t)S + 2) * 4) {
        const size_t s = t >> 2;
        const uint32_t c = (uint32_t)(t & 3) + 1;
        const uint32_t* et = X.segtab + s * X.seg_stride;
        const uint32_t rx = et[1 + c], ry = et[X.seg_hi + c];
        uint4 a = make_uint4(rx, ry, 0, 0), b = make_uint4(0, 0, 0, 0);
        if (ry == rx + 1 && X.srow) {
            const size_t row = (size_t)X.C[c] + rx;
            const uint4 s0 = X.srow[2 * row], s1 = X.srow[2 * row + 1];
            a.z = s0.x;
            a.w = s0.y;
            b = make_uint4(s0.z, s0.w, s1.z, s1.w);
        }
        out[2 * t] = a;
        out[2 * t + 1] = b;
    }
}

// per-'#'-row link rows (KIdx::eofrow): the segment link table's row of eof_seg[k], its segment in [15]
__global__ void k_eofrow(uint32_t W, const uint32_t* __restrict__ eof_seg, const uint32_t* __restrict__ segtab, uint32_t stride,
                         uint32_t* __restrict__ out) {
    GRID_STRIDE(t, (size_t)W * 16) {
        const size_t k = t >> 4;
        const uint32_t j = (uint32_t)(t & 15), s = eof_seg[k];
        out[t] = j == 15 ? s : segtab[(size_t)s * stride + j];
    }
}

// KIdx::segtext: per segment s, for c = 1..4, the text item of the one word of [seg_lo[s], s - 1]
// whose last character is c (its row is LF of the word's '#' row w: C[c] + rank_c(L, w)), from that
// row's srow entry as k_lvl_items would convert it: kTextItem | offset << 27 | segment, and the
// 15 characters before the row (2 bits each) | its segment's chain bit << 31; 0 when no or several
// words end with c, or the word is longer than 16
constexpr uint32_t kSegTextWords = 64;
__global__ void k_segtext(uint32_t S, KIdx X, uint32_t* __restrict__ tab) {
    GRID_STRIDE(s, (size_t)S + 2) {
        uint32_t* e = tab + s * X.seg_stride + 16;
        uint32_t cnt[5] = {0, 0, 0, 0, 0}, row[5] = {0, 0, 0, 0, 0};
        // segments 2..S only (row S + 1 is the table's sentinel), and links of at most
        // kSegTextWords words (a longer empty-word chain keeps the row path)
        const uint32_t lo = (s >= 2 && s <= S) ? X.seg_lo[s] : 0u;
        const uint32_t w0 = (s >= 2 && s <= S) ? X.seg_start[lo] : 0u, w1 = (s >= 2 && s <= S) ? X.seg_start[s] : 0u;
        if (w1 - w0 <= kSegTextWords) {
            for (uint32_t w = w0; w < w1; w++) {
                uint32_t rk;
                const uint32_t c = sym_rank(X.occ, w, &rk);
                if (c >= 1 && c <= 4) {
                    cnt[c]++;
                    row[c] = X.C[c] + rk;
                }
            }
        }
#pragma unroll
        for (uint32_t c = 1; c <= 4; c++) {
            uint32_t b = 0, f = 0;
            if (cnt[c] == 1) {
                const uint4 s0 = X.srow[2 * (size_t)row[c]], s1 = X.srow[2 * (size_t)row[c] + 1];
                if (s0.y <= 15 && s0.z < kTextSeg) {
                    b = kTextItem | (s0.y << 27) | s0.z;
                    f = (s1.z & 0x7fffffffu) | ((s1.y & 1u) << 31);
                }
            }
            e[2 * (c - 1)] = b;
            e[2 * (c - 1) + 1] = f;
        }
    }
}

__global__ void k_table_walk(uint32_t W, KIdx X, uint32_t* __restrict__ da, uint32_t* __restrict__ dist, uint32_t* __restrict__ wlen) {
    GRID_STRIDE(w, W) {
        uint32_t x = (uint32_t)w, t = 0;
        da[x] = (uint32_t)w;
        dist[x] = 0;
        for (;;) {
            uint32_t rk;
            const uint32_t c = sym_rank(X.occ, x, &rk);
            if (c == 0) break;
            x = X.C[c] + rk;
            t++;
            da[x] = (uint32_t)w;
            dist[x] = t;
        }
        wlen[w] = t;
    }
}

__global__ void k_table_finish(uint32_t N, const uint32_t* __restrict__ da, const uint32_t* __restrict__ wlen, uint32_t* __restrict__ off) {
    GRID_STRIDE(x, N) off[x] = wlen[da[x]] - off[x];
}
// text of the words from the per-row table (index open): row x is position (w, o) = (da[x],
// offt[x]); gpos[x] = wstart[w] + o; L[x] is the character at (w, o - 1) when o > 0, stored
// at reversed index tlen - gpos[x]; the row with o = 0 is the word's whole-word suffix
__global__ void k_text_build(uint32_t N, KIdx X, const uint32_t* __restrict__ da, const uint32_t* __restrict__ offt,
                             const uint32_t* __restrict__ wstart, uint64_t tlen, uint32_t* __restrict__ gpos,
                             uint32_t* __restrict__ wrow, uint32_t* __restrict__ rt32) {
    GRID_STRIDE(x, N) {
        const uint32_t w = da[x], o = offt[x];
        const uint32_t g = wstart[w] + o;
        gpos[x] = g;
        if (o == 0) {
            wrow[w] = (uint32_t)x;
        } else {
            uint32_t rk;
            const uint32_t c = sym_rank(X.occ, (uint32_t)x, &rk);
            const uint64_t r = tlen - g;
            atomicOr(rt32 + (r >> 4), (uint32_t)((c - 1u) & 3u) << (2u * (uint32_t)(r & 15u)));
        }
    }
}

// launched with a small grid (kReduceBlocks): one atomic per block
__global__ void __launch_bounds__(256) k_count_found(const Res* __restrict__ res, uint64_t P, uint32_t* __restrict__ counts,
                                                     unsigned long long* __restrict__ found, unsigned long long* __restrict__ sums,
                                                     uint64_t* __restrict__ scan_in) {
    // scan_in (locate): the packed scan input occurrences << 32 | tasks, in the same pass
    __shared__ unsigned long long sh[4];
    unsigned long long f = 0, so = 0, st = 0;
    GRID_STRIDE(i, P) {
        const Res r = res[i];
        const uint32_t oc = res_occ(r);
        counts[i] = oc;  // backwardSearch's return value per pattern
        if (scan_in) scan_in[i] = (uint64_t)oc << 32 | res_cnt(r);
        f += oc > 0;
        so += oc;
        st += res_cnt(r);
    }
    f = block_sum(f, sh);
    so = block_sum(so, sh);
    st = block_sum(st, sh);
    if (threadIdx.x == 0) {
        if (f) atomicAdd(found, f);
        if (so) atomicAdd(sums, so);
        if (st) atomicAdd(sums + 1, st);
    }
}

// the per-pattern locate's counts pass: k_count_found's counts and totals, and the occurrence sum
// of each 64-pattern tile (one wave of k_locate_pp), whose exclusive scan gives every tile its
// first record — a scan over tiles instead of over patterns (C3: 156K entries against 10M), and
// no block barrier per tile (wave shuffles)
// wbits != nullptr (engine.hip run_deep: this pass runs beside k_deep_wave, on a second stream):
// the patterns k_deep_wave still walks are marked there (k_mark_wide, by output index) and left
// out — neither their results nor their counts are read or written here; k_tile_fix adds them once
// both kernels are done.  Each marked word is cleared after it is read (the bitmap is zero again
// for the next search): a word's two readers are lanes of one wave, and the store depends on the
// loaded value, so it follows the loads.
__global__ void __launch_bounds__(256) k_count_tiles(const Res* __restrict__ res, uint64_t P, uint32_t* __restrict__ counts,
                                                     unsigned long long* __restrict__ stats, unsigned long long* __restrict__ tile_sum,
                                                     uint32_t* __restrict__ wbits) {
    // (a grid of up to 16384 blocks: the found / occurrence sums go to the sharded stats, folded by
    // k_gather_checks — the deferred path of this pass checks no interval total)
    __shared__ unsigned long long sh[4];
    CountSums cs;
    for (uint64_t p0 = (uint64_t)blockIdx.x * blockDim.x; p0 < P; p0 += (uint64_t)gridDim.x * blockDim.x) {  // block-uniform
        const uint64_t i = p0 + threadIdx.x;
        uint32_t oc = 0;
        if (i < P) {
            const uint32_t wb = wbits ? wbits[i >> 5] : 0u;
            if (!((wb >> (i & 31)) & 1u)) {
                oc = res_occ(res[i]);
                cs.put(counts, i, oc);
            }
            if (wb && (i & 31) == 0) wbits[i >> 5] = 0u;
        }
        const unsigned long long t = wave_sum(oc);
        if ((threadIdx.x & 63) == 0 && i < P) tile_sum[i >> 6] = t;  // (p0 is a multiple of 64)
    }
    cs.flush(counts, stats, sh);
}

// the patterns k_deep_wave walks (its list: count at ovf[0], queue indices after it, at most cap of
// them), marked by output index for k_count_tiles running beside it
__global__ void k_mark_wide(const uint32_t* __restrict__ ovf, uint32_t cap, const uint32_t* __restrict__ perm, uint32_t* __restrict__ wbits) {
    const uint32_t n = min(ovf[0], cap);
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
        const uint32_t o = perm[ovf[1 + j]];
        atomicOr(&wbits[o >> 5], 1u << (o & 31));
    }
}

// after k_count_tiles (without the marked patterns) and k_deep_wave: the walked patterns' counts into
// the caller's array, their occurrences into their tiles' sums and into the fused sums
__global__ void __launch_bounds__(256) k_tile_fix(const uint32_t* __restrict__ ovf, uint32_t cap, const uint32_t* __restrict__ perm,
                                                  const Res* __restrict__ res, uint32_t* __restrict__ counts,
                                                  unsigned long long* __restrict__ stats, unsigned long long* __restrict__ tile_sum) {
    __shared__ unsigned long long sh[4];
    CountSums cs;
    const uint32_t n = min(ovf[0], cap);
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
        const uint32_t o = perm[ovf[1 + j]];
        const uint32_t oc = res_occ(res[o]);
        cs.put(counts, o, oc);
        if (oc) atomicAdd(&tile_sum[o >> 6], (unsigned long long)oc);
    }
    cs.flush(counts, stats, sh);
}

// the same tile sums from the counts the deep kernels wrote (fused counts on a located search):
// 4 B per pattern read instead of the 16-B result, nothing else written
__global__ void __launch_bounds__(256) k_tile_sums(const uint32_t* __restrict__ counts, uint64_t P, unsigned long long* __restrict__ tile_sum) {
    for (uint64_t p0 = (uint64_t)blockIdx.x * blockDim.x; p0 < P; p0 += (uint64_t)gridDim.x * blockDim.x) {  // block-uniform
        const uint64_t i = p0 + threadIdx.x;
        const uint32_t oc = i < P ? counts[i] : 0u;
        const unsigned long long t = wave_sum(oc);
        if ((threadIdx.x & 63) == 0 && i < P) tile_sum[i >> 6] = t;  // (p0 is a multiple of 64)
    }
}

// per depth D: trie nodes M_D = #{i : lcp[i] < D <= slen[i]} (difference array over D)
// and patterns per length, in one pass (LDS bins, Lmax < 1023)
__global__ void __launch_bounds__(256) k_trie_counts(const uint32_t* __restrict__ slen, const uint32_t* __restrict__ lcp, uint64_t P,
                                                     uint32_t Lmax, unsigned long long* __restrict__ diff, unsigned long long* __restrict__ hist) {
    __shared__ unsigned int sd[1024], sh[1024];
    const uint32_t nb = Lmax + 2;
    for (uint32_t t = threadIdx.x; t < nb; t += blockDim.x) sd[t] = sh[t] = 0;
    __syncthreads();
    GRID_STRIDE(i, P) {
        const uint32_t l = slen[i], c = lcp[i];
        atomicAdd(&sh[l], 1u);
        if (c < l) {
            atomicAdd(&sd[c + 1], 1u);
            atomicSub(&sd[l + 1], 1u);
        }
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < nb; t += blockDim.x) {
        if (sd[t]) atomicAdd(diff + t, (unsigned long long)(int)sd[t]);
        if (sh[t]) atomicAdd(hist + t, (unsigned long long)sh[t]);
    }
}

__global__ void k_trie_counts_global(const uint32_t* __restrict__ slen, const uint32_t* __restrict__ lcp, uint64_t P,
                                     unsigned long long* __restrict__ diff, unsigned long long* __restrict__ hist) {
    GRID_STRIDE(i, P) {
        const uint32_t l = slen[i], c = lcp[i];
        atomicAdd(hist + l, 1ull);
        if (c < l) {
            atomicAdd(diff + c + 1, 1ull);
            atomicAdd(diff + l + 1, ~0ull);  // -1 mod 2^64
        }
    }
}

// zero up to four buffers in one launch
__global__ void k_zero4(uint32_t* __restrict__ a, uint64_t na, uint32_t* __restrict__ b, uint64_t nb, uint32_t* __restrict__ c, uint64_t nc,
                        uint32_t* __restrict__ d, uint64_t nd) {
    const uint64_t n = na + nb + nc + nd;
    GRID_STRIDE(i, n) {
        if (i < na) a[i] = 0;
        else if (i < na + nb) b[i - na] = 0;
        else if (i < na + nb + nc) c[i - na - nb] = 0;
        else d[i - na - nb - nc] = 0;
    }
}

__global__ void k_fill_u32(uint32_t* __restrict__ a, uint64_t n, uint32_t v) { GRID_STRIDE(i, n) a[i] = v; }

// ------------------------------------------------------- k-mer start table
// The order-free walk's state after D characters is a function of those D characters
// alone, so the index keeps it for every D-mer over the B = sigma-1
// non-'#' symbols and a search starts at depth D.  A D-mer's index has its LAST
// character as the least significant base-B digit (digit = code - 1).

// every K-mer as a pattern: pattern i spells i's base-B digits, last character = digit 0
// (so i mod B^D is the index of its last D characters); sym[v] = byte of code v + 1
// (mul, add): pattern i spells x = i * mul + add instead (the level table's groups: every K-mer
// whose last characters are those of `add`)
__global__ void k_kmer_batch(uint64_t P, uint32_t K, uint32_t B, uint64_t sym, uint8_t* __restrict__ bytes, uint64_t* __restrict__ off,
                             uint64_t mul, uint64_t add) {
    GRID_STRIDE(i, P) {
        uint64_t x = i * mul + add;
        for (uint32_t t = 0; t < K; t++) {
            bytes[i * K + (K - 1 - t)] = (uint8_t)(sym >> (8 * (x % B)));
            x /= B;
        }
        off[i] = i * K;
        if (i + 1 == P) off[P] = P * K;
    }
}

// captured items: node id at depth D -> index of the node's D-mer (from its first pattern's id)
__global__ void k_ktab_capture_map(uint64_t n, uint32_t* __restrict__ u, const uint32_t* __restrict__ node_first, const uint32_t* __restrict__ perm,
                                   uint64_t BD) {
    GRID_STRIDE(t, n) u[t] = (uint32_t)(perm[node_first[u[t]]] % BD);
}

__global__ void k_ktab_keys(uint64_t n, const uint32_t* __restrict__ km, const uint32_t* __restrict__ b, uint64_t* __restrict__ key) {
    GRID_STRIDE(t, n) key[t] = (uint64_t)km[t] << 32 | b[t];
}

// the k-mer start table built group by group (engine.hip build_ktab_grouped): group g holds the
// D-mers x = xl * G + g (the D-mers sharing their last two characters) with its own offsets
// goff[g * (EG + 1) + xl] into its lists pb[g] / pe[g].  len[x] = D-mer x's list length; then each
// D-mer's list copied to the table's layout at off[x] (the exclusive scan of len)
__global__ void k_ktab_group_lens(uint64_t E, uint32_t G, uint64_t EG, const uint32_t* __restrict__ goff, uint32_t* __restrict__ len) {
    GRID_STRIDE(x, E) {
        const uint64_t g = x % G, xl = x / G;
        const uint32_t* o = goff + g * (EG + 1) + xl;
        len[x] = o[1] - o[0];
    }
}
__global__ void k_ktab_group_copy(uint64_t E, uint32_t G, uint64_t EG, const uint32_t* __restrict__ goff,
                                  const uint32_t* const* __restrict__ pb, const uint32_t* const* __restrict__ pe,
                                  const uint32_t* __restrict__ off, uint32_t* __restrict__ b, uint32_t* __restrict__ e) {
    GRID_STRIDE(x, E) {
        const uint64_t g = x % G, xl = x / G;
        const uint32_t* o = goff + g * (EG + 1) + xl;
        const uint32_t a = o[0], n = o[1] - o[0], to = off[x];
        for (uint32_t t = 0; t < n; t++) {
            b[to + t] = pb[g][a + t];
            e[to + t] = pe[g][a + t];
        }
    }
}

// off[x] = first item of D-mer x in the sorted keys (off[E] = n)
__global__ void k_ktab_bounds(uint64_t E, const uint64_t* __restrict__ key, uint64_t n, uint32_t* __restrict__ off) {
    GRID_STRIDE(x, E + 1) {
        if (x == E) { off[E] = (uint32_t)n; continue; }
        uint64_t lo = 0, hi = n;
        const uint64_t want = (uint64_t)x << 32;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (key[mid] < want) lo = mid + 1; else hi = mid;
        }
        off[x] = (uint32_t)lo;
    }
}

// per D-mer: its one interval inline (bit 63 | e << 32 | b; rows < 2^31) or its list's
// length << 32 | offset — one 8-B read per pattern at the direct start
// gpos (N < 2^30, text < 2^31): a one-row interval's entry also holds that row's text position,
// so the single-row text compare of the direct start reads no gpos line: bit 63 | bit 62 |
// gpos << 31 | row (other inline intervals keep e < 2^30 in bits [32, 62), bit 62 clear)
__global__ void k_ktab_one(uint64_t E, const uint32_t* __restrict__ off, const uint32_t* __restrict__ b, const uint32_t* __restrict__ e,
                           uint64_t* __restrict__ one, const uint32_t* __restrict__ gpos) {
    GRID_STRIDE(u, E + 1) {
        const uint32_t o = off[u], n = off[u + 1] - o;
        if (n == 1 && gpos && b[o] == e[o])
            one[u] = 3ull << 62 | (uint64_t)(gpos[b[o]] & 0x7fffffffu) << 31 | (b[o] & 0x7fffffffu);
        else
            one[u] = n == 1 ? (1ull << 63 | (uint64_t)e[o] << 32 | b[o]) : ((uint64_t)n << 32 | o);
    }
}

// the wide form (k_deep_fast's direct start, one line per pattern): 32 B per D-mer — k_ktab_one's
// entry and, for a one-row entry with its text position, the 32 characters of the reversed text
// before the row's suffix (rtext_window at tlen - g) and the row's sample
__global__ void k_ktab_wide(uint64_t E, const uint32_t* __restrict__ off, const uint32_t* __restrict__ b, const uint32_t* __restrict__ e,
                            const uint32_t* __restrict__ gpos, const uint4* __restrict__ samples, const uint64_t* __restrict__ rtext,
                            uint64_t tlen, uint4* __restrict__ w, uint32_t ws, const uint32_t* __restrict__ segtab, uint32_t seg_stride,
                            uint32_t seg_hi, uint32_t sigma) {
    // ws = 4 (KIdx::kt1_ws): a one-row entry also gets its word's segment's link ranks for c = 1..4
    GRID_STRIDE(u, E + 1) {
        const uint32_t o = off[u], n = off[u + 1] - o;
        uint64_t ent, win = 0;
        uint4 s = make_uint4(0, 0, 0, 0);
        if (n == 1 && b[o] == e[o]) {
            const uint32_t g = gpos[b[o]];
            ent = 3ull << 62 | (uint64_t)(g & 0x7fffffffu) << 31 | (b[o] & 0x7fffffffu);
            win = rtext_window(rtext, tlen - g);
            s = samples[b[o]];
        } else {
            ent = n == 1 ? (1ull << 63 | (uint64_t)e[o] << 32 | b[o]) : ((uint64_t)n << 32 | o);
            if (n >= 2 && n <= kWideInline) {  // a short list inline (k_deep's start): (b, e) pairs
                win = (uint64_t)e[o] << 32 | b[o];
                s = make_uint4(b[o + 1], e[o + 1], n > 2 ? b[o + 2] : 0u, n > 2 ? e[o + 2] : 0u);
            }
        }
        w[(size_t)ws * u] = make_uint4((uint32_t)ent, (uint32_t)(ent >> 32), (uint32_t)win, (uint32_t)(win >> 32));
        w[(size_t)ws * u + 1] = s;
        if (ws == 4) {
            uint32_t rx[4] = {0, 0, 0, 0}, ry[4] = {0, 0, 0, 0};  // (s.z < 2: no link, as the walk decides)
            if ((ent >> 62) == 3ull && s.z >= 2) {
                const uint32_t* et = segtab + (size_t)s.z * seg_stride;
#pragma unroll
                for (uint32_t c = 1; c <= 4; c++)
                    if (c < sigma) {
                        rx[c - 1] = et[1 + c];
                        ry[c - 1] = et[seg_hi + c];
                    }
            }
            w[4 * (size_t)u + 2] = make_uint4(rx[0], rx[1], rx[2], rx[3]);
            w[4 * (size_t)u + 3] = make_uint4(ry[0], ry[1], ry[2], ry[3]);
        }
    }
}

// per-row text-compare entries (KIdx::srow): the row's sample, its text position and the 32
// characters of the reversed text before its suffix
__global__ void k_srow(uint64_t N, const uint4* __restrict__ samples, const uint32_t* __restrict__ gpos, const uint64_t* __restrict__ rtext,
                       uint64_t tlen, uint4* __restrict__ out, const uint32_t* __restrict__ seg_lo) {
    GRID_STRIDE(x, N) {
        const uint32_t g = gpos[x];
        const uint64_t win = rtext_window(rtext, tlen - g);
        const uint4 s = samples[x];
        out[2 * x] = s;
        // .y: the chain bit of the row's word segment (seg_lo[s] != s - 1), carried by text items
        // into their link keys
        const uint32_t ch = s.z >= 2 && seg_lo[s.z] != s.z - 1 ? 1u : 0u;
        out[2 * x + 1] = make_uint4(g, ch, (uint32_t)win, (uint32_t)(win >> 32));
    }
}

__global__ void k_ktab_split(uint64_t n, const uint64_t* __restrict__ key, uint32_t* __restrict__ b) {
    GRID_STRIDE(t, n) b[t] = (uint32_t)key[t];
}

// search side: per depth-D node, its D-mer and the length of that D-mer's list.  The
// D-mer comes from the node's first pattern's sorted key chunk 0 (reversed sort codes,
// BPS bits each, most significant first; D <= SPC): sort code v = 1 + symbol code, so a
// non-'#' alphabet symbol has v in [2, B+1] and digit v-2; '#' or a byte outside the
// alphabet -> empty list.
template <int BPS>
__global__ void k_ktab_count(uint32_t M, uint32_t D, uint32_t B, const uint32_t* __restrict__ node_first, const uint64_t* __restrict__ k0,
                             const uint32_t* __restrict__ toff, uint32_t* __restrict__ kid, uint32_t* __restrict__ cnt) {
    constexpr uint32_t SPC = 64 / BPS;
    GRID_STRIDE(u, M) {
        const uint64_t key = k0[node_first[u]];
        uint32_t x = 0, mul = 1;
        bool ok = true;
        for (uint32_t t = 0; t < D; t++) {
            const uint32_t v = (uint32_t)(key >> (BPS * (SPC - 1 - t))) & ((1u << BPS) - 1u);
            ok &= v >= 2 && v <= B + 1;
            x += (v - 2) * mul;
            mul *= B;
        }
        kid[u] = ok ? x : 0xFFFFFFFFu;
        cnt[u] = ok ? toff[x + 1] - toff[x] : 0u;
    }
}

// items of depth D: node u's list copied from the table to pos[u] (exclusive scan of cnt).
// One wave per 64 consecutive nodes, whose outputs are contiguous: the wave walks its
// items 64 at a time, each lane finding its item's node by a binary search over the
// lanes' running counts (balanced and coalesced however long single lists are).
__global__ void __launch_bounds__(256) k_ktab_emit(uint32_t M, const uint32_t* __restrict__ kid, const uint32_t* __restrict__ pos,
                                                   const uint32_t* __restrict__ toff, const uint32_t* __restrict__ tb,
                                                   const uint32_t* __restrict__ te, uint32_t* __restrict__ iu, uint32_t* __restrict__ ib,
                                                   uint32_t* __restrict__ ie) {
    const uint32_t lane = threadIdx.x & 63, wpb = blockDim.x >> 6;
    for (size_t base = ((size_t)blockIdx.x * wpb + (threadIdx.x >> 6)) * 64; base < M; base += (size_t)gridDim.x * wpb * 64) {
        const size_t u = base + lane;
        uint32_t n = 0, start = 0;
        if (u < M) {
            const uint32_t x = kid[u];
            if (x != 0xFFFFFFFFu) { start = toff[x]; n = toff[x + 1] - start; }
        }
        uint32_t incl = n;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if ((int)lane >= o) incl += y;
        }
        const uint32_t excl = incl - n;
        const uint32_t total = __shfl(incl, 63, 64);
        const uint32_t out0 = pos[base];
        for (uint32_t q0 = 0; q0 < total; q0 += 64) {  // wave-uniform trip count: every lane joins the shuffles
            const uint32_t q = q0 + lane;
            uint32_t lo = 0;
#pragma unroll
            for (uint32_t step = 32; step; step >>= 1)
                if ((uint32_t)__shfl(excl, (int)(lo + step), 64) <= q) lo += step;
            const uint32_t src = (uint32_t)__shfl(start, (int)lo, 64) + (q - (uint32_t)__shfl(excl, (int)lo, 64));
            if (q < total) {
                iu[out0 + q] = (uint32_t)base + lo;
                ib[out0 + q] = tb[src];
                ie[out0 + q] = te[src];
            }
        }
    }
}

// the same items, one thread per item: for a few nodes with long lists (a shallow table
// start of a grouped search holds millions of intervals per node, which k_ktab_emit would
// copy 64 at a time per wave).  pos[0..M] = exclusive scan of the list lengths; item q
// belongs to the last node u with pos[u] <= q (nodes with empty lists share their pos)
__global__ void __launch_bounds__(256) k_ktab_emit_flat(uint32_t n0, uint32_t M, const uint32_t* __restrict__ kid, const uint32_t* __restrict__ pos,
                                                        const uint32_t* __restrict__ toff, const uint32_t* __restrict__ tb,
                                                        const uint32_t* __restrict__ te, uint32_t* __restrict__ iu, uint32_t* __restrict__ ib,
                                                        uint32_t* __restrict__ ie) {
    GRID_STRIDE(q, n0) {
        uint32_t lo = 0, hi = M;  // pos[lo] <= q < pos[hi]
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (pos[mid] <= (uint32_t)q) lo = mid; else hi = mid;
        }
        const uint32_t src = toff[kid[lo]] + ((uint32_t)q - pos[lo]);
        iu[q] = lo;
        ib[q] = tb[src];
        ie[q] = te[src];
    }
}

// ------------------------------------------- level start table (engine.hip build_ltab)
// The deep level start table holds, for every L-mer x over the non-'#' symbols, the order-free
// walk's intervals after its L characters, sorted by row — as the k-mer start table above, for
// a depth whose lists do not fit one u32-indexed array (C5: depth 8, ~9.5G intervals).  It is
// kept in G groups by x mod G (the L-mer's last characters, the same split as run_grouped's
// trie-subtree groups): group g's intervals lb[g][..], le[g][..] with u32 offsets
// loff[g * (EG + 1) + x / G] (EG = B^L / G L-mers per group, loff[g * (EG + 1) + EG] = its count).

// per depth-L node: its L-mer (from the node's first pattern's sorted key chunk 0, as
// k_ktab_count) and its list length; the batch's total into *total (a search over more than
// 2^31 - 1 start items is retried in trie-subtree groups)
template <int BPS>
__global__ void k_ltab_count(uint32_t M, uint32_t D, uint32_t B, const uint32_t* __restrict__ node_first, const uint64_t* __restrict__ k0,
                             const uint32_t* __restrict__ loff, uint32_t G, uint32_t EG, uint32_t* __restrict__ kid,
                             uint32_t* __restrict__ cnt, unsigned long long* __restrict__ total) {
    constexpr uint32_t SPC = 64 / BPS;
    GRID_STRIDE(u, M) {
        const uint64_t key = k0[node_first[u]];
        uint32_t x = 0, mul = 1;
        bool ok = true;
        for (uint32_t t = 0; t < D; t++) {
            const uint32_t v = (uint32_t)(key >> (BPS * (SPC - 1 - t))) & ((1u << BPS) - 1u);
            ok &= v >= 2 && v <= B + 1;
            x += (v - 2) * mul;
            mul *= B;
        }
        uint32_t c = 0;
        if (ok) {
            const uint32_t* o = loff + (size_t)(x % G) * (EG + 1) + x / G;
            c = o[1] - o[0];
        }
        kid[u] = ok ? x : 0xFFFFFFFFu;
        cnt[u] = c;
        if (c) atomicAdd(total, (unsigned long long)c);
    }
}

// the depth-L items: node u's list copied to pos[u] (exclusive scan of k_ltab_count's lengths).
// A wave copies kLtabTile = 64 x kLtabR consecutive items, lane l the items tile + k * 64 + l
// (coalesced); each lane finds the node of its first item by a binary search over pos and steps
// forward from there (lists are long: mostly no step at all).  Empty nodes share their pos.
constexpr uint32_t kLtabR = 16;
__global__ void __launch_bounds__(256) k_ltab_emit(uint32_t n0, uint32_t M, const uint32_t* __restrict__ kid, const uint32_t* __restrict__ pos,
                                                   const uint32_t* __restrict__ loff, uint32_t G, uint32_t EG,
                                                   const uint32_t* const* __restrict__ lb, const uint32_t* const* __restrict__ le,
                                                   uint32_t* __restrict__ iu, uint32_t* __restrict__ ib, uint32_t* __restrict__ ie) {
    const uint32_t lane = threadIdx.x & 63;
    const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwave = ((size_t)gridDim.x * blockDim.x) >> 6;
    for (size_t tile = wave * 64 * kLtabR; tile < n0; tile += nwave * 64 * kLtabR) {
        const uint32_t q0 = (uint32_t)tile + lane;
        if (q0 >= n0) continue;
        uint32_t lo = 0, hi = M;  // pos[lo] <= q0 < pos[hi] (pos[M] = n0)
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (pos[mid] <= q0) lo = mid; else hi = mid;
        }
        uint32_t nend = pos[lo + 1];
        for (uint32_t k = 0; k < kLtabR; k++) {
            const uint32_t q = q0 + k * 64;
            if (q >= n0) break;
            while (q >= nend) nend = pos[++lo + 1];
            const uint32_t x = kid[lo], g = x % G;
            const uint32_t src = loff[(size_t)g * (EG + 1) + x / G] + (q - pos[lo]);
            iu[q] = lo;
            ib[q] = lb[g][src];
            ie[q] = le[g][src];
        }
    }
}

// ------------------------------------------- pattern-file lines (host pipeline)
// A chunk of the pattern file as it lies on disk (MOVE_EDSBWTSearch.cpp:111 reads it with
// getline): the '\n' bytes are dropped and the offsets of the lines are written, so the
// search sees the (bytes, offsets) batch of edsbwt_search.  kLineBlk bytes per block of
// 256 threads, 16 per thread: k_nl_count counts each block's '\n', a scan gives the
// newlines before each block, k_nl_compact moves the bytes and writes line ends.
constexpr uint32_t kLineBlk = 4096;
// small host<->device transfers on the engine stream (engine.hip small_copy)
// zero up to 8 ranges (byte sizes multiples of 4, 4-B aligned) in one launch: blockIdx.y = range
struct ZeroSet {
    uint32_t* p[8];
    uint64_t n4[8];
};
__global__ void __launch_bounds__(256) k_zero_multi(ZeroSet z) {
    uint32_t* p = z.p[blockIdx.y];
    const uint64_t n = z.n4[blockIdx.y];
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) p[i] = 0u;
}
// the deferred checks and the statistics shards of a search, to page-locked host memory in
// one launch (engine.hip finish_deferred: chk layout kChk*)
__global__ void k_gather_checks(const unsigned long long* __restrict__ counters, const uint32_t* __restrict__ ovf,
                                const uint32_t* __restrict__ ovf2, const unsigned long long* __restrict__ stats, uint32_t nstats,
                                uint32_t* __restrict__ chk, unsigned long long* __restrict__ pstats) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t == 0) {
        unsigned long long term = counters[10], found = counters[1], occ = counters[12], tasks = counters[13];
        for (uint32_t sh = 0; sh < kStatShards && (sh + 1) * kStatStride <= nstats; sh++) {  // fused counts (deep kernels)
            found += stats[sh * kStatStride + ST_FC_FOUND];
            occ += stats[sh * kStatStride + ST_FC_OCC];
        }
        chk[0] = (uint32_t)term; chk[1] = (uint32_t)(term >> 32);
        chk[2] = *ovf;
        chk[3] = *ovf2;
        chk[4] = *reinterpret_cast<const uint32_t*>(counters + 20);
        chk[6] = (uint32_t)found; chk[7] = (uint32_t)(found >> 32);
        chk[8] = (uint32_t)occ; chk[9] = (uint32_t)(occ >> 32);
        chk[10] = (uint32_t)tasks; chk[11] = (uint32_t)(tasks >> 32);
    }
    for (uint32_t i = t; i < nstats; i += gridDim.x * blockDim.x) pstats[i] = stats[i];
}
__global__ void k_copy_words(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) dst[i] = src[i];
}
// downloads of the host pipeline: device -> mapped page-locked host memory as kernel stores
__global__ void __launch_bounds__(256) k_copy_out(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) dst[i] = src[i];
}
// compact download of a chunk's records: (word, offset); the host restores the rest
__global__ void k_rec_compact(const edsbwt_occ* __restrict__ rec, uint64_t n, uint2* __restrict__ out) {
    GRID_STRIDE(i, n) {
        const edsbwt_occ r = rec[i];
        out[i] = make_uint2(r.word, r.offset);
    }
}
// zero n bytes at p: 16-B stores over the aligned interior, byte stores at both ends
__global__ void __launch_bounds__(256) k_zero_bytes(uint8_t* __restrict__ p, uint64_t n) {
    const uint64_t head = min(n, (uint64_t)((16u - ((uintptr_t)p & 15u)) & 15u));
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
    if (tid < head) p[tid] = 0;
    uint4* q = reinterpret_cast<uint4*>(p + head);
    const uint64_t n16 = (n - head) / 16;
    for (uint64_t i = tid; i < n16; i += nt) q[i] = make_uint4(0u, 0u, 0u, 0u);
    const uint64_t t0 = head + n16 * 16;
    if (tid < n - t0) p[t0 + tid] = 0;
}
// a chunk's lines after k_nl_compact: P = newlines + (1 if the chunk does not end with
// '\n'); that last line's end; P and the longest and shortest line into out[0..2]
// (out[1] = max, out[2] = ~min, both by atomicMax; out zeroed before) — no host round trip
__global__ void __launch_bounds__(256) k_line_fin(uint64_t* __restrict__ offs, const uint32_t* __restrict__ nl_total, uint32_t tail,
                                                  uint64_t nb, unsigned long long* __restrict__ out) {
    const uint32_t nl = *nl_total;
    const uint64_t P = (uint64_t)nl + tail;
    const uint64_t tail_end = nb - nl;  // compacted bytes: the last line ends there
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid == 0) {
        out[0] = P;
        if (tail) offs[P] = tail_end;
    }
    __shared__ unsigned int smx, smn;
    if (threadIdx.x == 0) smx = smn = 0;
    __syncthreads();
    uint32_t mx = 0, nmn = 0;
    GRID_STRIDE(i, P) {
        const uint64_t e = (tail && i == P - 1) ? tail_end : offs[i + 1];
        const uint32_t L = (uint32_t)(e - offs[i]);
        mx = max(mx, L);
        nmn = max(nmn, ~L);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        mx = max(mx, (uint32_t)__shfl_xor(mx, o, 64));
        nmn = max(nmn, (uint32_t)__shfl_xor(nmn, o, 64));
    }
    if ((threadIdx.x & 63) == 0) { atomicMax(&smx, mx); atomicMax(&smn, nmn); }
    __syncthreads();
    if (threadIdx.x == 0) { atomicMax(out + 1, (unsigned long long)smx); atomicMax(out + 2, (unsigned long long)smn); }
}
// a chunk the host packed to 2 bits per base (format.cpp edsbwt_pack_lines: P lines of L
// bases, line p's codes at pk + p*S, code (byte >> 1) & 3): the line bytes back, without
// their '\n' as k_nl_compact leaves them, the line offsets, and P / longest / ~shortest into
// mm[0..2] as k_line_fin writes them.  16 output bytes per thread.
__global__ void __launch_bounds__(256) k_unpack_lines(const uint8_t* __restrict__ pk, uint64_t P, uint32_t L, uint32_t S,
                                                      uint8_t* __restrict__ out, uint64_t* __restrict__ offs,
                                                      unsigned long long* __restrict__ mm) {
    const uint64_t nbytes = P * L, n16 = (nbytes + 15) / 16;
    const uint32_t base = 0x47544341u;  // "ACTG": the byte of code c is byte c of this word
    GRID_STRIDE(i, n16) {
        const uint64_t pos = i * 16;
        uint64_t p = pos / L;
        uint32_t j = (uint32_t)(pos - p * L);
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        const uint32_t m = (uint32_t)min<uint64_t>(16, nbytes - pos);
        for (uint32_t k = 0; k < m; k++) {
            const uint32_t c = (pk[p * S + (j >> 2)] >> ((j & 3u) * 2u)) & 3u;
            w[k >> 2] |= ((base >> (c * 8u)) & 0xFFu) << ((k & 3u) * 8u);
            if (++j == L) { j = 0; p++; }
        }
        if (m == 16) {
            *reinterpret_cast<uint4*>(out + pos) = make_uint4(w[0], w[1], w[2], w[3]);
        } else {
            for (uint32_t k = 0; k < m; k++) out[pos + k] = (uint8_t)(w[k >> 2] >> ((k & 3u) * 8u));
        }
    }
    GRID_STRIDE(q, P + 1) offs[q] = q * L;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        mm[0] = P;
        mm[1] = L;
        mm[2] = (unsigned long long)(~L);
    }
}
// a chunk's counts as one byte each for the download (engine.hip expand_c8): 255 marks a
// count of 255 or more, listed as (pattern, count) in exc (room for P) after the *nexc
// counter (zeroed before).  4 counts per thread.
__global__ void __launch_bounds__(256) k_counts_u8(const uint32_t* __restrict__ c, uint64_t P, uint8_t* __restrict__ c8,
                                                   uint2* __restrict__ exc, uint32_t* __restrict__ nexc) {
    GRID_STRIDE(i, (P + 3) / 4) {
        uint32_t w = 0;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint64_t p = i * 4 + k;
            if (p >= P) break;
            const uint32_t v = c[p];
            if (v >= 255u) exc[atomicAdd(nexc, 1u)] = make_uint2((uint32_t)p, v);
            w |= min(v, 255u) << (8 * k);
        }
        *reinterpret_cast<uint32_t*>(c8 + i * 4) = w;
    }
}
// offsets of a chunk of a packed batch, rebased to its first byte
__global__ void k_rebase(uint64_t* __restrict__ off, uint64_t n, uint64_t base) { GRID_STRIDE(i, n) off[i] -= base; }
__global__ void __launch_bounds__(256) k_nl_count(const uint8_t* __restrict__ in, uint64_t n, uint32_t* __restrict__ cnt) {
    const uint64_t b0 = (uint64_t)blockIdx.x * kLineBlk + threadIdx.x * 16u;
    uint32_t c = 0;
    if (b0 + 16 <= n) {
        const uint4 v = *reinterpret_cast<const uint4*>(in + b0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t x = w[k] ^ 0x0A0A0A0Au;  // a zero byte where the byte is '\n'
            // exact per byte (no borrow between bytes): the high bit of t is 0 only for a zero byte
            const uint32_t t = ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x;
            c += __builtin_popcount(~t & 0x80808080u);
        }
    } else {
        for (uint64_t i = b0; i < n && i < b0 + 16; i++) c += in[i] == '\n';
    }
    __shared__ unsigned long long sh[4];
    const unsigned long long t = block_sum(c, sh);
    if (threadIdx.x == 0) cnt[blockIdx.x] = (uint32_t)t;
}

// pre[b] = newlines before block b.  out[i - nl_before(i)] = in[i] for non-'\n' bytes; the
// j-th newline (at i) ends line j: offs[j + 1] = i - j (offs[0] = 0 is written by the host)
__global__ void __launch_bounds__(256) k_nl_compact(const uint8_t* __restrict__ in, uint64_t n, const uint32_t* __restrict__ pre,
                                                    uint8_t* __restrict__ out, uint64_t* __restrict__ offs) {
    const uint64_t b0 = (uint64_t)blockIdx.x * kLineBlk + threadIdx.x * 16u;
    uint8_t v[16];
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        v[k] = b0 + k < n ? in[b0 + k] : (uint8_t)0;
        c += (b0 + k < n && v[k] == '\n') ? 1u : 0u;
    }
    // exclusive scan of c over the block
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if ((int)lane >= o) incl += y;
    }
    __shared__ uint32_t wsum[4];
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    uint32_t before = pre[blockIdx.x] + incl - c;
    for (uint32_t t = 0; t < wv; t++) before += wsum[t];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint64_t i = b0 + k;
        if (i >= n) break;
        if (v[k] == '\n') {
            offs[before + 1] = i - before;
            before++;
        } else {
            out[i - before] = v[k];
        }
    }
}

}  // namespace edsbwt
