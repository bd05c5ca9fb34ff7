// eds-bwt_amd/csrc/kernels.h — device data layout shared by kernels.hip and engine.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "../../include/edsbwt.h"

namespace edsbwt {

#ifndef EDSBWT_OCC_ROWS
#define EDSBWT_OCC_ROWS 64
#endif
#if EDSBWT_OCC_ROWS == 256
// 128-B rank block over 256 BWT rows: 0.5 B/row
constexpr uint32_t kOccShift = 8;
struct alignas(128) OccBlock {
    uint32_t cnt[8];
    uint64_t plane[3][4];
};
static_assert(sizeof(OccBlock) == 128, "occ block must be one 128-B line");
#elif EDSBWT_OCC_ROWS == 64
// 64-B rank block over 64 BWT rows: 1 B/row, one half-line per rank query.
// When sigma <= 7 the block also carries the locate samples: `samp` marks the rows
// whose offset in their word is a multiple of the sample rate, and cnt[7] (no symbol
// has code 7) holds the number of sampled rows before the block.
constexpr uint32_t kOccShift = 6;
struct alignas(64) OccBlock {
    uint32_t cnt[8];
    uint64_t plane[3][1];
    uint64_t samp;
};
static_assert(sizeof(OccBlock) == 64, "occ block must be 64 B");
#else
#error "EDSBWT_OCC_ROWS must be 64 or 256"
#endif
constexpr uint32_t kOccRows = 1u << kOccShift;

// Rank entries (sigma <= 5): 32 BWT rows per block and one 16-B entry per query, so an
// interval end costs ONE 16-B load per step (the gathers are bound by load instructions
// per random line, not by bytes: DESIGN.md §5).
//   rent1[k * sigma + c] = {rank_c(32k), mask of the block's rows with L = c,
//                           rank_'#'(32k), mask of its '#' rows}
// answers a backward step by c and the '#' rows (link) of the interval at once.  Pair codes
// code(x) = 0 when L[x] = '#', else 1 + (L[x]-1)*sigma + L[LF(x)]: rows of the suffixes c2 c1 Q
// are [PC[p] + rank_p(b), PC[p] + rank_p(e+1)) for p = (c1, c2) and Q's rows [b, e], and
//   rent2[k * (nc-1) + p-1] = {rank_p(32k), mask_p, rank_{0|q}(32k), mask_{0|q}}, q = (c1, '#'),
// answers two steps at once when no row of [b, e] holds '#' or (c1, '#') — no link at
// either step.  Triple codes (L[x], L[LF(x)], L[LF^2(x)]) give, the same way,
//   rent3[k * (sigma-1)^3 + t] = {rank_p(32k), mask_p, rank of rows coded '#', (c1, '#') or
//                                 (c1, c2, '#') (32k), their mask} for p = (c1, c2, c3)
// and three steps per entry.
constexpr uint32_t kPairCodes = 21;  // sigma = 5: 1 + 4 * 5

// per-pattern result (backwardSearch's final list): archive offset of its intervals, their
// number and the occurrence count; one 16-B record, written with one store
struct alignas(16) Res {
    uint64_t off;
    uint32_t cnt, occ;
};

// kernel-side view of the device index (passed by value)
struct KIdx {
    const OccBlock* occ;       // ceil((N+1)/256) blocks
    const uint32_t* eof_seg;   // [W] segment (1-based) of the word of the k-th '#' row, 0 if segment 1
    const uint32_t* eof_word;  // [W] EOF_ID_Copy
    const uint32_t* seg_of_word;  // [W] 1-based segment of each word
    const uint32_t* seg_start;    // [S+2] first word of segment s (1-based), seg_start[S+1] = W
    const uint32_t* seg_lo;       // [S+2] lowest segment reached by link from segment s (empty-word chains)
    const uint32_t* da;        // [N] optional DA per row
    const uint32_t* offt;      // [N] optional offset-in-word per row
    uint32_t N, W, S, sigma;
    const uint4* samples;      // (word, offset, segment, word in segment) of the sampled rows, in row order (locate)
    uint32_t samp_dense;       // every row sampled: samples[x] is row x's (no occ-block rank needed)
    // per segment s (link of a word in s): [0] seg_lo[s]; [1 + c] rank_c at the first word of
    // segment seg_lo[s]; [seg_hi + c] rank_c at the first word of s.  seg_stride u32 per entry.
    const uint32_t* segtab;
    uint32_t seg_stride, seg_hi;
    uint32_t segbits;          // bits of a segment id (1..S): link keys are node << segbits | segment
    uint32_t rowbits;          // bits of a BWT row (< N): finisher keys are node << rowbits | row
    uint32_t C[8];             // first row of each pile
    const uint4* rent1;        // single-step rank entries (nullptr: not built)
    const uint4* rent2;        // two-step rank entries (nullptr: not built or not used)
    uint32_t r2stride;         // rent2 entries per block (pair codes - 1)
    const uint4* rent3;        // three-step rank entries (nullptr: not built or not used)
    uint32_t r3stride;         // rent3 entries per block ((sigma-1)^3)
    const uint32_t* PC3;       // first row of the suffixes c3 c2 c1 ... per rent3 entry
    uint32_t PC[kPairCodes + 3];  // first row of the suffixes c2 c1 ... for pair code p = (c1, c2)
    // Text of the words (sigma - 1 <= 4, every row sampled): a single-row interval is one text
    // position, so the next characters of the pattern are compared with the text instead of
    // stepped through the rank entries ("single rows").
    const uint64_t* rtext;     // nullptr: off.  2-bit symbol codes - 1 of the words' characters,
                               // concatenated in word order and reversed, 32 per u64 (char i at bits 2(i%32))
    uint64_t tlen;             // characters in the text
    const uint32_t* gpos;      // [N] text position of row x's suffix (word start + offset)
    const uint32_t* wrow;      // [W] row of each word's whole-word suffix (offset 0)
    const uint4* srow;         // nullptr, or [2N]: row x's sample (srow[2x]) and {gpos[x], 0, the 32
                               // reversed-text characters before its suffix} (srow[2x+1]): a single
                               // row's text compare from ONE line (k_srow; dense samples + text)
    // the direct start's link from a word start (k_deep_direct; sigma = 5 with srow; nullptr: not
    // built): per segment s, 128 B = one DRAM line, for c = 1..4 at seglink[8 s + 2 (c - 1)]:
    // {rx, ry, sample.x, sample.y}, {sample.z, sample.w, window lo, window hi} — the segment link
    // table's ranks (segtab [1 + c], [seg_hi + c]) and, when ry = rx + 1, the srow entry of the one
    // row C[c] + rx, so a link that lands on one row needs no second line for its text compare
    const uint4* seglink;
    uint32_t text_deep;        // k_deep compares single rows too (EDSBWT_TEXT_DEEP, A/B)
    uint32_t deep_filter;      // k_deep (packed build) filters a list start of single rows by their text (EDSBWT_DEEPQ_FILTER)
    uint32_t kt1_pos;          // the direct start's inline D-mer entries of ONE row hold that row's
                               // text position too (k_ktab_one): bit 62 set, gpos in bits [31, 62)
    // All-symbol rank entries (sigma <= 5; nullptr: not built or not used): the rank of every
    // symbol at a row from ONE 16-B load (the 64-B occ block takes four: the level step's
    // gathers are bound by load requests).
    //   rk16[k]    = {cnt_1 | cnt_2 << 16, cnt_3 | cnt_4 << 16, plane_0 | plane_1 << 16, plane_2}
    //                cnt_c: rows of symbol c in [65536 * (k >> 12), 16 k); planes: the 3 code bits
    //                of rows 16k .. 16k+15 (bit j = row 16k + j)
    //   rk16sup[s] = {rank_1 .. rank_4 at row 65536 s}
    // rank_'#'(x) = x - (rank_1 + rank_2 + rank_3 + rank_4).
    const uint4* rk16;
    const uint4* rk16sup;
    // link keys of the order-free level walk (k_lvl_items, k_lvl_chunks): link_seg[k] for the
    // k-th '#' row; link_cb = 1: link_seg holds segment << 1 | chain bit (seg_lo[s] != s - 1,
    // 0 for segment 1) and the keys are node << (segbits + 1) | link_seg, so k_run_flags needs
    // no seg_lo or bitmap read for a key without a chain; link_cb = 0: link_seg = eof_seg
    const uint32_t* link_seg;
    uint32_t link_cb;
    // per-'#'-row link rows (sigma <= 7, nullptr: not built): eofrow[16 k ..] = the segment link
    // table's row of segment s = eof_seg[k] with [15] = s (0: segment 1) — k_deep's link from a
    // '#' row reads ONE line (its segment and that segment's ranks) instead of eof_seg[k] and
    // then, dependent on it, segtab[s]
    const uint32_t* eofrow;
    // segtext = 1: the segment link table's rows are 32 u32 (128 B, one DRAM request as the 64-B
    // ones) and [16 + 2 (c - 1)], [17 + 2 (c - 1)] hold, for c = 1..4, the text-item form (kernels.hip
    // kTextItem) of the ONE word of [seg_lo[s], s - 1] ending with c, when there is one: the dollar
    // step then hands that single row on as a text item (no srow read at the next depth)
    uint32_t segtext;
    // the k-mer start table's D-mers (B^depth; entry kt_E is the empty list of D-mers outside the
    // alphabet) and intervals: the bounds a queued direct-start list is checked against in the
    // debug build (-DEDSBWT_DEBUG_CHECKS)
    uint32_t kt_E, kt_n;
    // uint4s per wide D-mer entry (kt1w): 2, or 4 when a one-row entry also holds the link ranks of
    // its row's word's segment for c = 1..4 (rx at uint4 2, ry at uint4 3: segtab's [1 + c] and
    // [seg_hi + c]) — the first link after the entry's text compare then reads the entry's own
    // 128-B DRAM line instead of a segment row (sigma <= 5; EDSBWT_KT1_LINK=1)
    uint32_t kt1_ws;
};

}  // namespace edsbwt
