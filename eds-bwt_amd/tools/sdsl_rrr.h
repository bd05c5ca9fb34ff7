// eds-bwt_amd/tools/sdsl_rrr.h — the `<base>_bv_<j>.aux` files of the reference index: per BWT
// pile j, the bitvector "L[i] == '#'" serialized as sdsl-lite's rrr_vector<63, int_vector<>, 32>
// (da_to_everything.cpp:170-171,218-236: `rrr_vector<> rrrb(b); store_to_file(rrrb, bvName)`).
//
// Restated from sdsl-lite 2.x (rrr_vector.hpp, rrr_helper.hpp, int_vector.hpp), not copied:
//   blocks of 63 bits (LSB first); bt[i] = popcount of block i, one extra empty block when the
//   length is a multiple of 63; each block's bits as their rank among the 63-bit words of that
//   popcount (combinatorial number: a set bit at position p adds C(63-p-1, ones still to come)),
//   stored in ceil(log2 C(63, bt)) bits (0 for bt = 0 or 63) one after another in btnr; every 32
//   blocks a pointer into btnr and the rank before the superblock, plus a last rank sample
//   holding the total; the invert flags (never set for 63-bit blocks: no 32 blocks can need more
//   than 32 * 63 bits).  Members serialized as m_size (u64), bt, btnr, btnrp, rank, invert (the
//   order the survey read from the prebuilt binary's DWARF); int_vector<0>: u64 size in bits,
//   u8 width, ceil(size/64) u64 words; bit_vector: u64 size, words.  An int_vector whose width
//   would be 0 (hi(0) + 1) is stored 64 bits wide, as sdsl's width() makes it.
//
// Parity is UNPINNED: sdsl-lite is not in this image, the reference's prebuilt binary is never
// run, and no reference-written _bv file exists here.  The search never reads these files
// (numEOF[j] = tableOcc[j]['#'], MOVE_EDSBWTSearch.cpp:705); tests/test_tools.py decodes every
// block back and checks the rank samples against the piles.
#pragma once
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

namespace edsbwt_tools {

struct SdslIntVector {  // int_vector<0> / bit_vector being built
    uint64_t n = 0;     // elements
    uint8_t width = 1;
    std::vector<uint64_t> words;
    SdslIntVector(uint64_t n_, int w) : n(n_), width((uint8_t)(w <= 0 || w > 64 ? 64 : w)), words((n_ * (w <= 0 || w > 64 ? 64 : w) + 63) / 64, 0) {}
    void set(uint64_t i, uint64_t v) { set_bits(i * width, v, width); }
    void set_bits(uint64_t pos, uint64_t v, uint32_t len) {
        if (!len) return;
        if (len < 64) v &= (1ull << len) - 1;
        const uint64_t w = pos >> 6, o = pos & 63;
        words[w] |= v << o;
        if (o + len > 64) words[w + 1] |= v >> (64 - o);
    }
};

inline int sdsl_hi(uint64_t x) { return x ? 63 - __builtin_clzll(x) : -1; }

struct Rrr63 {
    static constexpr uint32_t kBs = 63, kK = 32;
    uint64_t C[64][64] = {};
    uint8_t space[64] = {};
    Rrr63() {
        for (int i = 0; i < 64; i++) {
            C[i][0] = 1;
            for (int j = 1; j <= i; j++) C[i][j] = C[i - 1][j - 1] + (j <= i - 1 ? C[i - 1][j] : 0);
        }
        for (int k = 0; k <= 63; k++) space[k] = C[63][k] == 1 ? 0 : (uint8_t)(sdsl_hi(C[63][k]) + 1);
    }
    uint64_t bin_to_nr(uint64_t bin) const {
        const uint64_t all = (1ull << 63) - 1;
        if (bin == 0 || bin == all) return 0;
        uint64_t nr = 0;
        int k = __builtin_popcountll(bin), nn = 63;
        while (bin) {
            if (bin & 1) { nr += C[nn - 1][k]; k--; }
            nn--;
            bin >>= 1;
        }
        return nr;
    }
    static uint64_t get_bits(const std::vector<uint64_t>& bv, uint64_t pos, uint32_t len) {
        const uint64_t w = pos >> 6, o = pos & 63;
        uint64_t v = bv[w] >> o;
        if (o + len > 64 && w + 1 < bv.size()) v |= bv[w + 1] << (64 - o);
        return len == 64 ? v : v & ((1ull << len) - 1);
    }
    // serialized bytes of rrr_vector<63> over bits [0, m) of bv (LSB first in u64 words)
    std::vector<uint8_t> build(const std::vector<uint64_t>& bv, uint64_t m) const {
        const uint64_t nb = (m + kBs) / kBs;  // blocks + a dummy block when m % 63 == 0
        std::vector<uint32_t> bt(nb, 0);
        uint64_t pos = 0, i = 0, btnr_pos = 0, sum_rank = 0;
        for (; pos + kBs <= m; pos += kBs) {
            const uint32_t x = (uint32_t)__builtin_popcountll(get_bits(bv, pos, kBs));
            bt[i++] = x;
            sum_rank += x;
            btnr_pos += space[x];
        }
        if (pos < m) {
            const uint32_t x = (uint32_t)__builtin_popcountll(get_bits(bv, pos, (uint32_t)(m - pos)));
            bt[i++] = x;
            sum_rank += x;
            btnr_pos += space[x];
        }
        const uint64_t nsup = (nb + kK - 1) / kK;
        SdslIntVector vbt(nb, sdsl_hi(kBs) + 1), btnr(std::max<uint64_t>(btnr_pos, 64), 1);
        SdslIntVector btnrp(nsup, sdsl_hi(btnr_pos) + 1), rank(nsup + ((m % (kK * kBs)) > 0 ? 1 : 0), sdsl_hi(sum_rank) + 1), invert(nsup, 1);
        for (uint64_t q = 0; q < nb; q++) vbt.set(q, bt[q]);
        pos = 0; i = 0; btnr_pos = 0; sum_rank = 0;
        for (; pos + kBs <= m; pos += kBs) {
            if (i % kK == 0) { btnrp.set(i / kK, btnr_pos); rank.set(i / kK, sum_rank); }  // invert stays 0 (see header)
            const uint32_t x = bt[i++];
            sum_rank += x;
            if (space[x]) { btnr.set_bits(btnr_pos, bin_to_nr(get_bits(bv, pos, kBs)), space[x]); btnr_pos += space[x]; }
        }
        if (pos < m) {
            if (i % kK == 0) { btnrp.set(i / kK, btnr_pos); rank.set(i / kK, sum_rank); }
            const uint32_t x = bt[i++];
            sum_rank += x;
            if (space[x]) { btnr.set_bits(btnr_pos, bin_to_nr(get_bits(bv, pos, (uint32_t)(m - pos))), space[x]); btnr_pos += space[x]; }
        }
        rank.set(rank.n - 1, sum_rank);
        std::vector<uint8_t> out;
        auto put = [&](const void* p, size_t n) { const uint8_t* c = (const uint8_t*)p; out.insert(out.end(), c, c + n); };
        auto put_iv = [&](const SdslIntVector& v, bool var) {
            const uint64_t bits = v.n * v.width;
            put(&bits, 8);
            if (var) put(&v.width, 1);
            put(v.words.data(), v.words.size() * 8);
        };
        put(&m, 8);
        put_iv(vbt, true);
        put_iv(btnr, false);
        put_iv(btnrp, true);
        put_iv(rank, true);
        put_iv(invert, false);
        return out;
    }
};

}  // namespace edsbwt_tools
