// eds-bwt_amd/csrc/index_io.cpp — readers for <base>_info.aux, <base>.ebwt (or
// _bwt_<j>.aux piles) and <base>.bitvector.  See index_io.h for the layout.
#include "index_io.h"

#include <cstdio>
#include <cstring>

#include "../../include/edsbwt.h"

namespace edsbwt {

namespace {
struct File {
    FILE* f = nullptr;
    explicit File(const std::string& p) { f = std::fopen(p.c_str(), "rb"); }
    ~File() { if (f) std::fclose(f); }
    bool read(void* p, size_t n) { return n == 0 || std::fread(p, 1, n, f) == n; }
    long size() {
        long here = std::ftell(f);
        std::fseek(f, 0, SEEK_END);
        long s = std::ftell(f);
        std::fseek(f, here, SEEK_SET);
        return s;
    }
};
}  // namespace

int read_host_index(const std::string& base, HostIndex& H, std::string& err) {
    // recoverInfo (MOVE_EDSBWTSearch.cpp:628-770)
    {
        File f(base + "_info.aux");
        if (!f.f) { err = "Error opening " + base + "_info.aux."; return EDSBWT_E_IO; }
        uint8_t s8 = 0;
        if (!f.read(&H.N, 4) || !f.read(&H.W, 4) || !f.read(&s8, 1)) {
            err = "Error reading header of " + base + "_info.aux";
            return EDSBWT_E_FORMAT;
        }
        H.sigma = s8 ? s8 : 256;
        if (!f.read(H.alpha, H.sigma)) { err = "Error reading alphaInverse"; return EDSBWT_E_FORMAT; }
        H.eof_id.resize(H.W);
        H.tocc.resize((size_t)H.sigma * H.sigma);
        if (!f.read(H.eof_id.data(), (size_t)H.W * 4)) { err = "Error reading EOF_ID"; return EDSBWT_E_FORMAT; }
        if (!f.read(H.tocc.data(), H.tocc.size() * 4)) { err = "Error reading tableOcc"; return EDSBWT_E_FORMAT; }
    }
    std::memset(H.code_of, 0xFF, sizeof H.code_of);
    for (uint32_t j = 0; j < H.sigma; j++) {
        if (j && H.alpha[j] <= H.alpha[j - 1]) { err = "alphabet not ascending"; return EDSBWT_E_FORMAT; }
        H.code_of[H.alpha[j]] = (uint8_t)j;
    }
    if (H.sigma == 0 || H.alpha[0] != '#') { err = "alphabet must start with the end-marker '#'"; return EDSBWT_E_FORMAT; }
    // L: .ebwt (build_MLF.cpp:55-64), or the piles _bwt_<j>.aux (da_to_everything.cpp:185-213)
    H.L.resize(H.N);
    {
        File f(base + ".ebwt");
        if (f.f) {
            if ((uint64_t)f.size() != H.N || !f.read(H.L.data(), H.N)) { err = base + ".ebwt length != N"; return EDSBWT_E_FORMAT; }
        } else {
            uint64_t at = 0;
            for (uint32_t j = 0; j < H.sigma; j++) {
                File p(base + "_bwt_" + std::to_string(j) + ".aux");
                if (!p.f) { err = "Error opening " + base + ".ebwt and " + base + "_bwt_" + std::to_string(j) + ".aux"; return EDSBWT_E_IO; }
                long s = p.size();
                if (at + (uint64_t)s > H.N || !p.read(H.L.data() + at, (size_t)s)) { err = "pile sizes exceed N"; return EDSBWT_E_FORMAT; }
                at += (uint64_t)s;
            }
            if (at != H.N) { err = "piles do not add up to N"; return EDSBWT_E_FORMAT; }
        }
    }
    // .bitvector (MOVE_EDSBWTSearch.cpp:67-86): sdsl int_vector<1>
    {
        File f(base + ".bitvector");
        if (!f.f) { err = "Error opening \"" + base + ".bitvector\" file"; return EDSBWT_E_IO; }
        if (!f.read(&H.bv_bits, 8)) { err = "short .bitvector"; return EDSBWT_E_FORMAT; }
        H.bv.assign((H.bv_bits + 63) / 64 + 1, 0);
        if (!f.read(H.bv.data(), (size_t)((H.bv_bits + 63) / 64) * 8)) { err = "short .bitvector"; return EDSBWT_E_FORMAT; }
    }
    if (H.bv_bits != H.W) { err = ".bitvector size != number of words"; return EDSBWT_E_FORMAT; }
    uint64_t ones = 0;
    for (uint64_t w = 0; w < (H.bv_bits + 63) / 64; w++) ones += (uint64_t)__builtin_popcountll(H.bv[w]);
    H.S = (uint32_t)ones;
    if (H.W && !(H.bv[0] & 1)) { err = "first word must start a segment"; return EDSBWT_E_FORMAT; }
    // consistency: pile sizes vs L, '#' count vs nText
    std::vector<uint64_t> cnt(256, 0);
    for (uint32_t i = 0; i < H.N; i++) cnt[H.L[i]]++;
    for (int c = 0; c < 256; c++)
        if (cnt[c] && H.code_of[c] == 0xFF) { err = "L holds a byte outside the alphabet"; return EDSBWT_E_FORMAT; }
    if (cnt['#'] != H.W) { err = "ERROR: The end-marker must be #"; return EDSBWT_E_FORMAT; }
    for (uint32_t j = 0; j < H.sigma; j++) {
        uint64_t pile = 0;
        for (uint32_t h = 0; h < H.sigma; h++) pile += H.tocc[(size_t)j * H.sigma + h];
        if (pile != cnt[H.alpha[j]]) { err = "tableOcc does not match L"; return EDSBWT_E_FORMAT; }
    }
    return 0;
}

}  // namespace edsbwt
