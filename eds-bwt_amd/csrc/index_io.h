// eds-bwt_amd/csrc/index_io.h — host readers for the reference's index layout.
//
// Files (producers da_to_everything.cpp / eds_to_fasta.cpp):
//   <base>_info.aux   u32 N, u32 nText, u8 sigma, sigma alphabet bytes, nText u32
//                     EOF ids (per pile, row order), sigma*sigma u32 tableOcc
//                     (read as recoverInfo does, MOVE_EDSBWTSearch.cpp:628-770)
//   <base>.ebwt       N bytes of L (or the concatenation of <base>_bwt_<j>.aux)
//   <base>.bitvector  sdsl int_vector<1>: u64 bit count, then u64 words
//                     (loaded as MOVE_EDSBWTSearch.cpp:67-86 does)
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace edsbwt {

struct HostIndex {
    uint32_t N = 0, W = 0, sigma = 0, S = 0;
    uint8_t alpha[256] = {0};   // alphaInverse
    uint8_t code_of[256];       // byte -> code (0xFF: not in the alphabet)
    std::vector<uint32_t> eof_id;  // EOF_ID_Copy: DA of the k-th '#' row
    std::vector<uint32_t> tocc;    // tableOcc[j*sigma+h]
    std::vector<uint8_t> L;        // ebwt bytes
    std::vector<uint64_t> bv;      // segment bitvector words
    uint64_t bv_bits = 0;
};

// Returns 0 or a negative EDSBWT_E_* code with `err` set.
int read_host_index(const std::string& base, HostIndex& H, std::string& err);

}  // namespace edsbwt
