// eds-bwt_amd/tools/eds_transform.cpp — EDS → EDS-BWT index writer.
//
// Replaces the reference's EDS-BWTransform.sh chain (eds_to_fasta.cpp +
// gsufsort --da --bwt + da_to_everything.cpp) and writes the same files:
//   <base>.bitvector  sdsl int_vector<1> of segment starts     eds_to_fasta.cpp:151-153
//   <base>.ebwt       BWT with 'Z' and the terminator as '#'    da_to_everything.cpp:407-457
//   <base>_info.aux   N, nText, sigma, alphabet, EOF ids, tableOcc  da_to_everything.cpp:150-254
//   <base>_bwt_<j>.aux  pile j of the BWT                      da_to_everything.cpp:185-213
//   <base>_runs.aux / <base>_runs.txt  run heads and LF(run head)  da_to_everything.cpp:62-109,414-443
//   <base>_bv_<j>.aux   pile j's "L == '#'" as sdsl rrr_vector<63>  da_to_everything.cpp:170-171,218-236
//                       (tools/sdsl_rrr.h; parity unpinned: the search reads numEOF[j] from tableOcc)
//
// Suffix order (gsufsort's generalized suffix array over word·'#'): suffixes are
// compared up to and including their word's '#', '#' smallest, equal suffixes by
// word id.  Built here by a parallel LSD radix sort on packed prefixes of
// floor(64/b) symbols (b = bits per symbol code), ties on unterminated prefixes
// refined chunk by chunk (OpenMP), or with --gpu [device] on an MI355X by prefix
// doubling in libedsbwt.so (edsbwt_gsa: O(log longest word) radix sorts); both give
// the same order, so the same files.
//
// usage: eds_transform <file.eds> <base> [--no-runs] [--threads T] [--gpu [device]]
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "eds_common.h"
#include "sdsl_rrr.h"
#include "../../include/edsbwt.h"

using namespace edsbwt_tools;

namespace {

struct KP {
    uint64_t k;
    uint32_t pos, pad;
};

double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

void radix_sort(std::vector<KP>& a, int key_bits, int T) {
    std::vector<KP> b(a.size());
    const size_t n = a.size();
    const int passes = (key_bits + 7) / 8;
    std::vector<size_t> hist((size_t)T * 256);
    for (int p = 0; p < passes; p++) {
        const int sh = 8 * p;
        std::fill(hist.begin(), hist.end(), 0);
#pragma omp parallel num_threads(T)
        {
            const int t = omp_get_thread_num();
            const size_t lo = n * t / T, hi = n * (t + 1) / T;
            size_t* h = &hist[(size_t)t * 256];
            for (size_t i = lo; i < hi; i++) h[(a[i].k >> sh) & 255]++;
        }
        // digit-major, thread-minor exclusive offsets (stable)
        size_t acc = 0;
        bool trivial = false;
        for (int d = 0; d < 256; d++) {
            size_t dsum = 0;
            for (int t = 0; t < T; t++) dsum += hist[(size_t)t * 256 + d];
            if (dsum == n) trivial = true;
            for (int t = 0; t < T; t++) {
                size_t c = hist[(size_t)t * 256 + d];
                hist[(size_t)t * 256 + d] = acc;
                acc += c;
            }
        }
        if (trivial) continue;  // every key has the same digit here
#pragma omp parallel num_threads(T)
        {
            const int t = omp_get_thread_num();
            const size_t lo = n * t / T, hi = n * (t + 1) / T;
            size_t* h = &hist[(size_t)t * 256];
            for (size_t i = lo; i < hi; i++) b[h[(a[i].k >> sh) & 255]++] = a[i];
        }
        a.swap(b);
    }
}

void write_file(const std::string& path, const void* p, size_t n) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write " + path);
    if (n && std::fwrite(p, 1, n, f) != n) { std::fclose(f); throw std::runtime_error("short write " + path); }
    std::fclose(f);
}

char* put_u(char* p, uint64_t v) {
    char tmp[24];
    int k = 0;
    do { tmp[k++] = (char)('0' + v % 10); v /= 10; } while (v);
    while (k) *p++ = tmp[--k];
    return p;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s <file.eds> <base> [--no-runs] [--threads T]\n", argv[0]);
        return 1;
    }
    const std::string in = argv[1], base = argv[2];
    bool runs = true;
    int T = omp_get_max_threads();
    int gpu = -1;
    for (int i = 3; i < argc; i++) {
        if (!std::strcmp(argv[i], "--no-runs")) runs = false;
        else if (!std::strcmp(argv[i], "--threads") && i + 1 < argc) T = std::max(1, std::atoi(argv[++i]));
        else if (!std::strcmp(argv[i], "--gpu")) gpu = (i + 1 < argc && argv[i + 1][0] != '-') ? std::atoi(argv[++i]) : 0;
    }
    try {
        double t0 = now();
        Eds E = parse_eds(read_all(in));
        const uint64_t tot = E.text.size(), W = E.wstart.size();
        if (tot >= 0xFFFFFFFFull) throw std::runtime_error("text longer than 2^32-1 symbols (u32 rows, Parameters.h:71)");
        const uint8_t* Tx = E.text.data();
        // symbol codes: '#' = 0, the other bytes ascending
        int code[256];
        std::fill(code, code + 256, -1);
        {
            std::vector<uint8_t> present(256, 0);
            for (uint64_t i = 0; i < tot; i++) present[Tx[i]] = 1;
            present['#'] = 0;
            code['#'] = 0;
            int K = 0;
            for (int c = 0; c < 256; c++)
                if (present[c]) code[c] = ++K;
        }
        int K = 0;
        for (int c = 0; c < 256; c++) K = std::max(K, code[c]);
        const int b = std::max(1, 64 - __builtin_clzll((uint64_t)K));
        const int cpw = 64 / b;
        const uint64_t lastmask = (1ull << b) - 1;
        const int top = b * (cpw - 1);
        std::vector<KP> kp(tot);
        size_t ngroups = 0;
        double gpu_ms = -1;
        if (gpu >= 0) {
            // the suffix sort on the GPU (edsbwt_gsa): codes with '#' = 0 and the words' ends
            std::vector<uint8_t> codes(tot);
            std::vector<uint64_t> ends(W);
#pragma omp parallel for num_threads(T)
            for (int64_t i = 0; i < (int64_t)tot; i++) codes[i] = (uint8_t)code[Tx[i]];
#pragma omp parallel for num_threads(T)
            for (int64_t w = 0; w < (int64_t)W; w++) ends[w] = (w + 1 < (int64_t)W ? E.wstart[w + 1] : tot) - 1;
            std::vector<uint32_t> sa(tot);
            if (edsbwt_gsa(codes.data(), tot, ends.data(), W, (uint32_t)b, gpu, sa.data(), &gpu_ms) != 0)
                throw std::runtime_error(std::string("edsbwt_gsa: ") + edsbwt_last_error());
#pragma omp parallel for num_threads(T)
            for (int64_t i = 0; i < (int64_t)tot; i++) kp[i] = KP{0, sa[i], 0};
        } else {
        // packed prefix of every suffix (right to left inside each word)
        std::vector<uint64_t> key0(tot);
#pragma omp parallel for schedule(dynamic, 4096) num_threads(T)
        for (int64_t w = 0; w < (int64_t)W; w++) {
            const uint64_t s = E.wstart[w];
            const uint64_t e = (w + 1 < (int64_t)W ? E.wstart[w + 1] : tot) - 1;  // the '#'
            uint64_t key = 0;
            key0[e] = 0;
            for (uint64_t t = e; t-- > s;) {
                key = ((uint64_t)code[Tx[t]] << top) | (key >> b);
                key0[t] = key;
            }
        }
#pragma omp parallel for num_threads(T)
        for (int64_t i = 0; i < (int64_t)tot; i++) kp[i] = KP{key0[i], (uint32_t)i, 0};
        radix_sort(kp, b * cpw, T);
        // refine groups of equal unterminated prefixes
        std::vector<std::pair<uint64_t, uint64_t>> groups;
        for (uint64_t i = 0; i < tot;) {
            uint64_t j = i + 1;
            while (j < tot && kp[j].k == kp[i].k) j++;
            if (j - i > 1 && (kp[i].k & lastmask)) groups.emplace_back(i, j);
            i = j;
        }
        auto cmp = [&](const KP& x, const KP& y) {
            uint64_t a = x.pos, c = y.pos;
            for (;;) {
                a += cpw;
                c += cpw;
                const uint64_t ka = key0[a], kc = key0[c];
                if (ka != kc) return ka < kc;
                if (!(ka & lastmask)) return x.pos < y.pos;
            }
        };
#pragma omp parallel for schedule(dynamic, 1) num_threads(T)
        for (int64_t g = 0; g < (int64_t)groups.size(); g++) std::sort(kp.begin() + groups[g].first, kp.begin() + groups[g].second, cmp);
        ngroups = groups.size();
        }
        double t1 = now();
        // rows: drop the 'Z#' suffixes of empty words (remove_empty_symbols, :397,:438)
        const uint64_t N = tot - E.empty;
        for (uint64_t i = N; i < tot; i++)
            if (Tx[kp[i].pos] != 'Z') throw std::runtime_error("internal: 'Z' suffixes are not last");
        std::vector<uint8_t> rawL(N), L(N);
        std::vector<uint32_t> da(N);
#pragma omp parallel for num_threads(T)
        for (int64_t i = 0; i < (int64_t)N; i++) {
            const uint32_t p = kp[i].pos;
            const bool ws = (p == 0 || Tx[p - 1] == '#');
            const uint8_t c = ws ? (uint8_t)'#' : Tx[p - 1];
            rawL[i] = c;
            L[i] = (c == 'Z') ? (uint8_t)'#' : c;
            if (L[i] == '#') da[i] = (uint32_t)(std::upper_bound(E.wstart.begin(), E.wstart.end(), (uint64_t)p) - E.wstart.begin() - 1);
        }
        std::vector<KP>().swap(kp);
        // buildFreq (da_to_everything.cpp:301-366)
        std::vector<uint64_t> freq(256, 0);
        {
            std::vector<std::vector<uint64_t>> part(T, std::vector<uint64_t>(256, 0));
#pragma omp parallel num_threads(T)
            {
                const int t = omp_get_thread_num();
                for (uint64_t i = N * t / T; i < N * (t + 1) / T; i++) part[t][L[i]]++;
            }
            for (int t = 0; t < T; t++)
                for (int c = 0; c < 256; c++) freq[c] += part[t][c];
        }
        if (freq['#'] != W) throw std::runtime_error("ERROR: The end-marker must be #");
        int alpha[256] = {0};
        std::vector<uint8_t> ainv;
        for (int c = 0; c < 256; c++)
            if (freq[c]) { alpha[c] = (int)ainv.size(); ainv.push_back((uint8_t)c); }
        const uint32_t sigma = (uint32_t)ainv.size();
        // tableOcc + piles + EOF ids (da_to_everything.cpp:113-290)
        std::vector<uint64_t> pstart(sigma + 1, 0);
        for (uint32_t j = 0; j < sigma; j++) pstart[j + 1] = pstart[j] + freq[ainv[j]];
        std::vector<uint32_t> tocc((size_t)sigma * sigma, 0);
        for (uint32_t j = 0; j < sigma; j++) {
            std::vector<std::vector<uint32_t>> part(T, std::vector<uint32_t>(sigma, 0));
            const uint64_t lo = pstart[j], n = pstart[j + 1] - lo;
#pragma omp parallel num_threads(T)
            {
                const int t = omp_get_thread_num();
                for (uint64_t i = lo + n * t / T; i < lo + n * (t + 1) / T; i++) part[t][alpha[L[i]]]++;
            }
            for (int t = 0; t < T; t++)
                for (uint32_t h = 0; h < sigma; h++) tocc[(size_t)j * sigma + h] += part[t][h];
            write_file(base + "_bwt_" + std::to_string(j) + ".aux", L.data() + lo, n);
            {  // _bv_<j>.aux: the pile's '#' rows
                std::vector<uint64_t> bits((n + 63) / 64 + 1, 0);
                for (uint64_t i = 0; i < n; i++)
                    if (L[lo + i] == '#') bits[i >> 6] |= 1ull << (i & 63);
                static const Rrr63 rrr;
                const std::vector<uint8_t> bytes = rrr.build(bits, n);
                write_file(base + "_bv_" + std::to_string(j) + ".aux", bytes.data(), bytes.size());
            }
        }
        write_file(base + ".ebwt", L.data(), N);
        {
            std::vector<uint8_t> info;
            auto put32 = [&](uint32_t v) { const uint8_t* p = (const uint8_t*)&v; info.insert(info.end(), p, p + 4); };
            put32((uint32_t)N);
            put32((uint32_t)freq[ainv[0]]);
            info.push_back((uint8_t)sigma);
            info.insert(info.end(), ainv.begin(), ainv.end());
            info.reserve(info.size() + W * 4 + tocc.size() * 4);
            for (uint64_t i = 0; i < N; i++)
                if (L[i] == '#') put32(da[i]);
            for (uint32_t v : tocc) put32(v);
            write_file(base + "_info.aux", info.data(), info.size());
        }
        // .bitvector (eds_to_fasta.cpp:151-153)
        {
            std::vector<uint64_t> words(1 + (W + 63) / 64, 0);
            words[0] = W;
            for (uint64_t w = 0; w < W; w++)
                if (E.first[w]) words[1 + (w >> 6)] |= 1ull << (w & 63);
            write_file(base + ".bitvector", words.data(), words.size() * 8);
        }
        // _runs.aux (da_to_everything.cpp:414-443) and _runs.txt (build_ilf, :62-109)
        if (runs) {
            std::vector<uint64_t> sp(sigma, 0);
            for (uint32_t j = 0; j + 1 < sigma; j++) sp[j + 1] = pstart[j + 1];
            std::vector<char> ra, rt;
            ra.reserve(N * 6);
            rt.reserve(N * 12);
            char buf[64];
            uint8_t prev = '#';
            bool have = false;
            uint64_t ip = 0;
            uint8_t let = 0;
            for (uint64_t i = 0; i < N; i++) {
                const uint8_t c = rawL[i];
                const bool head = (prev != c || c == 'Z' || c == '#');
                prev = c;
                if (!head) continue;
                char* p = put_u(buf, i);
                *p++ = ',';
                *p++ = (char)c;
                *p++ = '\n';
                ra.insert(ra.end(), buf, p);
                if (have) sp[alpha[let]] += i - ip;  // alpha['Z'] == 0 (zero-initialised global)
                ip = i;
                let = c;
                have = true;
                p = put_u(buf, ip);
                *p++ = ',';
                p = put_u(p, sp[alpha[let]]);
                *p++ = '\n';
                rt.insert(rt.end(), buf, p);
            }
            write_file(base + "_runs.aux", ra.data(), ra.size());
            write_file(base + "_runs.txt", rt.data(), rt.size());
        }
        double t2 = now();
        if (gpu >= 0)
            std::fprintf(stderr, "eds_transform: %llu words, %llu rows, sigma %u; GPU suffix sort %.3fs (device %d, %.1f ms on the device), "
                                 "sort total %.2fs, write %.2fs (%d threads)\n",
                         (unsigned long long)W, (unsigned long long)N, sigma, gpu_ms / 1e3, gpu, gpu_ms, t1 - t0, t2 - t1, T);
        else
            std::fprintf(stderr, "eds_transform: %llu words, %llu rows, sigma %u, %zu tie groups; sort %.2fs, write %.2fs (%d threads)\n",
                         (unsigned long long)W, (unsigned long long)N, sigma, ngroups, t1 - t0, t2 - t1, T);
        std::fprintf(stderr, "File %s done.\n", in.c_str());
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
