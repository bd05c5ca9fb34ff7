// eds-bwt_amd/tools/edsbwtsearch_cli.cpp — the EDSBWTsearch / MOVE_EDSBWTSearch CLI.
//
//   EDSBWTsearch <index_base> <pattern_file> [--device D] [--quiet] [--count-only] [--table] [--legacy]
//
// Same argv, files and console contract as mainMove_EDSBWT.cpp:17-62 driving
// MOVE_EDSBWT::MOVE_EDSBWT (MOVE_EDSBWTSearch.cpp:23-176):
//   * wrong argc → usage on stderr, exit 1 (:19-25); success also exits 1 (:61);
//   * writes <pattern_file>output_M_LF.csv with header "#Pat\t$_i\tD[i]\tS_j\tS_j[r] \n" (:55-64);
//   * stdout: banner (mainMove_EDSBWT.cpp:27-29), "DEBUG: 0" (:28), recoverInfo's index summary,
//     "NUM OF EOF", TableOcc (:664-671,:725,:761-766), retrieve_MLF's "size= " (:191),
//     "BitVector size: " (:86); per pattern "Pattern: <p> of length <n>" (:113) and — unless
//     backwardSearch returned before its locate loop (:250-253,:295-297) — "num occ <k>" (:371);
//     then "bs took:<secs>" without a newline (:145);
//   * stderr: "Backward Search" (:25), "OCCORRENZA DI: <p> TROVATA|NON TROVATA" per pattern
//     (:124,:129), then "count_found = N" / "count_not_found = M" (:154-155) — the lines the
//     reference's scripts grep (launch_COVID.sh:106-108) — and main's closing lines (:50-59).
//   Each pattern's stdout lines are flushed before its stderr line, as endl does, so the two
//   streams interleave as the reference's do when they share a file.
//   backwardSearch returns early exactly when the list after all but the first character is
//   empty, i.e. when the pattern without its first character does not occur (its own final
//   list is that list): the console stream asks the engine for those counts too.
// --quiet drops the per-pattern lines (they dominate console time at 10^7 patterns).
// --legacy writes <pattern_file>output.csv in the legacy EDSBWTsearch engine's record order
// and header (EDSBWTsearch.cpp:180-186, findMultipleDollarsBackward :300-610) instead.
// --gpus N (or --devices a,b,..): the pattern loop (:111-136) sharded over N devices — one index
// per device (opened in parallel), contiguous line ranges searched concurrently with
// first_pattern_id = first line + 1 so #Pat stays the file's line number, and each shard's CSV
// rows written at its byte offset of the one output file: the same bytes
// as --gpus 1.  With fewer devices than N the shards share them (device k mod count), opened one
// after another on a shared device, each sizing its tables for its share (EDSBWT_HBM_SHARE).
// The search itself runs on the GPU through libedsbwt.so (include/edsbwt.h).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/edsbwt.h"

namespace {
// one device's share of the pattern file: lines [line0, line0 + nlines), bytes [b0, b1)
struct Shard {
    int device = 0;
    edsbwt_index* idx = nullptr;
    uint64_t line0 = 0, nlines = 0, b0 = 0, b1 = 0;
    edsbwt_occ* occ = nullptr;
    uint64_t nocc = 0, npat = 0, csv_at = 0;
    int rc = 0;
    std::string err;
};

// f(k) for k < n, each on its own thread (n = 1: the calling thread)
template <class F>
void each(size_t n, F f) {
    if (n == 1) { f(0); return; }
    std::vector<std::thread> th;
    for (size_t k = 0; k < n; k++) th.emplace_back([&, k] { f(k); });
    for (auto& t : th) t.join();
}

std::vector<int> parse_devices(const char* s) {
    std::vector<int> d;
    for (const char* p = s; *p;) {
        char* e = nullptr;
        const long v = std::strtol(p, &e, 10);
        if (e == p) break;
        d.push_back((int)v);
        p = *e == ',' ? e + 1 : e;
    }
    return d;
}
}  // namespace

int main(int argc, char** argv) {
    std::vector<std::string> pos;
    int device = 0, gpus = 1;
    std::vector<int> devs;
    bool quiet = false, count_only = false, table = false, legacy = false;
    for (int i = 1; i < argc; i++) {
        if (!std::strcmp(argv[i], "--quiet")) quiet = true;
        else if (!std::strcmp(argv[i], "--count-only")) count_only = true;
        else if (!std::strcmp(argv[i], "--table")) table = true;
        else if (!std::strcmp(argv[i], "--legacy")) legacy = true;
        else if (!std::strcmp(argv[i], "--device") && i + 1 < argc) device = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--gpus") && i + 1 < argc) gpus = std::max(1, std::atoi(argv[++i]));
        else if (!std::strcmp(argv[i], "--devices") && i + 1 < argc) devs = parse_devices(argv[++i]);
        else pos.push_back(argv[i]);
    }
    if (pos.size() != 2) {
        std::fprintf(stderr, "usage: %s inputEBWTfileName inputPATTERNfile\n", argv[0]);
        std::fprintf(stderr, "where:\n");
        std::fprintf(stderr, "  inputEBWTfile is the BWT filename without the extension .ebwt (and .ebwt.qs for the QS string)\n");
        std::fprintf(stderr, "  inputPATTERNfile is the pattern file\n");
        return 1;
    }
    if (devs.empty()) {
        const int nd = std::max(1, edsbwt_device_count());
        for (int k = 0; k < gpus; k++) devs.push_back((device + k) % nd);
    }
    const size_t N = devs.size();
    const std::string base = pos[0], pfile = pos[1];
    std::printf("BCR_eds: %s\nBCR_eds: The input ebwt file is %s\nBCR_eds: The pattern file is %s\n", argv[0], base.c_str(), pfile.c_str());
    std::fflush(stdout);
    std::fprintf(stderr, "Backward Search\n");
    std::printf("DEBUG: 0\n");
    std::vector<Shard> sh(N);
    auto close_all = [&] {
        for (auto& x : sh) {
            if (x.occ) edsbwt_occ_free(x.occ);
            x.occ = nullptr;
            if (x.idx) edsbwt_index_close(x.idx);
            x.idx = nullptr;
        }
    };
    // one index per shard, the devices' opens in parallel (each builds its device tables).  Shards
    // that share a device (--gpus N above the device count, or a repeated --devices entry) open one
    // after another on it, each sizing its optional tables for its share of that device's HBM
    // (EDSBWT_HBM_SHARE, unless the caller set it): opened together, each would size them from the
    // whole device's free memory and the device would be oversubscribed
    std::vector<int> udev;
    size_t per_dev = 0;
    for (int d : devs)
        if (std::find(udev.begin(), udev.end(), d) == udev.end()) udev.push_back(d);
    for (int d : udev) per_dev = std::max<size_t>(per_dev, (size_t)std::count(devs.begin(), devs.end(), d));
    if (per_dev > 1 && !std::getenv("EDSBWT_HBM_SHARE")) {
        char share[32];
        std::snprintf(share, sizeof share, "%.4f", 0.9 / (double)per_dev);
        setenv("EDSBWT_HBM_SHARE", share, 1);
    }
    each(udev.size(), [&](size_t g) {
        for (size_t k = 0; k < N; k++) {
            if (devs[k] != udev[g]) continue;
            sh[k].device = devs[k];
            sh[k].rc = edsbwt_index_open(base.c_str(), devs[k], 8, &sh[k].idx);
            if (sh[k].rc) sh[k].err = edsbwt_last_error();
        }
    });
    for (auto& x : sh)
        if (x.rc) {
            std::fprintf(stderr, "%s\n", x.err.c_str());
            close_all();
            return 1;
        }
    edsbwt_index* idx = sh[0].idx;
    edsbwt_index_info info;
    edsbwt_index_get_info(idx, &info);
    std::printf("\nFrom %s_info.aux file:\n\tNumber of sequences: %llu\n\tTotal length (with $): %llu\n\tSize alpha: %u\n\tAlphabet: ",
                base.c_str(), (unsigned long long)info.n_words, (unsigned long long)info.n_rows, info.sigma);
    for (uint32_t j = 0; j < info.sigma; j++) std::printf("%c\t", info.alphabet[j]);
    std::printf("\nNUM OF EOF%llu\n", (unsigned long long)info.n_words);
    {
        // tableOcc (sigma x sigma u32 after the header and the EOF ids of <base>_info.aux,
        // da_to_everything.cpp:249-254), printed as recoverInfo prints it
        // (header: u32 N, u32 W, u8 sigma, sigma alphabet bytes — 4-byte dataTypeNChar and
        // dataTypeNSeq, Parameters.h:65-71 — then W u32 EOF ids).  A short or unreadable file ends
        // the run as recoverInfo's failed fread does (MOVE_EDSBWTSearch.cpp:751-755: message, exit
        // EXIT_FAILURE, before the table is printed)
        const std::string fn = base + "_info.aux";
        FILE* fi = std::fopen(fn.c_str(), "rb");
        std::vector<uint32_t> tocc((size_t)info.sigma * info.sigma);
        const long at = 9L + (long)info.sigma + 4L * (long)info.n_words;
        long fsz = -1;
        if (fi && std::fseek(fi, 0, SEEK_END) == 0) fsz = std::ftell(fi);
        const bool ok = fi && fsz >= at + 4L * (long)tocc.size() && std::fseek(fi, at, SEEK_SET) == 0 &&
                        std::fread(tocc.data(), 4, tocc.size(), fi) == tocc.size();
        if (fi) std::fclose(fi);
        if (!ok) {
            std::fflush(stdout);
            std::fprintf(stderr, "Error reading tableOcc%s.\n", fn.c_str());
            close_all();
            return EXIT_FAILURE;
        }
        std::printf("\nFrom %s file (TableOcc):\n", fn.c_str());
        for (uint32_t j = 0; j < info.sigma; j++) {
            for (uint32_t h = 0; h < info.sigma; h++) std::printf("%u\t", tocc[(size_t)j * info.sigma + h]);
            std::printf("\n");
        }
    }
    std::printf("size= %llu\nBitVector size: %llu\n", (unsigned long long)info.n_rows, (unsigned long long)info.n_words);
    // the pattern file, read into page-locked memory; the library splits its lines
    // (std::getline semantics, :111) on the device
    FILE* f = std::fopen(pfile.c_str(), "rb");
    if (!f) {
        std::fprintf(stderr, "Error opening %s\n", pfile.c_str());
        close_all();
        return 1;
    }
    std::fseek(f, 0, SEEK_END);
    const long fsz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    const uint64_t len = fsz > 0 ? (uint64_t)fsz : 0;
    char* text = nullptr;
    uint32_t* counts = nullptr;
    auto fail = [&](const char* msg) {
        std::fprintf(stderr, "%s\n", msg);
        if (counts) edsbwt_host_free(counts);
        if (text) edsbwt_host_free(text);
        close_all();
        return 1;
    };
    if (edsbwt_host_alloc(len + 1, (void**)&text)) {
        std::fclose(f);
        return fail(edsbwt_last_error());
    }
    const bool read_ok = !len || std::fread(text, 1, len, f) == len;
    std::fclose(f);
    if (!read_ok) return fail(("Error reading " + pfile).c_str());
    // line starts: the shards' contiguous line ranges (as even as N divides the lines) and
    // their byte ranges
    uint64_t nlines = 0;
    std::vector<uint64_t> starts{0};
    for (const char* q = text; (q = (const char*)std::memchr(q, '\n', (size_t)(text + len - q))) != nullptr; q++) {
        nlines++;
        starts.push_back((uint64_t)(q + 1 - text));
    }
    if (len && text[len - 1] != '\n') nlines++;
    else starts.pop_back();  // (the trailing '\n' opens no line)
    starts.push_back(len);   // starts[nlines] = end of the file
    for (size_t k = 0; k < N; k++) {
        sh[k].line0 = nlines * k / N;
        sh[k].nlines = nlines * (k + 1) / N - sh[k].line0;
        sh[k].b0 = starts[sh[k].line0];
        sh[k].b1 = starts[sh[k].line0 + sh[k].nlines];
    }
    if (edsbwt_host_alloc((nlines + 1) * 4, (void**)&counts)) return fail(edsbwt_last_error());
    const std::string out = pfile + (legacy ? "output.csv" : "output_M_LF.csv");
    FILE* fo = std::fopen(out.c_str(), "wb");
    if (!fo) return fail(("ERROR opening file " + out + " to write output").c_str());
    std::fputs(legacy ? "#Pat\t$_i\tD[i]\tS_j\tS_j[r]\n" : "#Pat\t$_i\tD[i]\tS_j\tS_j[r] \n", fo);
    const uint32_t flags = count_only ? EDSBWT_COUNT_ONLY
                                      : (EDSBWT_LOCATE | (table ? EDSBWT_LOCATE_TABLE : 0) | (legacy ? EDSBWT_LEGACY_ORDER : 0));
    // setup before the clock, as the reference loads its index and M_LF before :109: each device's
    // pipeline, buffers and record arena sized for its shard (edsbwt_prepare: synthetic lines of the
    // shard's mean length, none of the pattern file's)
    if (std::getenv("EDSBWT_CLI_NO_PREPARE") == nullptr) {
        each(N, [&](size_t k) {
            Shard& x = sh[k];
            if (x.nlines && edsbwt_prepare(x.idx, x.b1 - x.b0, x.nlines, 0, flags)) { x.rc = -1; x.err = edsbwt_last_error(); }
        });
        for (auto& x : sh)
            if (x.rc) {
                std::fclose(fo);
                return fail(x.err.c_str());
            }
    }
    const auto t0 = std::chrono::steady_clock::now();
    // the pattern loop: every shard's lines on its own device, concurrently
    each(N, [&](size_t k) {
        Shard& x = sh[k];
        if (!x.nlines) return;
        x.rc = edsbwt_search_lines(x.idx, text + x.b0, x.b1 - x.b0, (uint32_t)(x.line0 + 1), flags, counts + x.line0, x.nlines, &x.npat,
                                   &x.occ, &x.nocc);
        if (x.rc) x.err = edsbwt_last_error();
        else if (x.npat != x.nlines) { x.rc = EDSBWT_E_FORMAT; x.err = "line count mismatch"; }
    });
    uint64_t npat = 0, nocc = 0;
    for (auto& x : sh) {
        if (x.rc) {
            std::fclose(fo);
            return fail(x.err.c_str());
        }
        npat += x.npat;
        nocc += x.nocc;
    }
    // EDSBWT_CLI_TIMES=1: the pattern loop's phases on stderr (search, CSV, console)
    const bool times = std::getenv("EDSBWT_CLI_TIMES") != nullptr;
    auto since = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
    if (times) std::fprintf(stderr, "[cli] search %.4f s (%llu patterns, %llu records, %zu shards)\n", since(), (unsigned long long)npat,
                            (unsigned long long)nocc, N);
    if (nocc) {
        // the rows go straight to the file: each shard's rows sized, then formatted per thread range
        // and pwrite()n at the shard's offset after the header (edsbwt_write_csv) — no buffer of the
        // whole CSV, shards in parallel
        std::fflush(fo);
        const long at = std::ftell(fo);
        const int thr = std::max(1, 16 / (int)N);
        each(N, [&](size_t k) { sh[k].csv_at = sh[k].nocc ? edsbwt_format_csv(sh[k].occ, sh[k].nocc, nullptr, 0, thr) : 0; });
        uint64_t o = at < 0 ? 0 : (uint64_t)at;
        for (auto& x : sh) {
            const uint64_t n = x.csv_at;
            x.csv_at = o;
            o += n;
        }
        bool ok = at >= 0;
        if (ok)
            each(N, [&](size_t k) {
                if (sh[k].nocc && edsbwt_write_csv(sh[k].occ, sh[k].nocc, fileno(fo), sh[k].csv_at, thr) < 0) sh[k].rc = -1;
            });
        for (auto& x : sh) ok = ok && x.rc == 0;
        if (!ok) {
            std::fclose(fo);
            return fail(("ERROR writing file " + out).c_str());
        }
    }
    std::fclose(fo);
    if (times) std::fprintf(stderr, "[cli] csv written %.4f s\n", since());
    // the console stream: which patterns reach the locate loop (the pattern without its first
    // character occurs, or the pattern is one character long) — one more count-only search,
    // sharded as the first
    std::vector<uint8_t> reach;
    if (!quiet && npat) {
        char* suf = nullptr;
        uint32_t* c2 = nullptr;
        if (edsbwt_host_alloc(len + npat + 1, (void**)&suf) || edsbwt_host_alloc((npat + 1) * 4, (void**)&c2)) return fail(edsbwt_last_error());
        uint64_t sl = 0;
        std::vector<uint32_t> plen(npat);
        std::vector<uint64_t> sstart(npat + 1);
        for (uint64_t i = 0; i < npat; i++) {
            const char* q = text + starts[i];
            const char* nl = (const char*)std::memchr(q, '\n', (size_t)(text + len - q));
            const char* end = nl ? nl : text + len;
            plen[i] = (uint32_t)(end - q);
            sstart[i] = sl;
            if (end > q + 1) { std::memcpy(suf + sl, q + 1, (size_t)(end - q - 1)); sl += (uint64_t)(end - q - 1); }
            suf[sl++] = '\n';
        }
        sstart[npat] = sl;
        each(N, [&](size_t k) {
            Shard& x = sh[k];
            if (!x.nlines) return;
            uint64_t n2 = 0, no2 = 0;
            edsbwt_occ* o2 = nullptr;
            x.rc = edsbwt_search_lines(x.idx, suf + sstart[x.line0], sstart[x.line0 + x.nlines] - sstart[x.line0], 1, EDSBWT_COUNT_ONLY,
                                       c2 + x.line0, x.nlines, &n2, &o2, &no2);
            if (x.rc) x.err = edsbwt_last_error();
            else if (n2 != x.nlines) { x.rc = EDSBWT_E_FORMAT; x.err = "line count mismatch"; }
            edsbwt_occ_free(o2);
        });
        for (auto& x : sh)
            if (x.rc) {
                edsbwt_host_free(c2);
                edsbwt_host_free(suf);
                return fail(x.err.c_str());
            }
        reach.resize(npat);
        for (uint64_t i = 0; i < npat; i++) reach[i] = plen[i] == 1 || (plen[i] > 1 && c2[i] > 0);
        edsbwt_host_free(c2);
        edsbwt_host_free(suf);
    }
    uint64_t found = 0;
    if (quiet) {
        for (uint64_t i = 0; i < npat; i++) found += counts[i] > 0;
    } else {
        for (uint64_t i = 0; i < npat; i++) {
            const char* line = text + starts[i];
            const char* nl = (const char*)std::memchr(line, '\n', (size_t)(text + len - line));
            const size_t pl = (size_t)((nl ? nl : text + len) - line);
            const bool ok = counts[i] > 0;
            found += ok;
            std::fputs("Pattern: ", stdout);
            std::fwrite(line, 1, pl, stdout);
            std::printf(" of length %zu\n", pl);
            if (reach[i]) std::printf("num occ %u\n", counts[i]);
            std::fflush(stdout);
            std::fputs("OCCORRENZA DI: ", stderr);
            std::fwrite(line, 1, pl, stderr);
            std::fputs(ok ? " TROVATA\n" : " NON TROVATA\n", stderr);
        }
    }
    if (times) std::fprintf(stderr, "[cli] console loop done %.4f s\n", since());
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("bs took:%g", secs);
    std::fflush(stdout);
    std::fprintf(stderr, "\ncount_found = %llu\ncount_not_found = %llu\n", (unsigned long long)found, (unsigned long long)(npat - found));
    std::fprintf(stderr, count_only ? "\nThe search is finished! \n" : "\nThe csv file is ready! \n");
    std::fprintf(stderr, "The End!\n");
    edsbwt_host_free(counts);
    edsbwt_host_free(text);
    close_all();
    return 1;  // mainMove_EDSBWT.cpp:61
}
