// eds-bwt_amd/csrc/engine.hip — device index + batch search orchestrator + C ABI.
//
// Replaces, for the MOVE_EDSBWTSearch path of riccardo-nozza/EDS-BWT:
//   recoverInfo / retrieve_MLF / bitvector load  MOVE_EDSBWTSearch.cpp:23-95,178-218,628-770
//   build_MLF (M_LF + rank/select over L')        build_MLF.cpp:53-164
//   the pattern loop + backwardSearch             MOVE_EDSBWTSearch.cpp:97-155,228-374
//   link / dollars_in_interval / pdf              MOVE_EDSBWTSearch.cpp:512-625
//   locate (position recovery)                    MOVE_EDSBWTSearch.cpp:328-369
//
// The state of backwardSearch after its last q steps depends only on the last q
// pattern characters, so the batch is processed as a trie of reversed patterns,
// one depth per launch group: every distinct pattern suffix is searched once.
// DESIGN.md §Search walks through the phases and why each equals the reference.
#include <hipcub/hipcub.hpp>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <dlfcn.h>
#include <rccl/rccl.h>  // (types only: librccl.so is dlopen'ed by the native exchange, edsbwt_comm_init)
#include <execinfo.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <condition_variable>
#include <deque>
#include <tuple>
#include <exception>
#include <functional>
#include <thread>
#include <unordered_map>
#include <vector>

#include "index_io.h"
#include "kernels.hip"

// format.cpp: the 2-bit packer of fixed-length pattern lines (host side of k_unpack_lines)
extern "C" uint64_t edsbwt_lines_fixed(const uint8_t* s, uint64_t nb, uint32_t* L_out);
extern "C" int edsbwt_pack_lines(const uint8_t* s, uint64_t nb, uint32_t L, uint64_t p0, uint64_t p1, const uint8_t* end, uint8_t* out);

#ifndef EDSBWT_BUILD_ID
#define EDSBWT_BUILD_ID "unknown"
#endif

namespace edsbwt {

static thread_local std::string g_err;

// EDSBWT_SEGV_TRACE=1 (diagnostics): a fault in the process prints the faulting thread's native
// frames (library offsets: addr2line -f -C -e libedsbwt.so <offset>) to stderr, then the handler
// that was installed before (e.g. Python's faulthandler) runs
static struct sigaction g_old_act[32];
static void segv_trace(int sig, siginfo_t* si, void* uc) {
    char head[160];
    const int n0 = std::snprintf(head, sizeof head, "[edsbwt] signal %d at address %p in thread %ld (pid %d)\n", sig, si ? si->si_addr : nullptr,
                                 (long)syscall(SYS_gettid), (int)getpid());
    if (n0 > 0) (void)!write(2, head, (size_t)n0);
    void* fr[64];
    const int n = backtrace(fr, 64);
    backtrace_symbols_fd(fr, n, 2);
    Dl_info di{};
    if (dladdr((void*)&segv_trace, &di) && di.dli_fbase) {
        const int m = std::snprintf(head, sizeof head, "[edsbwt] libedsbwt.so base %p\n", di.dli_fbase);
        if (m > 0) (void)!write(2, head, (size_t)m);
    }
    struct sigaction& o = g_old_act[sig & 31];
    sigaction(sig, &o, nullptr);
    if (o.sa_flags & SA_SIGINFO) {
        if (o.sa_sigaction) { o.sa_sigaction(sig, si, uc); return; }
    } else if (o.sa_handler != SIG_DFL && o.sa_handler != SIG_IGN) {
        o.sa_handler(sig);
        return;
    }
    raise(sig);
}
__attribute__((constructor)) static void segv_trace_install() {
    const char* e = std::getenv("EDSBWT_SEGV_TRACE");
    if (!e || !*e || *e == '0') return;
    for (int sig : {SIGSEGV, SIGBUS, SIGFPE, SIGILL}) {
        struct sigaction a{};
        a.sa_sigaction = segv_trace;
        a.sa_flags = SA_SIGINFO | SA_ONSTACK;
        sigemptyset(&a.sa_mask);
        sigaction(sig, &a, &g_old_act[sig & 31]);
    }
}

struct Fail : std::runtime_error {
    int code;
    Fail(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};
// a depth of the batch outgrew 32-bit counts: search() retries it in trie-subtree groups
struct TooBig : Fail {
    explicit TooBig(const std::string& m) : Fail(EDSBWT_E_UNSUPPORTED, m) {}
};

// hipcub / rocPRIM take int item counts: a count past 2^31 - 1 is refused (TooBig: a search
// retries in trie-subtree groups) rather than wrapping negative
static inline int cub_n(uint64_t n) {
    if (n > 0x7fffffffull) throw TooBig("hipcub call over more than 2^31-1 items");
    return (int)n;
}

#define HIPCHK(x)                                                                                 \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess)                                                                     \
            throw Fail(EDSBWT_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_));          \
    } while (0)

// device bytes the engines' DBufs hold (this process), and per index_open the most that open held
// at once (edsbwt_index_info::open_peak_bytes): the open running on a thread tracks its own
// allocations and frees (thread_local), so concurrent opens on other threads (the CLI's --gpus N
// opens its indexes in parallel) neither inflate nor hide it
struct MemTrack {
    int64_t live = 0, peak = 0;
};
struct DevMem {
    static inline std::atomic<uint64_t> live{0};
    static inline thread_local MemTrack* track = nullptr;
    static void add(uint64_t n) {
        live.fetch_add(n);
        if (track) {
            track->live += (int64_t)n;
            track->peak = std::max(track->peak, track->live);
        }
    }
    static void sub(uint64_t n) {
        live.fetch_sub(n);
        if (track) track->live -= (int64_t)n;
    }
};

template <class T>
struct DBuf {
    T* p = nullptr;
    size_t cap = 0;
    DBuf() = default;
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    DBuf(DBuf&& o) noexcept : p(o.p), cap(o.cap) { o.p = nullptr; o.cap = 0; }
    DBuf& operator=(DBuf&& o) noexcept {
        if (this != &o) { release(); p = o.p; cap = o.cap; o.p = nullptr; o.cap = 0; }
        return *this;
    }
    ~DBuf() { release(); }  // index_close frees the HBM the index and its workspace hold
    void ensure(size_t n) {
        if (n <= cap && p) return;
        if (p) { (void)hipFree(p); DevMem::sub(cap * sizeof(T)); p = nullptr; cap = 0; }
        size_t c = std::max<size_t>(n, 1024);
        if (hipMalloc(&p, c * sizeof(T)) != hipSuccess) {
            p = nullptr;
            throw Fail(EDSBWT_E_NOMEM, "hipMalloc of " + std::to_string(c * sizeof(T)) + " bytes failed");
        }
        cap = c;
        DevMem::add(c * sizeof(T));
        if (poison()) { (void)hipMemsetD32((hipDeviceptr_t)p, poison_value(), c * sizeof(T) / 4); (void)hipDeviceSynchronize(); }
    }
    // EDSBWT_POISON=<u32> (debugging): fresh allocations are filled with that 32-bit word
    // (0 or empty: 0xA5A5A5A5) so a read of memory no kernel wrote shows up as a parity
    // failure instead of depending on what the allocator hands back
    static bool poison() {
        static const bool on = std::getenv("EDSBWT_POISON") != nullptr;
        return on;
    }
    static uint32_t poison_value() {
        static const uint32_t v = [] {
            const uint32_t x = (uint32_t)std::strtoul(std::getenv("EDSBWT_POISON"), nullptr, 0);
            return x ? x : 0xA5A5A5A5u;
        }();
        return v;
    }
    // grow keeping contents (archive)
    void grow_keep(size_t n, hipStream_t s) {
        if (n <= cap && p) return;
        size_t c = std::max<size_t>({n, cap + cap / 2, 1024});
        T* q = nullptr;
        if (hipMalloc(&q, c * sizeof(T)) != hipSuccess) {
            // the 1.5x headroom does not fit beside the old buffer: exactly n, or fail
            (void)hipGetLastError();
            c = std::max<size_t>(n, 1024);
            if (hipMalloc(&q, c * sizeof(T)) != hipSuccess) {
                (void)hipGetLastError();
                throw Fail(EDSBWT_E_NOMEM, "hipMalloc (grow) of " + std::to_string(c * sizeof(T)) + " bytes failed (" +
                                               std::to_string(cap * sizeof(T)) + " held)");
            }
        }
        if (poison()) { (void)hipMemsetD32((hipDeviceptr_t)q, poison_value(), c * sizeof(T) / 4); (void)hipDeviceSynchronize(); }
        DevMem::add(c * sizeof(T));
        if (p) {
            HIPCHK(hipMemcpyAsync(q, p, cap * sizeof(T), hipMemcpyDeviceToDevice, s));
            HIPCHK(hipStreamSynchronize(s));
            (void)hipFree(p);
            DevMem::sub(cap * sizeof(T));
        }
        p = q;
        cap = c;
    }
    void release() {
        if (p) {
            (void)hipFree(p);
            DevMem::sub(cap * sizeof(T));
        }
        p = nullptr;
        cap = 0;
    }
};

// KC_DEEP: k_deep_fast (and the deep stage's small helpers); KC_DEEPQ: k_deep (queued patterns,
// register lists); KC_DEEPW: k_deep_wide
enum KClass { KC_TRIE = 0, KC_NODES, KC_EXPAND, KC_LINK, KC_LINKSORT, KC_STEP, KC_MERGE, KC_FINISH, KC_DEEP, KC_LOCPREP, KC_LOCATE, KC_SCAN,
              KC_TABLE, KC_DEEPQ, KC_DEEPW, KC_COUNT };
static const char* kKNames[KC_COUNT] = {"trie_sort", "trie_nodes", "expand", "link", "link_sort", "step", "merge", "finish",
                                        "deep", "locate_prep", "locate", "scan", "table", "deep_list", "deep_wide"};
// k_deep keeps at most kDeepK intervals per list in registers (C3 sweep, 1x MI355X: K=2 1.08e9,
// K=3 1.20e9, K=4 1.21e9, K=8 1.15e9 patterns/s; longer lists retry in k_deep_wide)
constexpr int kDeepK = 4;
// switch to k_deep once depth-D nodes >= kDeepShare x patterns of length >= D
constexpr double kDeepShare = 0.5;
// ... and once a depth's lists average at most kDeepItems intervals per node
constexpr double kDeepItems = 2.0;
// ... and text items (count-only level walks) stop being made once they average at most this many
// (C5 with the level start table, profiles/r04_ab_c5_*.json: at the first cutover-eligible depth
// 973 ms, at 32 per node 989 ms)
constexpr double kTextStopItems = 1e30;
// locate samples every 2^kSampleShift positions of a word (16 B per sampled row).  0: every
// row, 16 B/row (C3: 1.66 GB of the 288 GB), and locate reads one sample per occurrence with
// no LF walk and no occ-block read; EDSBWT_SAMPLE_SHIFT=2 keeps 1 in 4 (0.43 GB at C3)
constexpr uint32_t kSampleShift = 0;
// patterns k_deep<kDeepK> cannot hold retry with lists of up to kDeepWide intervals
constexpr int kDeepWide = 64;
// k-mer start table: deepest depth tried, most D-mers (offsets) and intervals kept, and the
// shallowest depth worth a table
constexpr double kKtabK = 15;  // D-mer ids stay below 2^32 (B^15 = 2^30 for B = 4)
constexpr uint64_t kKtabMaxEntries = 1ull << 31;  // 8 GiB of offsets at most
constexpr double kKtabItems = 268435456.0;  // at least 2^28 intervals (2 GiB) ...
constexpr double kKtabHbmShare = 0.15;      // ... or as many as kKtabHbmShare of the free HBM holds at
constexpr double kKtabBuildBytes = 40.0;    // the build's transient bytes per interval (capture + sort)
constexpr uint32_t kKtabMinDepth = 2;
// the whole-table walk's transient bytes per K-mer (the trie of B^K patterns: keys, sort buffers,
// nodes, items of two depths) and the share of the free HBM it may take before the table is built
// group by group (build_ktab_grouped: C3's 4^15 15-mers in 16 walks of 4^13)
constexpr double kKtabWalkBytes = 100.0;
constexpr double kKtabWalkShare = 0.25;
// the wide k-mer entries (32 B per D-mer) are built when the free HBM exceeds this many times their bytes
constexpr double kKt1WideHbmShare = 2.5;
// per-'#'-row link rows (KIdx::eofrow) up to this size (C3 243 MB; C5's 264M words would take 17 GB: not built)
constexpr double kEofRowMaxBytes = 2.0e9;
// deep level start table (build_ltab): deepest depth tried, most L-mers, and the share of the
// free HBM (after every other table) its intervals may take (C5: depth 8, ~9.5G intervals, 76 GB)
constexpr double kLtabK = 8;
constexpr uint64_t kLtabMaxEntries = 1ull << 20;
constexpr double kLtabHbmShare = 0.5;  // (the share of the free HBM named above)
// ... and no deeper than B^(K-1) <= kKtabOver * N: most longer D-mers do not occur (an
// entry is 12 B; C2, 12.5M rows: depth 15 = 12.9 GB of the 288 GB, searches 4.6x faster
// than at depth 11)
constexpr double kKtabOver = 64.0;
// levels2() result meaning "the batch needs the ordered path"
constexpr uint32_t kNeedOrdered = 0xFFFFFFFFu;

struct Engine;
// Occurrence buffers handed out by search_host are page-locked and owned by their engine,
// which reuses one once edsbwt_occ_free gives it back; a buffer still held by the caller
// when its engine moves on (a new call, close) is detached and freed by edsbwt_occ_free.
struct OccRegistry {
    std::mutex m;
    std::unordered_map<const void*, std::pair<Engine*, bool>> own;  // buffer -> (engine or null, checked out)
};
static OccRegistry& occ_registry() {
    static OccRegistry r;
    return r;
}

// ---- RCCL, loaded on first use (edsbwt_comm_init): dlopen'ed with local binding, so a process that
// already holds another RCCL (PyTorch's own) keeps its symbols apart from this library's calls
struct Rccl {
    decltype(&ncclGetUniqueId) get_id = nullptr;
    decltype(&ncclCommInitRank) init = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) err = nullptr;
    bool ok = false;
    static Rccl& get() {
        static Rccl r = [] {
            Rccl x;
            void* h = nullptr;
            for (const char* n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
                if ((h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
            if (!h) return x;
            x.get_id = (decltype(x.get_id))dlsym(h, "ncclGetUniqueId");
            x.init = (decltype(x.init))dlsym(h, "ncclCommInitRank");
            x.destroy = (decltype(x.destroy))dlsym(h, "ncclCommDestroy");
            x.send = (decltype(x.send))dlsym(h, "ncclSend");
            x.recv = (decltype(x.recv))dlsym(h, "ncclRecv");
            x.group_start = (decltype(x.group_start))dlsym(h, "ncclGroupStart");
            x.group_end = (decltype(x.group_end))dlsym(h, "ncclGroupEnd");
            x.err = (decltype(x.err))dlsym(h, "ncclGetErrorString");
            x.ok = x.get_id && x.init && x.destroy && x.send && x.recv && x.group_start && x.group_end && x.err;
            return x;
        }();
        return r;
    }
};
#define NCCLCHK(x)                                                                                        \
    do {                                                                                                  \
        ncclResult_t r_ = (x);                                                                            \
        if (r_ != ncclSuccess) throw Fail(EDSBWT_E_DEVICE, std::string(#x) + ": " + Rccl::get().err(r_)); \
    } while (0)

struct Engine {
    int device = 0;
    hipStream_t stream = nullptr;
    uint32_t* pinned = nullptr;  // host scalars
    // index
    uint32_t N = 0, W = 0, S = 0, sigma = 0;
    uint8_t alpha[16] = {0};
    uint32_t C[8] = {0};
    uint64_t device_bytes = 0;
    DBuf<OccBlock> occ;
    DBuf<uint32_t> eof_seg, eof_word, seg_of_word, seg_start, seg_lo, da, offt, segtab;
    DBuf<uint32_t> seg_chain;  // bit s: seg_lo[s] != s - 1 (k_run_flags gathers seg_lo only there)
    DBuf<uint32_t> eof_key;    // [W] eof_seg[k] << 1 | chain bit of that segment (0: segment 1): KIdx::link_seg
    DBuf<uint32_t> eofrow;     // [W][16] per-'#'-row link rows (KIdx::eofrow; sigma <= 7, W * 64 B <= kEofRowMaxBytes)
    // the segment link table in 128-B rows with the text-item entries of KIdx::segtext (sigma <= 5;
    // EDSBWT_SEGTEXT=0: 64-B rows, none); filled after the per-row text entries (build_segtext)
    bool segtab_wide = false, have_segtext = false;
    DBuf<uint32_t> kpos;  // '#'-row rank of each word (inverse of eof_word): legacy output order
    DBuf<uint8_t> code_of;
    uint8_t h_code_of[256];
    bool have_table = false;
    // words' text for the single-row compare (k_text_build): reversed 2-bit text, per-row text
    // position, per-word whole-word row; built with dense samples when sigma - 1 <= 4
    DBuf<uint64_t> rtext;
    DBuf<uint32_t> gpos, wrow;
    uint64_t tlen = 0;
    bool have_text = false;
    bool kt1_pos = false;  // k_ktab_one's one-row entries carry the row's text position (kernels.h KIdx)
    bool text_deep = env_double("EDSBWT_TEXT_DEEP", 1) != 0;
    bool text_on = true;     // per search (EDSBWT_NO_TEXT, the walk and table locate modes clear it)
    DBuf<uint4> samples;     // locate samples (word, offset, segment, word in segment) of rows whose offset % 2^kSampleShift == 0
    bool have_samples = false;
    uint32_t samp_shift = 0;  // rows sampled: offset % 2^samp_shift == 0 (0: every row)
    // k-mer start table (build_ktab): for every D-mer x over the non-'#' symbols, the
    // order-free walk's intervals after its D characters, [ktab_off[x], ktab_off[x+1]) of
    // ktab_b / ktab_e; searches whose patterns are all longer than D start at depth D
    uint32_t ktab_depth = 0;
    uint64_t ktab_items = 0;
    uint64_t ktab_entries = 0;  // B^ktab_depth
    bool use_direct = true;     // direct start from the table (EDSBWT_NO_DIRECT turns it off)
    bool direct_sort = env_double("EDSBWT_DIRECT_SORT", 1) != 0;  // direct start: patterns sorted by D-mer
    bool use_packed = env_double("EDSBWT_DIRECT_PACKED", 1) != 0;  // ... carrying index + remaining symbols
    // (default -1: 16 bits, or input order with the wide k-mer table — C3, round 3: 1.96 ms
    // against 2.22 sorted, the deep walk equal: a wide entry brings what the order shared)
    // ... by the D-mer's leading bits (C3 A/B, round 1: 20 bits 2.67e9, 30 2.52e9, 12 2.43e9; round 2:
    // 16 bits 3.115 ms against 20 bits 3.145)
    int direct_sort_bits_env = (int)env_double("EDSBWT_DIRECT_SORT_BITS", -1);
    int sort_bits() const { return direct_sort_bits_env >= 0 ? direct_sort_bits_env : ktab_wide.p ? 0 : 16; }
    // ... for batches of at least this many patterns (C3 pipeline chunks: 7.84 ms per call against
    // 7.92-8.06 sorting every chunk)
    uint64_t direct_sort_min = (uint64_t)env_double("EDSBWT_DIRECT_SORT_MIN", 2000000);
    bool keys_packed = env_double("EDSBWT_KEYS_PACKED", 1) != 0;
    bool acgt_alpha = false;
    // direct(): lengths assumed rather than measured (deferred); a batch that failed the guess
    // turns it off for this index (mixed-length batches then measure first, as before)
    bool len_guess = env_double("EDSBWT_LEN_GUESS", 1) != 0, guessed_len = false;  // the alphabet is {#, A, C, G, T}: k_keys_acgt (EDSBWT_KEYS_SWAR=0: k_keys_packed)
    bool keys_swar = env_double("EDSBWT_KEYS_SWAR", 1) != 0;
    bool locate_pp = env_double("EDSBWT_LOCATE_TASKS", 0) == 0;  // deferred path: per-pattern locate
    DBuf<uint32_t> lbig;  // patterns with more than kLocBig records (k_locate_big)
    // edsbwt_search_device_ids: the #Pat of batch pattern i is pat_ids[i] (device; null: first_id + i)
    const uint32_t* pat_ids = nullptr;
    DBuf<uint64_t> pv_in, pv_out;
    DBuf<uint32_t> bhist, bscan;  // direct start buckets (k_keys histogram, its scan / scatter cursors)
    // (measured on C3, 10M patterns: k_keys' histogram atomics +0.2 ms and the scatter 0.69 ms
    // against 0.34 ms for the radix sort: off by default)
    bool use_buckets = env_double("EDSBWT_BUCKETS", 0) != 0;
    bool split_scans = env_double("EDSBWT_SPLIT_SCANS", 0) != 0;  // tests: locate offsets by two scans
    DBuf<uint32_t> ktab_off, ktab_b, ktab_e;
    DBuf<uint64_t> ktab_one;  // per D-mer: its one interval inline, else list length and offset (k_ktab_one)
    DBuf<uint4> ktab_wide;    // ... or the wide form, 32 or 64 B per D-mer (k_ktab_wide; replaces ktab_one)
    uint32_t kt1_ws = 2;      // its uint4s per D-mer (KIdx::kt1_ws)
    DBuf<uint4> srow;         // per-row text-compare entries, 32 B per row (k_srow; KIdx::srow)
    DBuf<uint4> seglink;      // k_deep_direct's link lines, 128 B per segment (k_seglink; KIdx::seglink)
    // deep level start table (build_ltab; kernels.hip k_ltab_*): every L-mer's walk items after
    // its L characters, in lt_G groups by the L-mer's last characters (x mod lt_G); a level walk
    // whose patterns are all at least L long starts at depth L from it (C5: L = 8)
    uint32_t lt_depth = 0, lt_G = 0, lt_EG = 0;
    uint64_t lt_items = 0;
    DBuf<uint32_t> lt_off;                       // [lt_G][lt_EG + 1] u32 offsets within the group
    std::vector<DBuf<uint32_t>> lt_b, lt_e;      // per group: interval starts / ends
    DBuf<const uint32_t*> lt_pb, lt_pe;          // device arrays of the groups' pointers
    DBuf<unsigned long long> lt_total;           // k_ltab_count's batch total
    bool use_ltab = true;                        // per search (EDSBWT_NO_LTAB, EDSBWT_NO_KTAB clear it)
    // most start items one level-table start takes before the batch goes to trie-subtree groups
    // (EDSBWT_LTAB_START_MAX: tests force the grouped retry with a small value)
    uint64_t lt_start_max = (uint64_t)env_double("EDSBWT_LTAB_START_MAX", 2147483647.0);
    bool use_ktab = true;  // per search (EDSBWT_NO_KTAB clears it)
    // rank entries (build_rank_entries, kernels.h): one 16-B load per interval end and step;
    // rent2 (sigma <= 5) answers two steps
    DBuf<uint4> rent1, rent2, rent3;
    // host-pipeline calls also leave every pattern's u32 count in this device array (the
    // multi-GPU exchange gathers them over RCCL without copying them back up; nullptr: off)
    uint32_t* counts_mirror = nullptr;
    uint64_t counts_mirror_cap = 0;
    DBuf<uint4> rk16, rk16sup;  // all-symbol rank entries (sigma <= 5; kernels.h): the level step's ranks
    bool use_rk16 = env_double("EDSBWT_NO_RANK16", 0) == 0;
    DBuf<uint32_t> pc3;
    uint32_t r2stride = 0, r3stride = 0;
    bool use_triples = env_double("EDSBWT_NO_TRIPLES", 0) == 0;
    bool use_rent = env_double("EDSBWT_NO_RANK_ENTRIES", 0) == 0;
    uint32_t PC[kPairCodes + 3] = {0};
    bool use_pairs = true;  // per search (EDSBWT_NO_PAIRS clears it)
    // levels2() capture mode (table build): the items of the deepest depth <= K whose
    // count fits the budget, as (D-mer index, b, e)
    struct Capture {
        uint32_t K = 0, B = 0;
        uint64_t budget = 0;
        bool only_last = false;  // keep depth K's items only (the level table's groups)
        uint32_t reached = 0;    // deepest depth whose items stayed within the budget
        uint32_t depth = 0;
        uint64_t n = 0;
        DBuf<uint32_t> k, b, e;
    };
    Capture* cap = nullptr;
    DBuf<uint32_t> kt_kid, kt_cnt, kt_pos;
    // workspace
    DBuf<uint32_t> len, perm, perm2, slen, lcp, nid[2], flag, scan, node_first, node_parent, child_first, child_end;
    DBuf<uint8_t> node_char;
    DBuf<uint64_t> child_info;  // per parent node: first child | live-child symbol mask << 32
    DBuf<uint64_t> keys, kc, kc2, skey;
    DBuf<uint32_t> ib[2], ie[2], iu[2], ioff[2], iend[2], iocb, ioce;
    DBuf<uint32_t> hcnt, hoff, rflag, rscan, rb, re, ru, doff, dend, docb, doce;
    DBuf<uint64_t> lkeys, lkeys2;
    DBuf<uint32_t> tcnt, toff, tb, te, tu, tflag, tscan, cb, ce, cu, mflag, mscan;
    DBuf<uint32_t> fcnt, foff, node_occ;
    DBuf<uint32_t> ab, ae;
    DBuf<Res> res, sub_res, g_res;  // per-pattern results (kernels.h Res)
    DBuf<uint64_t> occ64, oscan, tc64, tscan64, tout;
    DBuf<uint32_t> trow, tpat;
    DBuf<uint64_t> blk_first;  // per kLocRun records: the task holding the first (k_tasks -> k_locate)
    DBuf<edsbwt_occ> rec, rec2;
    DBuf<uint64_t> lk, lk2;                 // legacy_order keys
    DBuf<uint32_t> lp, lp2, li, li2;
    DBuf<unsigned long long> counters;
    DBuf<uint8_t> tmp;      // hipcub temp storage
    DBuf<unsigned long long> lhist;
    DBuf<uint32_t> ovf_orig, ovf_scan, sub_map;
    DBuf<uint64_t> sub_len, sub_off;
    DBuf<uint8_t> sub_bytes, fin;
    DBuf<uint32_t> lcnt, ck_u, ck_k, ck_e, gcnt, gfill, goff, gend, gb, gee, fv, fv2, fend, hterm;
    DBuf<uint64_t> fk, fk2, ekeys, efk;
    DBuf<uint32_t> eu, eb, ee, eck_u, eck_k, eck_e, efv, shpre;
    DBuf<uint32_t> fu, fb, fe, fpre;  // the previous depth's item shards, read in place by k_lvl_items
    // run_grouped: group of each pattern, its members as a sub-batch
    DBuf<uint32_t> glen, gid, gflag, gscan, g_map;
    // path tags (EDSBWT_PATH_TAGS=1, tests): per pattern of the last edsbwt_search_device call,
    // the EDSBWT_PATH_* bits of the kernels it went through (edsbwt_last_paths)
    bool tag_paths = env_double("EDSBWT_PATH_TAGS", 0) != 0, tag_now = false;
    DBuf<uint8_t> ptag;
    uint64_t ptag_n = 0;
    const uint32_t* tag_map = nullptr;  // grouped search: group index -> batch index
    void tag_queue(const uint4* q, const uint32_t* qcnt, uint32_t qcap, uint32_t bit) {
        if (!tag_now) return;
        hipLaunchKernelGGL(k_tag_queue, dim3((unsigned)std::min<uint64_t>(65535, ((uint64_t)qcap * NSHARD + 255) / 256)), dim3(256), 0,
                           stream, q, qcnt, qcap, (const uint32_t*)perm.p, tag_map, ptag.p, bit);
        HIPCHK(hipGetLastError());
    }
    void tag_list(const uint32_t* list, uint64_t cap, uint32_t bit) {
        if (!tag_now || !cap) return;
        hipLaunchKernelGGL(k_tag_list, dim3((unsigned)std::min<uint64_t>(65535, (cap + 255) / 256)), dim3(256), 0, stream, list, cap,
                           (const uint32_t*)perm.p, tag_map, ptag.p, bit);
        HIPCHK(hipGetLastError());
    }
    DBuf<uint64_t> g_len, g_off;
    DBuf<uint8_t> g_bytes;
    DBuf<uint4> dq;                   // k_deep_fast -> k_deep queue (pattern, depth, b, e), sharded
    DBuf<uint64_t> dq2;               // ... and, for the packed direct start, each entry's packed start
    DBuf<uint32_t> dqpre;
    // One page-locked, device-mapped, coherent host block holds pinned, pinned_big,
    // pinned_stats and a staging area: the search's small transfers are copied by a kernel
    // (small_copy) on the engine stream, because a DMA copy would queue behind the host
    // pipeline's bulk uploads / downloads on the copy engines and stall the search
    uint8_t* hostblk = nullptr;
    uint8_t* hostblk_dev = nullptr;
    size_t hostblk_size = 0;
    static constexpr size_t kStageBytes = 256 << 10;
    uint8_t* hstage = nullptr;
    uint32_t* pinned_big = nullptr;  // host shard counters + prefix
    DBuf<unsigned long long> stats;  // kStatSlots sharded statistics counters (stat_add)
    unsigned long long* pinned_stats = nullptr;
    // sum of the kStatShards shards of each statistic, from pinned_stats (already copied)
    uint64_t trace_single = 0, trace_lines = 0;  // EDSBWT_TRACE: stats at the previous depth's print
    std::vector<uint64_t> fold_pinned_stats() const {
        std::vector<uint64_t> v(kStatStride, 0);
        for (uint32_t s = 0; s < kStatShards; s++)
            for (uint32_t k = 0; k < kStatStride; k++) v[k] += pinned_stats[s * kStatStride + k];
        return v;
    }
    // the search workspace sized by the k-mer table build (B^D patterns): given back after it,
    // so an open index holds its tables only and searches size the workspace to their batches
    void release_workspace() {
        for (auto* b : {&len, &perm, &perm2, &slen, &lcp, &nid[0], &nid[1], &flag, &scan, &node_first, &node_parent, &child_first,
                        &child_end, &ib[0], &ib[1], &ie[0], &ie[1], &iu[0], &iu[1], &ioff[0], &ioff[1], &iend[0], &iend[1], &iocb, &ioce,
                        &hcnt, &hoff, &rflag, &rscan, &rb, &re, &ru, &doff, &dend, &docb, &doce, &tcnt, &toff, &tb, &te, &tu, &tflag,
                        &tscan, &cb, &ce, &cu, &mflag, &mscan, &fcnt, &foff, &node_occ, &ab, &ae, &trow, &tpat, &lp, &lp2, &li, &li2,
                        &ovf_orig, &ovf_scan, &sub_map, &lcnt, &ck_u, &ck_k, &ck_e, &gcnt, &gfill, &goff, &gend, &gb, &gee, &fv, &fv2,
                        &fend, &hterm, &eu, &eb, &ee, &eck_u, &eck_k, &eck_e, &efv, &shpre, &fu, &fb, &fe, &fpre, &glen, &gid, &gflag,
                        &gscan, &g_map, &dqpre, &kt_kid, &kt_cnt, &kt_pos})
            b->release();
        for (auto* b : {&keys, &kc, &kc2, &skey, &child_info, &lkeys, &lkeys2, &occ64, &oscan, &tc64, &tscan64, &tout, &blk_first, &lk,
                        &lk2, &sub_len, &sub_off, &fk, &fk2, &ekeys, &efk, &g_len, &g_off, &dq2, &pv_in, &pv_out, &tile_sum, &tile_pre})
            b->release();
        for (auto* b : {&node_char, &tmp, &sub_bytes, &fin, &g_bytes}) b->release();
        res.release(); sub_res.release(); g_res.release();
        rec.release(); rec2.release();
        dq.release();
    }
    // ---- host pipeline (search_host): batches in host memory are cut into chunks; chunk k+1
    // is uploaded on `up` while chunk k is searched on `stream` and chunk k-1's counts and
    // records go back on `down` (two device slots per buffer, events between the streams)
    hipStream_t up = nullptr, down = nullptr;
    // chunk k reuses chunk k-kSlots's device buffers, so its search waits for that chunk's
    // download: five slots keep the searches clear of a download backlog
    static constexpr int kSlots = 5;
    hipEvent_t up_done[kSlots] = {}, comp_done[kSlots] = {}, down_done[kSlots] = {}, prep_done[kSlots] = {};
    // per-slot prep on `up` after each upload: the chunk's lines split (lines mode) or its offsets
    // rebased, and its pattern count and longest / shortest pattern measured, so the search
    // itself reads nothing back before its final check
    DBuf<uint32_t> nlcnt_s[kSlots], nlpre_s[kSlots];
    DBuf<uint8_t> ptmp[kSlots];
    DBuf<unsigned long long> prep_mm[kSlots];
    uint32_t* prep_host(int sl) { return pinned + 64 + 8 * sl; }  // P, max, ~min as u64 (in hostblk)
    DBuf<uint8_t> hraw[kSlots], hbytes[kSlots], hpack[kSlots];  // hpack: a packed chunk (k_unpack_lines)
    DBuf<uint64_t> hoffs[kSlots];
    DBuf<uint32_t> hcounts[kSlots], nlcnt, nlpre;
    DBuf<edsbwt_occ> hrec[kSlots];
    struct Pinned {  // page-locked host staging (inputs or counts in pageable caller memory)
        void* p = nullptr;
        size_t cap = 0;
        void ensure(size_t n) {
            if (n <= cap && p) return;
            if (p) (void)hipHostFree(p);
            p = nullptr;
            cap = 0;
            if (hipHostMalloc(&p, std::max<size_t>(n, 1 << 20), hipHostMallocDefault) != hipSuccess) {
                p = nullptr;
                throw Fail(EDSBWT_E_NOMEM, "hipHostMalloc of " + std::to_string(n) + " bytes failed");
            }
            cap = std::max<size_t>(n, 1 << 20);
        }
        void release() { if (p) (void)hipHostFree(p); p = nullptr; cap = 0; }
    };
    Pinned stage_in[kSlots], stage_off[kSlots], stage_cnt[kSlots], stage_pack[kSlots], stage_c8[kSlots], stage_exc[kSlots];
    DBuf<uint8_t> hc8[kSlots];  // a chunk's counts as bytes, then the number of larger ones (k_counts_u8)
    DBuf<uint2> hexc[kSlots];   // ... and those: (pattern, count)
    // the occurrence records handed to the caller (library-owned, page-locked, reused once
    // edsbwt_occ_free gives them back: see occ_arena_*)
    edsbwt_occ* arena = nullptr;
    size_t arena_cap = 0;
    edsbwt_stats st{};
    // profiling
    bool prof = false;
    bool no_wide = false;
    bool count_only = false;  // current search returns counts only (no interval archive at finishing depths)
    // count only: the level step sums finishing nodes' occurrences itself (EDSBWT_FUSE_FINISH=0: k_fin_emit, A/B)
    bool fuse_finish = env_double("EDSBWT_FUSE_FINISH", 1) != 0;
    // ... and walks single rows as text items (kernels.hip kTextItem; EDSBWT_TEXT_ITEMS=0: off, A/B)
    bool text_items = env_double("EDSBWT_TEXT_ITEMS", 1) != 0;
    // link keys carry their segment's chain bit (KIdx::link_cb; EDSBWT_LINK_CB=0: eof_seg keys, A/B)
    bool link_cb_on = env_double("EDSBWT_LINK_CB", 1) != 0;
    // deep cutover thresholds (EDSBWT_DEEP_SHARE / EDSBWT_DEEP_ITEMS override, for tuning)
    double deep_share = env_double("EDSBWT_DEEP_SHARE", kDeepShare);
    double deep_items = env_double("EDSBWT_DEEP_ITEMS", kDeepItems);
    // text items stop being made when a cutover-eligible depth's lists average at most this many
    // intervals per node (EDSBWT_TEXT_STOP; the default 1e30: at the first cutover-eligible depth, as round 3)
    double text_stop_items = env_double("EDSBWT_TEXT_STOP", kTextStopItems);
    // direct start only from tables whose lists average at most this many intervals per D-mer
    double direct_items = env_double("EDSBWT_DIRECT_ITEMS", kDeepItems);
    uint32_t deep_k = [] {  // register list length of k_deep: 2, 3, 4 or 8
        const uint32_t k = (uint32_t)env_double("EDSBWT_DEEP_K", kDeepK);
        return k == 2 || k == 3 || k == 4 || k == 8 ? k : (uint32_t)kDeepK;
    }();
    uint32_t force_groups = (uint32_t)env_double("EDSBWT_FORCE_GROUPS", 0);  // tests: always search in trie-subtree groups
    uint32_t sticky_groups = 0;  // grouping depth a previous batch on this index needed
    static double env_double(const char* name, double dflt) {
        const char* v = std::getenv(name);
        return v && *v ? std::atof(v) : dflt;
    }  // EDSBWT_NO_WIDE (tests): overflowed deep patterns go straight to the level path
    uint32_t prof_mask = ~0u;  // kernel classes timed with events when profiling
    bool trace = std::getenv("EDSBWT_TRACE") != nullptr;
    // EDSBWT_TRACE=2: host time of every launch inside a search (what the host spends per call)
    bool trace2 = env_double("EDSBWT_TRACE", 0) >= 2;
    std::chrono::steady_clock::time_point t_search0;
    void hmark(const char* what) {
        if (trace2)
            std::fprintf(stderr, "[edsbwt]   +%7.1f us %s\n",
                         std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_search0).count(), what);
    }
    void hmark_kern(const void* kern) {
        if (!trace2) return;
        Dl_info di{};
        hmark(kern && dladdr(kern, &di) && di.dli_sname ? di.dli_sname : "?");
    }
    struct Ev { int k; hipEvent_t a, b; };
    std::vector<Ev> evs, ev_pool;
    // deferred checks (direct start): the search runs without read-backs between its stages;
    // what they decided ('#' in a pattern, overflow lists, record totals) is read once at the
    // end, and a batch that fails a check is searched again on the checked path
    bool defer_ok = env_double("EDSBWT_NO_DEFER", 0) == 0;  // per call (cleared for a redo)
    bool defer = false;                                      // the current search deferred its checks
    bool defer_call = false;                                 // ... may defer them (set by search())
    static constexpr uint32_t kFlagNoDefer = 0x80000000u;    // internal flag: the checked path
    uint32_t defer_wide_cap = 0;
    const uint32_t* defer_ovf2 = nullptr;
    // fused counts (deferred direct start, count-only or per-pattern locate): k_deep_direct, k_deep
    // and k_deep_wave write every final count into the caller's counts and add found / occurrences
    // / intervals into the stats shards that k_gather_checks folds, so finish_deferred runs no
    // k_count_found pass over the results (EDSBWT_FUSED_COUNTS=0: the pass)
    bool fused_counts = env_double("EDSBWT_FUSED_COUNTS", 1) != 0;
    bool locate_counts = env_double("EDSBWT_LOCATE_COUNTS", 0) != 0;
    bool tile_scan = env_double("EDSBWT_TILE_SCAN", 1) != 0;
    // EDSBWT_LOC_FC=1: located searches have the deep kernels write the counts too (as count-only
    // searches do), and sum the record-offset tiles from those 4-B counts (k_tile_sums) instead of
    // the 16-B results (k_count_tiles) — slower at C3: 1.459-1.467 against 1.443-1.461 ms, the deep
    // kernels' count stores cost 0.035 ms, the tile pass saves less (profiles/r06_ab_c3_loc_fc.txt)
    bool loc_fc = env_double("EDSBWT_LOC_FC", 0) != 0;
    // k_locate_pp's LDS record stage (512 or 1024 records; 512 lets 8 blocks share a CU: the
    // locate class 0.190 against 0.189 ms at C3, profiles/r04_ab_locstage_c3_*.json — not the bound)
    uint32_t loc_stage = (uint32_t)env_double("EDSBWT_LOC_STAGE", 1024);
    DBuf<uint64_t> tile_sum, tile_pre;  // per-pattern locate: occurrences per 64-pattern tile, and their exclusive scan
    uint32_t* fc_counts = nullptr;  // this search's counts when the deep kernels write them
    // (round 5 also summed the per-pattern locate's record-offset tiles inside the deep kernels: C3 1.85 /
    // 1.83 ms against 1.69 ms with k_count_tiles, k_deep_direct 1.11 against 0.96 ms —
    // profiles/r05_ab_c3_tile_fuse_*.json — so that path was removed)
    // the level walk's located results with dense samples: k_locate_lists (a wave per pattern, records
    // from the lists directly); EDSBWT_LOCATE_LISTS=0: tasks + k_locate (C5 located step: see DESIGN §6)
    bool locate_lists = env_double("EDSBWT_LOCATE_LISTS", 1) != 0;
    // the direct start's deep kernels with their per-lane work counters (steps, lines, text rows: the
    // line model of bench.py's roofline); off for a call with EDSBWT_NO_COUNTERS (or every call with
    // EDSBWT_DEEP_STATS=0): the builds without them (k_deep_direct 8 waves fused, k_deep 6 waves)
    bool deep_stats_env = env_double("EDSBWT_DEEP_STATS", 1) != 0;
    bool deep_stats = true;  // (this call's)
    bool fc_done = false;           // ... and k_deep_direct took them
    static constexpr uint32_t kWideCap = 16384;
    static constexpr uint32_t kWaveGrid = 2048;  // k_deep_wave's waves (each strides over the wide list)
    // wide lists one wavefront per pattern (k_deep_wave); EDSBWT_DEEP_WAVE=0: one lane per pattern (k_deep_wide, A/B)
    bool deep_wave = env_double("EDSBWT_DEEP_WAVE", 1) != 0;
    // k_deep_fast's register budget: waves per SIMD (5 unbounded; 6 without scratch; 8 spills)
    int deep_waves = (int)env_double("EDSBWT_DEEP_WAVES", 6);
    // the packed start with the wide table: k_deep_direct (EDSBWT_DEEP_DIRECT=0: k_deep_fast), held
    // to EDSBWT_DIRECT_WAVES waves per SIMD
    bool deep_direct = env_double("EDSBWT_DEEP_DIRECT", 1) != 0;
    // the level step (k_lvl_items, k_lvl_dollar): 7 waves per SIMD (SGPR-bound) or 8 (arguments
    // spilled to VGPR lanes)
    int lvl_waves = (int)env_double("EDSBWT_LVL_WAVES", 7);
    // (7 since the walk returns to the text compare: 72 VGPRs against 64 + 9 spilled at 8; C3 1.246-1.250
    // against 1.255 ms, C2 equal — profiles/r06_ab_direct_waves_back.txt)
    int direct_waves = (int)env_double("EDSBWT_DIRECT_WAVES", 7);
    // ... and computes the pattern keys itself, no k_keys_acgt (EDSBWT_FUSED_KEYS=0: off, A/B); the
    // fused launch's inputs, set by direct() for run_deep
    bool fused_keys = env_double("EDSBWT_FUSED_KEYS", 1) != 0;
    struct FusedKeys {
        bool on = false;
        const uint8_t* bytes = nullptr;
        const uint64_t* off = nullptr;
        unsigned long long* n_term = nullptr;
        uint32_t E = 0, lmin = 0, lmax = 0;
    } fk_now;
    // k_deep<4, 3> likewise (5 or 6; C3 0.371 / 0.478 ms against 0.369 unbounded, profiles/r03_ab_occupancy.txt);
    // 1: the unbounded builds (k_deep<4, 3, 1>, <4, 4, 1>, the '#'-row link rows' <4, 3, 1, true>) —
    // every build is run through the parity tests (tests/test_gpu_parity.py::test_k_deep_builds_gpu)
    // (round 5, 32-bit queue indices: 6 waves 0.294-0.301 ms against 0.310-0.316 at 5 and 0.71 at 8,
    // profiles/r05_ab_c3_deepq_waves_568.txt)
    int deepq_waves = (int)env_double("EDSBWT_DEEPQ_WAVES", 6);
    // locate tasks one wave per pattern when lists average more than kTasksWaveRatio intervals
    // (EDSBWT_TASKS_WAVE=0: k_tasks, one lane per pattern, always)
    static constexpr uint64_t kTasksWaveRatio = 8;
    int tasks_wave = (int)env_double("EDSBWT_TASKS_WAVE", 1);  // (2: always — tests)
    // located finishers at the level table's start take their archive ranges straight from the
    // emitted (row-sorted) items (EDSBWT_LT_FIN_DIRECT=0: k_fin_emit + sort, as at other depths)
    bool lt_fin_direct = env_double("EDSBWT_LT_FIN_DIRECT", 1) != 0;
    // k_deep takes two characters per rank entry when no interval of its list meets a link
    // (rent2, as k_deep_direct; EDSBWT_DEEPQ_PAIRS=0: one character per step)
    uint32_t deepq_pairs = env_double("EDSBWT_DEEPQ_PAIRS", 1) != 0 ? 1u : 0u;
    // the packed direct start's k_deep build without the generic key reader (k_deep<.., PACKED>)
    bool deepq_packed = env_double("EDSBWT_DEEPQ_PACKED", 1) != 0;
    // k_deep_direct returns to the text compare when a rank step leaves one row (k_deep_direct<.., BACK>)
    bool direct_back = env_double("EDSBWT_DIRECT_BACK", 1) != 0;
    // k_deep's packed build filters a list start of single rows by their text (KIdx::deep_filter)
    bool deepq_filter = env_double("EDSBWT_DEEPQ_FILTER", 1) != 0;
    unsigned loc_blocks = (unsigned)env_double("EDSBWT_LOC_BLOCKS", 0);
    unsigned loc_ppt = (unsigned)env_double("EDSBWT_LOC_PPT", 2);
    // a located deferred direct-start search sums its record-offset tiles (k_count_tiles) on the second
    // stream beside k_deep_wave, leaving out the patterns k_deep_wave walks (a bitmap, k_mark_wide);
    // k_tile_fix adds those after both (EDSBWT_WAVE_TILES=0: k_count_tiles after k_deep_wave).  C3
    // 1.373-1.387 against 1.392-1.396 ms with bench.py's e2e leg first in the process — with the second
    // stream created at open; created on first use (inside the host pipeline, after its copy streams)
    // it made the step 1.55-1.73 ms (profiles/r06_ab_c3_wave_tiles.txt)
    bool wave_tiles = env_double("EDSBWT_WAVE_TILES", 1) != 0;
    DBuf<uint32_t> wbits;           // the bitmap (zero between searches: k_count_tiles clears what it read)
    uint64_t wbits_words = 0;
    uint32_t* early_counts = nullptr;  // this search's counts when the early tiles may run (search())
    bool in_direct = false;            // run_deep called from the direct start (nothing writes results after it)
    bool tiles_early = false;          // the early tiles were queued (finish_deferred joins them)
    hipEvent_t tiles_ev = nullptr, tiles_ev0 = nullptr;
    // the library stream waits for the early tiles (before anything else may touch their outputs)
    void join_early() {
        if (!tiles_early) return;
        HIPCHK(hipStreamWaitEvent(stream, tiles_ev, 0));
        tiles_early = false;
    }
    const uint32_t* early_ovf = nullptr;
    uint32_t early_cap = 0;
    // the deferred direct start in pieces (EDSBWT_DEEP_PIECES, batches of at least
    // EDSBWT_DEEP_PIECE_MIN patterns): k_deep_direct over piece j + 1 runs while k_deep walks piece
    // j's queue on a second stream (an event per piece), so k_deep's long-tailed lanes share the
    // GPU with the next piece's direct walk instead of running after the whole batch
    uint32_t deep_pieces = std::max(1u, std::min(16u, (uint32_t)env_double("EDSBWT_DEEP_PIECES", 1)));
    uint64_t deep_piece_min = (uint64_t)env_double("EDSBWT_DEEP_PIECE_MIN", 1 << 20);
    hipStream_t stream2 = nullptr;  // (created on first use)
    // native RCCL exchange (edsbwt_comm_init / edsbwt_gather_counts): the communicator, its stream,
    // and the gathers still reading a count buffer (a search writing that buffer waits for them)
    ncclComm_t comm = nullptr;
    int comm_rank = 0, comm_size = 0;
    hipStream_t xs = nullptr;
    struct PendingGather {
        const void* p = nullptr;
        hipEvent_t ev = nullptr;
    };
    PendingGather gathers[4];
    uint32_t gather_next = 0;
    hipEvent_t xs_after = nullptr;
    // the search stream waits for the queued gathers that read buffer p (the caller alternates
    // buffers, so normally for one that ended a step ago)
    void wait_gathers_on(const void* p) {
        if (!p) return;
        for (auto& g : gathers)
            if (g.p == p) HIPCHK(hipStreamWaitEvent(stream, g.ev, 0));
    }
    std::vector<hipEvent_t> piece_ev;
    DBuf<uint32_t> pcnt;  // queue counters of the pieces (NSHARD * 32 per piece)
    uint32_t wide_cap = (uint32_t)env_double("EDSBWT_WIDE_CAP", kWideCap);  // (tests: small caps force redos)
    uint64_t defer_cap = (uint64_t)env_double("EDSBWT_DEFER_CAP", 0);        // (tests: record / task buffer caps)
    // pinned + 32..: the deferred checks' landing slots (u32 words)
    static constexpr uint32_t kChkTerm = 0, kChkOvf = 2, kChkOvf2 = 3, kChkOflow = 4, kChkFound = 6, kChkSums = 8;
    uint32_t* chk() { return pinned + 32; }
    double occ_per_pat = 0, tasks_per_pat = 0;  // record and task rates seen so far (deferred buffer sizing)
    // lengths of the batch's patterns measured by the caller (host pipeline prep): no k_lminmax read-back
    bool known_len = false;
    uint32_t known_lmin = 0, known_lmax = 0;

    // bits needed for values 0..v
    static uint32_t bits_for(uint64_t v) {
        uint32_t b = 1;
        while (b < 64 && (v >> b)) b++;
        return b;
    }
    KIdx kidx() const {
        KIdx X{};  // (every field set below; value-initialised so a new one cannot reach a kernel unset)
        X.occ = occ.p;
        X.eof_seg = eof_seg.p;
        X.eofrow = eofrow.p;
        // (segment ids below 2^31: the chain bit fits beside them)
        X.link_cb = link_cb_on && eof_key.p && S < 0x7fffffffu ? 1u : 0u;
        X.link_seg = X.link_cb ? eof_key.p : eof_seg.p;
        X.eof_word = eof_word.p;
        X.seg_of_word = seg_of_word.p;
        X.seg_start = seg_start.p;
        X.seg_lo = seg_lo.p;
        X.da = da.p;
        X.offt = offt.p;
        X.samples = samples.p;
        X.samp_dense = have_samples && samp_shift == 0 ? 1u : 0u;
        X.segtab = segtab.p;
        X.seg_stride = (sigma <= 7 && !segtab_wide) ? 16u : 32u;
        X.seg_hi = sigma <= 7 ? 8u : 9u;
        X.segtext = have_segtext ? 1u : 0u;
        X.N = N; X.W = W; X.S = S; X.sigma = sigma;
        X.segbits = bits_for(S);
        X.rowbits = bits_for(N);
        for (int c = 0; c < 8; c++) X.C[c] = C[c];
        X.rent1 = use_rent ? rent1.p : nullptr;
        X.rent2 = use_rent && use_pairs ? rent2.p : nullptr;
        X.r2stride = r2stride;
        X.rent3 = use_rent && use_pairs && use_triples ? rent3.p : nullptr;
        X.r3stride = r3stride;
        X.PC3 = pc3.p;
        for (uint32_t k = 0; k < kPairCodes + 3; k++) X.PC[k] = PC[k];
        const bool txt = have_text && text_on && X.samp_dense;
        X.rtext = txt ? rtext.p : nullptr;
        X.tlen = tlen;
        X.gpos = gpos.p;
        X.wrow = wrow.p;
        X.srow = txt && srow.p ? (const uint4*)srow.p : nullptr;
        X.seglink = X.srow && seglink.p ? (const uint4*)seglink.p : nullptr;
        X.text_deep = text_deep ? 1u : 0u;
        X.deep_filter = deepq_filter ? 1u : 0u;
        X.kt1_pos = kt1_pos ? 1u : 0u;
        X.kt1_ws = kt1_ws;
        X.rk16 = use_rk16 ? rk16.p : nullptr;
        X.rk16sup = use_rk16 ? rk16sup.p : nullptr;
        X.kt_E = (uint32_t)std::min<uint64_t>(ktab_entries, 0xffffffffu);
        X.kt_n = (uint32_t)std::min<uint64_t>(ktab_items, 0xffffffffu);
        return X;
    }

    // ------------------------------------------------------------ helpers
    // The free HBM the index's optional tables are sized by (k-mer table budget, wide entries,
    // per-row text entries, level table): the device's free memory, and with EDSBWT_HBM_SHARE = f < 1
    // at most f of the device's memory less what this index already holds — several processes
    // sharing one GPU (bench.py's 8-rank rehearsal sets f = 1 / ranks per GPU) each size their
    // tables for their share instead of the first-come ones taking the device
    size_t hbm_free(size_t* total_out = nullptr) const {
        size_t f = 0, t = 0;
        if (hipMemGetInfo(&f, &t) != hipSuccess) { (void)hipGetLastError(); f = t = 0; }
        if (total_out) *total_out = t;
        const double share = env_double("EDSBWT_HBM_SHARE", 1.0);
        if (share > 0 && share < 1.0) {
            const double cap = share * (double)t - (double)device_bytes;
            f = std::min<size_t>(f, cap > 0 ? (size_t)cap : 0);
        }
        return f;
    }
    static unsigned grid_for(size_t n) { return (unsigned)std::max<size_t>(1, std::min<size_t>((n + 255) / 256, 16384)); }

    // timing events of an attempt that will not be reported go back to the pool
    void discard_attempt() {
        for (auto& e : evs) ev_pool.push_back(e);
        evs.clear();
    }
    Ev ev_get(int k) {
        Ev e;
        if (!ev_pool.empty()) { e = ev_pool.back(); ev_pool.pop_back(); }
        else { HIPCHK(hipEventCreate(&e.a)); HIPCHK(hipEventCreate(&e.b)); }
        e.k = k;
        return e;
    }
    template <typename F>
    void timed(int k, F&& f) {
        if (!prof || !((prof_mask >> k) & 1)) { f(); return; }
        Ev e = ev_get(k);
        HIPCHK(hipEventRecord(e.a, stream));
        f();
        HIPCHK(hipEventRecord(e.b, stream));
        evs.push_back(e);
    }
    // reductions: a fixed small grid, one global atomic per block
    static constexpr unsigned kReduceBlocks = 1024;
    template <typename K, typename... A>
    void launch_reduce(int k, K kern, A... a) {
        timed(k, [&] { hipLaunchKernelGGL(kern, dim3(kReduceBlocks), dim3(256), 0, stream, a...); });
        HIPCHK(hipGetLastError());
        hmark_kern((const void*)kern);
        sync_check((const void*)kern);
        st.launches_kernel[k]++;
    }
    template <typename K, typename... A>
    void launch(int k, K kern, size_t n, A... a) {
        if (!n) return;
        timed(k, [&] { hipLaunchKernelGGL(kern, dim3(grid_for(n)), dim3(256), 0, stream, a...); });
        HIPCHK(hipGetLastError());
        hmark_kern((const void*)kern);
        sync_check((const void*)kern);
        st.launches_kernel[k]++;
    }
    template <typename K, typename... A>
    void launch_grid(int k, K kern, unsigned blocks, A... a) {  // an explicit grid (a kernel that strides itself)
        if (!blocks) return;
        timed(k, [&] { hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, stream, a...); });
        HIPCHK(hipGetLastError());
        hmark_kern((const void*)kern);
        sync_check((const void*)kern);
        st.launches_kernel[k]++;
    }
    // EDSBWT_SYNC_CHECK=1 (debugging): wait for every launch and name the kernel that failed
    const bool sync_checks = std::getenv("EDSBWT_SYNC_CHECK") != nullptr;
    void sync_check(const void* kern, const char* label = nullptr) {
        if (!sync_checks) return;
        const hipError_t e = hipStreamSynchronize(stream);
        if (e == hipSuccess) return;
        Dl_info di{};
        const char* name = label ? label : (kern && dladdr(kern, &di) && di.dli_sname ? di.dli_sname : "?");
        std::fprintf(stderr, "[edsbwt] kernel %s failed: %s\n", name, hipGetErrorString(e));
        throw Fail(EDSBWT_E_DEVICE, std::string("kernel ") + name + ": " + hipGetErrorString(e));
    }
    uint32_t read_u32(const uint32_t* d) {
        small_copy(pinned, d, 4);
        HIPCHK(hipStreamSynchronize(stream));
        return pinned[0];
    }
    uint64_t read_u64(const void* d) {
        small_copy(pinned, d, 8);
        HIPCHK(hipStreamSynchronize(stream));
        uint64_t v;
        std::memcpy(&v, pinned, 8);
        return v;
    }
    // the deferred search's result array before a walk that leaves results unwritten (k_deep_direct
    // writes every one: its search skips the 160 MB zeroing at C3)
    bool res_unzeroed = false;
    void settle_res(const Res* r) {
        if (!res_unzeroed || r != res.p) return;  // (a group's or a subset's results have their own zeroing)
        zero(res.p, st.patterns * sizeof(Res));
        res_unzeroed = false;
    }
    // zeroing by our own kernel: hipMemsetAsync's fill kernel ran at PCIe-like rates beside the
    // host pipeline's download blits (0.4-0.7 ms for a 32 MB result array)
    void zero(void* p, size_t bytes) { zero_on(p, bytes, stream); }
    // several (4-B multiple) ranges in one launch
    void zero_many(std::initializer_list<std::pair<void*, size_t>> rs) {
        ZeroSet z{};
        uint32_t n = 0;
        uint64_t mx = 0;
        for (auto& r : rs) {
            if (!r.second) continue;
            if (n == 8) throw Fail(EDSBWT_E_ARG, "zero_many: more than 8 ranges");
            z.p[n] = static_cast<uint32_t*>(r.first);
            z.n4[n] = r.second / 4;
            mx = std::max<uint64_t>(mx, z.n4[n]);
            n++;
        }
        if (!n) return;
        const unsigned gx = (unsigned)std::min<uint64_t>(1024, std::max<uint64_t>(1, (mx + 1023) / 1024));
        hipLaunchKernelGGL(k_zero_multi, dim3(gx, n), dim3(256), 0, stream, z);
        HIPCHK(hipGetLastError());
    }
    static void zero_on(void* p, size_t bytes, hipStream_t s) {
        if (!bytes) return;
        const unsigned g = (unsigned)std::min<size_t>(2048, std::max<size_t>(1, (bytes / 16 + 255) / 256));
        hipLaunchKernelGGL(k_zero_bytes, dim3(g), dim3(256), 0, s, (uint8_t*)p, (uint64_t)bytes);
        HIPCHK(hipGetLastError());
    }
    // small transfer on the engine stream by a kernel (see hostblk); host pointers must lie in hostblk
    const void* dev_alias(const void* p) const {
        const uint8_t* q = static_cast<const uint8_t*>(p);
        return (q >= hostblk && q < hostblk + hostblk_size) ? hostblk_dev + (q - hostblk) : p;
    }
    void small_copy(void* dst, const void* src, size_t bytes) { small_copy_on(dst, src, bytes, stream); }
    void small_copy_on(void* dst, const void* src, size_t bytes, hipStream_t s) {
        if (!bytes) return;
        if (bytes % 4) throw Fail(EDSBWT_E_ARG, "small_copy of a size that is not a multiple of 4");
        const uint32_t n = (uint32_t)(bytes / 4);
        hipLaunchKernelGGL(k_copy_words, dim3(std::min<uint32_t>(64, (n + 255) / 256)), dim3(256), 0, s,
                           (const uint32_t*)dev_alias(src), (uint32_t*)const_cast<void*>(dev_alias(dst)), n);
        HIPCHK(hipGetLastError());
    }

    // reversed-code chunk of depth D for the patterns in trie order (chunk 0 is the
    // last radix pass's output, chunks 1.. were gathered by build_trie)
    uint32_t bps = 4;                // bits per symbol code of the current batch (3 or 4)
    std::vector<uint64_t> nodes_at;  // trie nodes per depth of the current batch
    const uint64_t* sorted_chunk(uint32_t D, uint64_t P) {
        const uint32_t c = (D - 1) / (64 / bps);
        return c == 0 ? kc2.p : skey.p + (size_t)(c - 1) * P;
    }

    // ---- sharded appends (kernels.hip NSHARD): per-shard counters on the host
    static constexpr uint32_t kCnt = NSHARD * 32 + 32;  // shard counters + device scalars (link runs)
    std::vector<uint32_t> hsh = std::vector<uint32_t>(kCnt, 0);
    void fetch_shards() {
        small_copy(pinned_big, lcnt.p, kCnt * 4);
        HIPCHK(hipStreamSynchronize(stream));
        std::memcpy(hsh.data(), pinned_big, kCnt * 4);
    }
    std::vector<uint32_t> shard_counts(int k) const {
        std::vector<uint32_t> v(NSHARD);
        for (uint32_t sh = 0; sh < NSHARD; sh++) v[sh] = hsh[sh * 32 + k];
        return v;
    }
    // most items one shard can receive from a launch over n inputs (<= fanout each)
    static size_t shard_bound(size_t n, size_t fanout) {
        const size_t G = grid_for(n), iters = (n + G * 256 - 1) / (G * 256);
        return ((G + NSHARD - 1) / NSHARD) * 256 * iters * fanout;
    }
    uint32_t shard_max(int k) const {
        uint32_t m = 0;
        for (uint32_t sh = 0; sh < NSHARD; sh++) m = std::max(m, hsh[sh * 32 + k]);
        return m;
    }
    uint32_t shard_total(int k) const {
        uint64_t t = 0;
        for (uint32_t sh = 0; sh < NSHARD; sh++) t += hsh[sh * 32 + k];
        if (t > 0xffffffffull) throw TooBig("more than 2^32 items at one depth");
        return (uint32_t)t;
    }
    void upload_prefix(int k) {
        uint32_t* pre = pinned_big + kCnt;
        pre[0] = 0;
        for (uint32_t sh = 0; sh < NSHARD; sh++) pre[sh + 1] = pre[sh] + hsh[sh * 32 + k];
        shpre.ensure(NSHARD + 1);
        small_copy(shpre.p, pre, (NSHARD + 1) * 4);
    }
    template <typename A, typename B, typename C>
    void unshard3(int k, size_t cap, const A* a, const B* b, const C* c, A* oa, B* ob, C* oc, uint32_t total) {
        upload_prefix(k);
        launch(KC_MERGE, k_unshard<A, B, C>, total, total, (const uint32_t*)shpre.p, (uint32_t)cap, a, b, c, oa, ob, oc);
    }
    template <typename A, typename B>
    void unshard2(int k, size_t cap, const A* a, const B* b, A* oa, B* ob, uint32_t total) {
        unshard3<A, B, uint8_t>(k, cap, a, b, (const uint8_t*)nullptr, oa, ob, (uint8_t*)nullptr, total);
    }
    template <typename A>
    void unshard1(int k, size_t cap, const A* a, A* oa, uint32_t total) {
        unshard3<A, uint8_t, uint8_t>(k, cap, a, (const uint8_t*)nullptr, (const uint8_t*)nullptr, oa, (uint8_t*)nullptr, (uint8_t*)nullptr, total);
    }
    // grow three sharded buffers from cap to ncap per shard, keeping keep[sh] items of each shard
    void regrow3(DBuf<uint32_t>& a, DBuf<uint32_t>& b, DBuf<uint32_t>& c, size_t cap, size_t ncap, const std::vector<uint32_t>& keep) {
        for (DBuf<uint32_t>* x : {&a, &b, &c}) {
            DBuf<uint32_t> n;
            n.ensure(ncap * NSHARD);
            for (uint32_t sh = 0; sh < NSHARD; sh++)
                HIPCHK(hipMemcpyAsync(n.p + sh * ncap, x->p + sh * cap, (size_t)keep[sh] * 4, hipMemcpyDeviceToDevice, stream));
            std::swap(n.p, x->p);
            std::swap(n.cap, x->cap);
            HIPCHK(hipStreamSynchronize(stream));
            n.release();
        }
    }

    // scan.p[0..P) = exclusive prefix sum of the depth-D node-start flags, computed on the fly
    void node_scan(uint32_t D, uint64_t P) {
        if (P > 0x7fffffffull) throw TooBig("scan over >2^31 items");
        using It = hipcub::TransformInputIterator<uint32_t, NodeFlag, hipcub::CountingInputIterator<uint32_t>>;
        It in(hipcub::CountingInputIterator<uint32_t>(0), NodeFlag{slen.p, lcp.p, D});
        size_t tb = 0;
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, scan.p, cub_n(P), stream));
        tmp.ensure(tb);
        timed(KC_NODES, [&] { HIPCHK(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb, in, scan.p, cub_n(P), stream)); });
        sync_check(nullptr, "hipcub call at engine.hip:396");
    }

    void sort_link_keys(const uint64_t* in, uint64_t* out, size_t n, int end_bit) {
        size_t tb = 0;
        HIPCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, in, out, cub_n(n), 0, end_bit, stream));
        tmp.ensure(tb);
        timed(KC_LINKSORT, [&] { HIPCHK(hipcub::DeviceRadixSort::SortKeys(tmp.p, tb, in, out, cub_n(n), 0, end_bit, stream)); });
        sync_check(nullptr, "link key sort");
    }

    // out[0..n) = exclusive prefix sum of in[0..n) (no read-back)
    void exclusive_scan(const uint32_t* in, uint32_t* out, size_t n) {
        if (!n) return;
        if (n > 0x7fffffffull) throw TooBig("scan over >2^31 items");
        size_t tb = 0;
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, out, cub_n(n), stream));
        tmp.ensure(tb);
        timed(KC_SCAN, [&] { HIPCHK(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb, in, out, cub_n(n), stream)); });
        sync_check(nullptr, "hipcub call at engine.hip:414");
    }

    // out[0..n] = exclusive prefix sum (out[0] = 0, out[n] = total), no read-back
    void inclusive_scan_u64(const uint64_t* in, DBuf<uint64_t>& out, size_t n, bool zero_first = true) {
        out.ensure(n + 1);
        if (zero_first) zero(out.p, 8);
        if (!n) return;
        if (n > 0x7fffffffull) throw TooBig("scan over >2^31 items");
        size_t tb = 0;
        HIPCHK(hipcub::DeviceScan::InclusiveSum(nullptr, tb, in, out.p + 1, cub_n(n), stream));
        tmp.ensure(tb);
        timed(KC_SCAN, [&] { HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp.p, tb, in, out.p + 1, cub_n(n), stream)); });
        sync_check(nullptr, "hipcub call at engine.hip:426");
    }

    // out[0..n] = exclusive prefix sum of in[0..n); returns out[n]
    uint32_t scan_u32(const uint32_t* in, DBuf<uint32_t>& out, size_t n) {
        out.ensure(n + 1);
        zero(out.p, 4);
        if (n) {
            if (n > 0x7fffffffull) throw TooBig("scan over >2^31 items");
            size_t tb = 0;
            HIPCHK(hipcub::DeviceScan::InclusiveSum(nullptr, tb, in, out.p + 1, cub_n(n), stream));
            tmp.ensure(tb);
            timed(KC_SCAN, [&] { HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp.p, tb, in, out.p + 1, cub_n(n), stream)); });
            sync_check(nullptr, "hipcub call at engine.hip:438");
        }
        return read_u32(out.p + n);
    }
    uint64_t scan_u64(const uint64_t* in, DBuf<uint64_t>& out, size_t n) {
        out.ensure(n + 1);
        zero(out.p, 8);
        if (n) {
            if (n > 0x7fffffffull) throw TooBig("scan over >2^31 items");
            size_t tb = 0;
            HIPCHK(hipcub::DeviceScan::InclusiveSum(nullptr, tb, in, out.p + 1, cub_n(n), stream));
            tmp.ensure(tb);
            timed(KC_SCAN, [&] { HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp.p, tb, in, out.p + 1, cub_n(n), stream)); });
            sync_check(nullptr, "hipcub call at engine.hip:450");
        }
        return read_u64(out.p + n);
    }

    // ------------------------------------------------------------ index
    void open(const std::string& base, int dev) {
        const auto t_open = std::chrono::steady_clock::now();
        MemTrack mt;
        struct TrackScope {
            explicit TrackScope(MemTrack* m) { DevMem::track = m; }
            ~TrackScope() { DevMem::track = nullptr; }
        } track_scope(&mt);
        device = dev;
        HIPCHK(hipSetDevice(device));
        HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        // the second stream (run_deep_pieces, the wave tiles) next to it, before the host pipeline's
        // copy streams exist (EDSBWT_STREAM2_EARLY=0: created on first use)
        if (env_double("EDSBWT_STREAM2_EARLY", 1) != 0) HIPCHK(hipStreamCreateWithFlags(&stream2, hipStreamNonBlocking));
        {
            const size_t a = 512, big = ((kCnt + 2 * (NSHARD + 8)) * 4 + 255) / 256 * 256, stb = kStatSlots * 8;
            hostblk_size = a + big + stb + kStageBytes;
            HIPCHK(hipHostMalloc((void**)&hostblk, hostblk_size, hipHostMallocMapped | hipHostMallocCoherent));
            HIPCHK(hipHostGetDevicePointer((void**)&hostblk_dev, hostblk, 0));
            pinned = reinterpret_cast<uint32_t*>(hostblk);
            pinned_big = reinterpret_cast<uint32_t*>(hostblk + a);
            pinned_stats = reinterpret_cast<unsigned long long*>(hostblk + a + big);
            hstage = hostblk + a + big + stb;
        }
        stats.ensure(kStatSlots);
        HostIndex H;
        std::string err;
        int rc = read_host_index(base, H, err);
        if (rc) throw Fail(rc, err);
        if (H.sigma > 8)
            throw Fail(EDSBWT_E_UNSUPPORTED, "alphabet of " + std::to_string(H.sigma) + " symbols (incl. '#'): the device layout supports 8");
        N = H.N; W = H.W; S = H.S; sigma = H.sigma;
        for (uint32_t j = 0; j < sigma; j++) alpha[j] = H.alpha[j];
        std::memcpy(h_code_of, H.code_of, 256);
        acgt_alpha = H.sigma == 5 && H.code_of[(uint8_t)'#'] == 0 && H.code_of[(uint8_t)'A'] == 1 && H.code_of[(uint8_t)'C'] == 2 &&
                     H.code_of[(uint8_t)'G'] == 3 && H.code_of[(uint8_t)'T'] == 4;
        if (W > N) throw Fail(EDSBWT_E_FORMAT, "more words than rows");
        // rows are u32 (Parameters.h:71); the top values mark k_deep's queue entries (kernels.hip kQNode / kQWide)
        if (N > 0xFFFFFFF0u) throw Fail(EDSBWT_E_UNSUPPORTED, "more than 2^32 - 16 BWT rows");
        // occ blocks (parallel over block ranges)
        const size_t nblk = (size_t)N / kOccRows + 1;
        std::vector<OccBlock> hb(nblk);
        std::vector<uint32_t> tot(8, 0);
        {
            unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
            std::vector<std::vector<uint32_t>> part(T, std::vector<uint32_t>(8, 0));
            auto rng = [&](unsigned t) { return std::make_pair(nblk * t / T, nblk * (t + 1) / T); };
            std::vector<std::thread> th;
            for (unsigned t = 0; t < T; t++)
                th.emplace_back([&, t] {
                    auto [b0, b1] = rng(t);
                    for (size_t b = b0; b < b1; b++) {
                        OccBlock& B = hb[b];
                        std::memset(&B, 0, sizeof B);
                        for (uint32_t r = 0; r < kOccRows; r++) {
                            size_t x = b * kOccRows + r;
                            uint32_t c = x < N ? H.code_of[H.L[x]] : 7u;
                            if (x < N) part[t][c]++;
                            B.plane[0][r >> 6] |= (uint64_t)(c & 1) << (r & 63);
                            B.plane[1][r >> 6] |= (uint64_t)((c >> 1) & 1) << (r & 63);
                            B.plane[2][r >> 6] |= (uint64_t)((c >> 2) & 1) << (r & 63);
                        }
                    }
                });
            for (auto& x : th) x.join();
            // block-start counts: each part's running counts start from the parts before it
            std::vector<std::vector<uint32_t>> base(T, std::vector<uint32_t>(8, 0));
            for (unsigned t = 1; t < T; t++)
                for (int c = 0; c < 8; c++) base[t][c] = base[t - 1][c] + part[t - 1][c];
            std::vector<std::thread> th2;
            for (unsigned t = 0; t < T; t++)
                th2.emplace_back([&, t] {
                    auto [b0, b1] = rng(t);
                    std::vector<uint32_t> run = base[t];
                    for (size_t b = b0; b < b1; b++) {
                        for (int c = 0; c < 8; c++) hb[b].cnt[c] = run[c];
                        for (uint32_t r = 0; r < kOccRows; r++) {
                            size_t x = b * kOccRows + r;
                            if (x < N) run[H.code_of[H.L[x]]]++;
                        }
                    }
                });
            for (auto& x : th2) x.join();
            for (int c = 0; c < 8; c++) tot[c] = base[T - 1][c] + part[T - 1][c];
        }
        uint32_t acc = 0;
        for (uint32_t c = 0; c < 8; c++) { C[c] = acc; acc += tot[c]; }
        if (tot[0] != W) throw Fail(EDSBWT_E_FORMAT, "number of '#' rows != nText");
        // segments
        std::vector<uint32_t> sow(W), sst(S + 2, 0), slo(S + 2, 0), eseg(W);
        std::vector<uint8_t> has_empty(S + 2, 0);
        {
            uint32_t s = 0;
            for (uint32_t w = 0; w < W; w++) {
                if ((H.bv[w >> 6] >> (w & 63)) & 1) { s++; sst[s] = w; }
                sow[w] = s;
                if (H.L[w] == '#') has_empty[s] = 1;  // row w is the '#'-suffix of word w
            }
            sst[S + 1] = W;
            // link from a word of segment s >= 2 covers segments [seg_lo[s], s-1]: the
            // chain of dollars_in_interval pushes through empty words (:557,:620)
            for (uint32_t t = 2; t <= S; t++) {
                uint32_t v = t - 1;
                slo[t] = (v >= 2 && has_empty[v]) ? slo[v] : v;
            }
            for (uint32_t k = 0; k < W; k++) {
                uint32_t sg = sow[H.eof_id[k]];
                eseg[k] = sg >= 2 ? sg : 0;
            }
        }
        auto up = [&](auto& buf, const auto& v) {
            using T = typename std::decay_t<decltype(v)>::value_type;
            buf.ensure(v.size());
            HIPCHK(hipMemcpy(buf.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
            device_bytes += v.size() * sizeof(T);
        };
        up(occ, hb);
        up(eof_seg, eseg);
        up(eof_word, H.eof_id);
        {
            std::vector<uint32_t> kp(W);
            for (uint32_t t = 0; t < W; t++) kp[H.eof_id[t]] = t;
            up(kpos, kp);
        }
        up(seg_of_word, sow);
        up(seg_start, sst);
        h_seg_of_word = sow;  // the host pipeline's record expansion (search_host)
        h_seg_start = sst;
        up(seg_lo, slo);
        {
            std::vector<uint32_t> chain(((size_t)S + 2 + 31) / 32, 0u);
            for (uint32_t t = 2; t <= S; t++)
                if (slo[t] != t - 1) chain[t >> 5] |= 1u << (t & 31);
            up(seg_chain, chain);
            std::vector<uint32_t> ek(W);
            for (uint32_t k = 0; k < W; k++) ek[k] = eseg[k] ? eseg[k] << 1 | (slo[eseg[k]] != eseg[k] - 1 ? 1u : 0u) : 0u;
            up(eof_key, ek);
        }
        std::vector<uint8_t> co(H.code_of, H.code_of + 256);
        up(code_of, co);
        counters.ensure(32);
        {  // segment link table (k_deep)
            segtab_wide = sigma <= 5 && env_double("EDSBWT_SEGTEXT", 1) != 0;
            const KIdx X0 = kidx();
            segtab.ensure((size_t)(S + 2) * X0.seg_stride);
            device_bytes += (size_t)(S + 2) * X0.seg_stride * 4;
            launch(KC_TABLE, k_segtab, (size_t)S + 2, S, kidx(), segtab.p);
            // k_deep's links from '#' rows: one line per row instead of eof_seg then segtab
            // (C3: 3.8M words, 243 MB; EDSBWT_EOF_ROWS=0: off)
            if (X0.seg_hi == 8 && (double)W * 64 <= kEofRowMaxBytes && env_double("EDSBWT_EOF_ROWS", 0) != 0) {
                eofrow.ensure((size_t)W * 16);
                launch(KC_TABLE, k_eofrow, (size_t)W * 16, W, (const uint32_t*)eof_seg.p, (const uint32_t*)segtab.p, X0.seg_stride, eofrow.p);
                device_bytes += (size_t)W * 64;
            }
            HIPCHK(hipStreamSynchronize(stream));
        }
        if (env_double("EDSBWT_LOCATE_SAMPLES", 1.0) != 0.0) build_samples();
        build_rank_entries();
        build_ktab();
        // last: the k-mer table's interval budget is a share of the free HBM, which the 32-B
        // per-row entries would take first (C5: 40 GB, the table then one depth shallower)
        build_srow();
        build_segtext();
        build_seglink();
        // after the per-row entries: the level table's budget is a share of what HBM has left
        build_ltab();
        open_peak_bytes = (uint64_t)std::max<int64_t>(0, mt.peak);
        open_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_open).count();
        if (trace)
            std::fprintf(stderr, "[edsbwt] index open: %.2f s, %llu device bytes held, peak %llu while building\n", open_seconds,
                         (unsigned long long)device_bytes, (unsigned long long)open_peak_bytes);
    }
    uint64_t open_peak_bytes = 0;  // DevMem peak over this open (tables + transient build workspace)
    double open_seconds = 0;

    // Deep level start table: when the k-mer start table stopped shallow because its lists are
    // long (C5: depth 3, 0.87G intervals; the items per depth then grow ~1.6x per depth up to
    // depth 9), every L-mer's item list after its L characters is built too, group
    // by group (the L-mers sharing their last two characters: one walk over B^L / B^2 patterns
    // each, so the build's workspace is a group's, not the whole table's), and kept in those
    // groups with u32 offsets.  A level walk whose patterns are all >= L long then starts at
    // depth L (levels2), skipping the depths where most items and link runs are.  L is the
    // deepest <= EDSBWT_LTAB_K (default kLtabK) whose table fits kLtabHbmShare of the free HBM
    // (estimated from the first group, checked as groups complete).  EDSBWT_LTAB_K=0: off.
    void build_ltab() {
        const uint32_t B = sigma - 1;
        uint32_t L = (uint32_t)env_double("EDSBWT_LTAB_K", kLtabK);
        if (!L || B < 2 || !ktab_depth || ktab_depth + 2 > L || sigma + 2 > 8) return;
        auto pw = [&](uint32_t k) { uint64_t v = 1; for (uint32_t t = 0; t < k; t++) v *= B; return v; };
        while (L > ktab_depth + 1 && pw(L) > kLtabMaxEntries) L--;
        size_t free_b = 0, total_b = 0;
        free_b = hbm_free(&total_b);
        const double budget = env_double("EDSBWT_LTAB_SHARE", kLtabHbmShare) * (double)free_b;
        uint64_t sym = 0;
        for (uint32_t v = 0; v < B; v++) sym |= (uint64_t)alpha[v + 1] << (8 * v);
        const auto t0 = std::chrono::steady_clock::now();
        for (; L >= ktab_depth + 2; L--) {
            const uint32_t G = (uint32_t)pw(2);
            const uint64_t E = pw(L), EG = E / G;
            if (EG > 0x7fffffffull) continue;
            lt_off.ensure((size_t)G * (EG + 1));
            lt_b.clear(); lt_e.clear();
            lt_b.resize(G); lt_e.resize(G);
            uint64_t tot = 0;
            bool ok = true;
            for (uint32_t g = 0; g < G && ok; g++) {
                try {
                    DBuf<uint8_t> kb;
                    DBuf<uint64_t> ko;
                    kb.ensure(EG * L);
                    ko.ensure(EG + 1);
                    launch(KC_TABLE, k_kmer_batch, EG, EG, L, B, sym, kb.p, ko.p, (uint64_t)G, (uint64_t)g);
                    res.ensure(EG); ovf_orig.ensure(EG);
                    zero(stats.p, kStatSlots * 8);
                    Capture c;
                    // the group walk's items bounded by what the free HBM holds at the build's transient
                    // bytes per item (a walk past it stops short of depth L: this L is given up)
                    size_t fg = 0, tg = 0;
                    fg = hbm_free(&tg);
                    c.K = L; c.B = B; c.only_last = true;
                    c.budget = std::min<uint64_t>(0x7fffffffull, (uint64_t)(0.5 * (double)fg / kKtabBuildBytes));
                    cap = &c;
                    const bool was_count_only = count_only;
                    count_only = true;
                    uint64_t abase = 0;
                    try {
                        levels2(kb.p, ko.p, EG, false, res.p, abase, ovf_orig.p);
                    } catch (const TooBig&) {
                        c.depth = 0;
                    } catch (const Fail& f) {
                        // an optional table: a device allocation that fails during its build gives up
                        // this depth (a shallower one, or none, is tried) instead of failing the open
                        if (f.code != EDSBWT_E_NOMEM) { cap = nullptr; count_only = was_count_only; throw; }
                        (void)hipGetLastError();
                        c.depth = 0;
                    }
                    cap = nullptr;
                    count_only = was_count_only;
                    st = edsbwt_stats{};
                    HIPCHK(hipStreamSynchronize(stream));
                    const uint64_t n = c.n;
                    tot += n;
                    // the first group's size x G estimates the table; every group is checked as it lands
                    if (c.depth != L || (double)tot * 8 > budget || (g == 0 && (double)n * G * 8 > budget)) {
                        ok = false;
                        if (trace) std::fprintf(stderr, "[edsbwt] level table depth %u: group %u holds %llu intervals (depth %u): too large\n", L, g,
                                                (unsigned long long)n, c.depth);
                        break;
                    }
                    lt_b[g].ensure(n);
                    lt_e[g].ensure(n);
                    if (n) {
                        DBuf<uint64_t> k1, k2;
                        DBuf<uint32_t> e2;
                        k1.ensure(n); k2.ensure(n); e2.ensure(n);
                        launch(KC_TABLE, k_ktab_keys, n, n, (const uint32_t*)c.k.p, (const uint32_t*)c.b.p, k1.p);
                        c.k.release(); c.b.release();
                        size_t tb = 0;
                        const int endbit = 32 + (int)bits_for(EG);
                        HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k1.p, k2.p, c.e.p, e2.p, cub_n(n), 0, endbit, stream));
                        tmp.ensure(tb);
                        HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, k1.p, k2.p, c.e.p, e2.p, cub_n(n), 0, endbit, stream));
                        sync_check(nullptr, "hipcub call in build_ltab");
                        k1.release();
                        c.e.release();
                        launch(KC_TABLE, k_ktab_split, n, n, (const uint64_t*)k2.p, lt_b[g].p);
                        HIPCHK(hipMemcpyAsync(lt_e[g].p, e2.p, n * 4, hipMemcpyDeviceToDevice, stream));
                        launch(KC_TABLE, k_ktab_bounds, EG + 1, EG, (const uint64_t*)k2.p, n, lt_off.p + (size_t)g * (EG + 1));
                        HIPCHK(hipStreamSynchronize(stream));
                    } else {
                        zero(lt_off.p + (size_t)g * (EG + 1), (EG + 1) * 4);
                    }
                } catch (const Fail& f) {
                    // (the group's sort buffers or lists did not fit: as a walk past the budget)
                    if (f.code != EDSBWT_E_NOMEM) throw;
                    (void)hipGetLastError();
                    ok = false;
                }
            }
            if (!ok) {
                lt_b.clear(); lt_e.clear();
                lt_off.release();
                release_workspace();
                continue;
            }
            std::vector<const uint32_t*> pb(G), pe(G);
            for (uint32_t g = 0; g < G; g++) { pb[g] = lt_b[g].p; pe[g] = lt_e[g].p; }
            lt_pb.ensure(G); lt_pe.ensure(G);
            HIPCHK(hipMemcpy(lt_pb.p, pb.data(), G * sizeof(void*), hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(lt_pe.p, pe.data(), G * sizeof(void*), hipMemcpyHostToDevice));
            lt_total.ensure(1);
            lt_depth = L;
            lt_G = G;
            lt_EG = (uint32_t)EG;
            lt_items = tot;
            device_bytes += tot * 8 + (uint64_t)G * (EG + 1) * 4;
            release_workspace();
            if (trace)
                std::fprintf(stderr, "[edsbwt] level start table: depth %u, %u groups of %llu L-mers, %llu intervals, built in %.2f s\n", L, G,
                             (unsigned long long)EG, (unsigned long long)tot,
                             std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
            return;
        }
    }

    // KIdx::seglink: k_deep_direct's link from a word start reads the segment's ranks for the next
    // character and, when they give one row, that row's text-compare entry from one 128-B line
    // instead of the segment row and then the row's srow line (C3: 243 MB; EDSBWT_SEGLINK=0: off).
    // At most EDSBWT_SEGLINK_GB (default 2) GB: it is built before the level start table, whose
    // budget is a share of the HBM left (C5's 88M segments would take 11 GB of it)
    void build_seglink() {
        if (!srow.p || sigma != 5 || !segtab.p || env_double("EDSBWT_SEGLINK", 1) == 0) return;
        const size_t bytes = ((size_t)S + 2) * 128;
        if ((double)bytes > env_double("EDSBWT_SEGLINK_GB", 2) * 1073741824.0) return;
        size_t tb_ = 0;
        if ((double)hbm_free(&tb_) < 4.0 * (double)bytes) return;
        seglink.ensure(((size_t)S + 2) * 8);
        launch(KC_TABLE, k_seglink, ((size_t)S + 2) * 4, S, kidx(), seglink.p);
        HIPCHK(hipStreamSynchronize(stream));
        device_bytes += bytes;
    }

    // KIdx::segtext: each segment row's text-item entries, from the per-row text entries (k_segtext)
    void build_segtext() {
        if (!segtab_wide || !srow.p || sigma > 5) return;
        launch(KC_TABLE, k_segtext, (size_t)S + 2, S, kidx(), segtab.p);
        HIPCHK(hipStreamSynchronize(stream));
        have_segtext = true;
    }

    // Per-row text-compare entries (KIdx::srow, 32 B per row: C3 3.3 GB): with dense samples and
    // the text, a single row reached through a link is compared with the text from one line
    // instead of three (sample, text position, text window).  EDSBWT_SROW=0: off.
    void build_srow() {
        if (!have_text || !have_samples || samp_shift != 0 || !samples.p || !gpos.p || !rtext.p) return;
        if (env_double("EDSBWT_SROW", 1) == 0) return;
        size_t fb = 0, tb_ = 0;
        fb = hbm_free(&tb_);
        if ((double)fb < 4.0 * (double)N * 32) return;
        srow.ensure(2 * (size_t)N);
        launch(KC_TABLE, k_srow, N, (uint64_t)N, (const uint4*)samples.p, (const uint32_t*)gpos.p, (const uint64_t*)rtext.p,
               (uint64_t)tlen, srow.p, (const uint32_t*)seg_lo.p);
        HIPCHK(hipStreamSynchronize(stream));
        device_bytes += (size_t)N * 32;
    }

    // Rank entries (kernels.h): rent1 for every alphabet, rent2 (the pair codes of every row,
    // their 64-row counts scanned, then one entry per 32-row block and pair code) for
    // sigma <= 5, and PC[p], the first row of the suffixes c2 c1 ... (C[c2] + rank_c2(L, C[c1])).
    void build_rank_entries() {
#if EDSBWT_OCC_ROWS == 64
        const uint64_t nb32 = (uint64_t)N / 32 + 1;
        const KIdx X = kidx();
        rent1.ensure(nb32 * sigma);
        launch(KC_TABLE, k_rent1, nb32, nb32, X, rent1.p);
        device_bytes += nb32 * sigma * 16;
        if (sigma > 5 || sigma < 2) {
            HIPCHK(hipStreamSynchronize(stream));
            return;
        }
        {
            // all-symbol rank entries: 16 B per 16 rows + 16 B per 65536 rows
            const uint64_t n16 = (uint64_t)N / 16 + 1, nsup = (uint64_t)N / 65536 + 1;
            rk16.ensure(n16);
            rk16sup.ensure(nsup);
            launch(KC_TABLE, k_rk16, n16, n16, X, rk16.p);
            launch(KC_TABLE, k_rk16_sup, nsup, nsup, X, rk16sup.p);
            device_bytes += (n16 + nsup) * 16;
        }
        const uint32_t nc = 1 + (sigma - 1) * sigma;
        const uint64_t nblk = (uint64_t)N / 64 + 1, nrows = nblk * 64;
        if ((uint64_t)nc * nblk > 0x7fffffffull) return;  // scan_u32 bound
        DBuf<uint8_t> code;
        DBuf<uint32_t> cnt, cscan;
        code.ensure(nrows);
        cnt.ensure((size_t)nc * nblk);
        launch(KC_TABLE, k_pair_codes, nrows, nrows, X, code.p);
        launch(KC_TABLE, k_pair_counts, nrows, nblk, (const uint8_t*)code.p, nc, cnt.p);
        scan_u32(cnt.p, cscan, (size_t)nc * nblk);
        cnt.release();
        r2stride = nc - 1;
        rent2.ensure(nb32 * r2stride);
        launch(KC_TABLE, k_rent2, nb32, nb32, nblk, (const uint8_t*)code.p, nc, sigma, (const uint32_t*)cscan.p, rent2.p);
        device_bytes += nb32 * r2stride * 16;
        std::vector<uint32_t> rk((size_t)sigma * sigma);
        DBuf<uint32_t> d_rk;
        d_rk.ensure(rk.size());
        launch(KC_TABLE, k_pile_ranks, 1, X, d_rk.p);
        HIPCHK(hipMemcpyAsync(rk.data(), d_rk.p, rk.size() * 4, hipMemcpyDeviceToHost, stream));  // the stream is non-blocking
        HIPCHK(hipStreamSynchronize(stream));
        for (uint32_t c1 = 1; c1 < sigma; c1++)
            for (uint32_t c2 = 0; c2 < sigma; c2++) PC[1 + (c1 - 1) * sigma + c2] = C[c2] + rk[(size_t)c1 * sigma + c2];
        code.release();
        cscan.release();
        build_triples();
#endif
    }

    // rent3 (kernels.h): triple codes, their 64-row counts scanned, one entry per 32-row block
    // and (c1, c2, c3) over the non-'#' symbols; PC3 = C[c3] + rank_c3(L, PC[(c1, c2)])
    void build_triples() {
        const uint32_t B = sigma - 1, nc = 1 + B * sigma * sigma;
        const uint64_t nb32 = (uint64_t)N / 32 + 1, nblk = (uint64_t)N / 64 + 1, nrows = nblk * 64;
        // off by default: C3 A/B (3 x 20 steps) 2.73e9 with rent3 vs 2.75e9 without — the third
        // step per entry saves no time once two are taken, and rent3 costs 32 B per row
        if (env_double("EDSBWT_TRIPLES", 0) == 0 || nc > 255 || (uint64_t)nc * nblk > 0x7fffffffull) return;
        const KIdx X = kidx();
        DBuf<uint8_t> code;
        DBuf<uint32_t> cnt, cscan;
        code.ensure(nrows);
        cnt.ensure((size_t)nc * nblk);
        launch(KC_TABLE, k_triple_codes, nrows, nrows, X, code.p);
        launch(KC_TABLE, k_pair_counts, nrows, nblk, (const uint8_t*)code.p, nc, cnt.p);
        scan_u32(cnt.p, cscan, (size_t)nc * nblk);
        cnt.release();
        r3stride = B * B * B;
        rent3.ensure(nb32 * r3stride);
        launch(KC_TABLE, k_rent3, nb32, nb32, nblk, (const uint8_t*)code.p, sigma, (const uint32_t*)cscan.p, rent3.p);
        device_bytes += nb32 * r3stride * 16;
        // PC3 from the ranks at the pair pile starts PC[(c1, c2)]
        std::vector<uint32_t> rows((size_t)B * B), rk((size_t)B * B * sigma), h3(r3stride);
        for (uint32_t c1 = 1; c1 < sigma; c1++)
            for (uint32_t c2 = 1; c2 < sigma; c2++) rows[(c1 - 1) * B + (c2 - 1)] = PC[1 + (c1 - 1) * sigma + c2];
        DBuf<uint32_t> d_rows, d_rk;
        d_rows.ensure(rows.size());
        d_rk.ensure(rk.size());
        HIPCHK(hipMemcpyAsync(d_rows.p, rows.data(), rows.size() * 4, hipMemcpyHostToDevice, stream));
        launch(KC_TABLE, k_ranks_at, rows.size(), (uint32_t)rows.size(), (const uint32_t*)d_rows.p, X, d_rk.p);
        HIPCHK(hipMemcpyAsync(rk.data(), d_rk.p, rk.size() * 4, hipMemcpyDeviceToHost, stream));
        HIPCHK(hipStreamSynchronize(stream));
        for (uint32_t i = 0; i < B * B; i++)
            for (uint32_t c3 = 1; c3 < sigma; c3++) h3[i * B + (c3 - 1)] = C[c3] + rk[(size_t)i * sigma + c3];
        pc3.ensure(r3stride);
        HIPCHK(hipMemcpyAsync(pc3.p, h3.data(), h3.size() * 4, hipMemcpyHostToDevice, stream));
        HIPCHK(hipStreamSynchronize(stream));
    }

    // k-mer start table: the order-free walk run once over every K-mer of the non-'#'
    // symbols (B = sigma-1 of them), capturing the items of the deepest depth D <= K whose
    // count stays within the budget; kept as per-D-mer interval lists sorted by row.
    // EDSBWT_KTAB_K (default kKtabK, 0 = no table) and EDSBWT_KTAB_ITEMS bound it.
    void build_ktab() {
        const uint32_t B = sigma - 1;
        uint32_t K = (uint32_t)env_double("EDSBWT_KTAB_K", kKtabK);
        // the interval budget scales with the device's free HBM (EDSBWT_KTAB_ITEMS overrides)
        size_t free_b = 0, total_b = 0;
        free_b = hbm_free(&total_b);
        const double by_hbm = kKtabHbmShare * (double)free_b / kKtabBuildBytes;
        const uint64_t budget = (uint64_t)env_double("EDSBWT_KTAB_ITEMS", std::max(kKtabItems, by_hbm));
        K = std::min(K, 16u);  // a search reads a node's D-mer from its sorted key chunk 0 (>= 16 symbols)
        if (B < 1 || K < 2) return;
        auto pw = [&](uint32_t k) { uint64_t v = 1; for (uint32_t t = 0; t < k; t++) v *= B; return v; };
        // no deeper than B^(K-1) <= kKtabOver*N: most longer D-mers do not occur at all
        const uint64_t max_entries = (uint64_t)env_double("EDSBWT_KTAB_ENTRIES", (double)kKtabMaxEntries);
        const double over = env_double("EDSBWT_KTAB_OVER", kKtabOver);
        while (K > 2 && (pw(K) > max_entries || (double)pw(K - 1) > over * (double)N)) K--;
        if (pw(K) > max_entries) return;
        uint64_t sym = 0;
        for (uint32_t v = 0; v < B; v++) sym |= (uint64_t)alpha[v + 1] << (8 * v);
        // the walk over all B^K K-mers at once keeps ~kKtabWalkBytes per K-mer of transient workspace
        // (C3: 4^15 K-mers, > 100 GB): when that passes kKtabWalkShare of the free HBM the table is
        // built in B^2 groups (build_ktab_grouped); a group walk that outgrows the budget names the
        // depth it reached, and the whole-table walk runs there (C5: depth 3)
        uint32_t depth = 0;
        uint64_t n = 0;
        // (EDSBWT_KTAB_GROUPED: 0 never, 2 always — tests — else by the workspace estimate)
        const double gmode = env_double("EDSBWT_KTAB_GROUPED", 1);
        const bool grouped = B >= 2 && K >= 4 && gmode != 0 &&
                             (gmode == 2 || (double)pw(K) * kKtabWalkBytes > kKtabWalkShare * (double)free_b);
        if (grouped) {
            const uint32_t r = build_ktab_grouped(K, budget, sym);
            if (r == K) {
                depth = K;
                n = ktab_items;
            } else {
                K = std::max(2u, r);
            }
        }
        if (!depth) {
            const uint64_t P = pw(K);
            DBuf<uint8_t> kb;
            DBuf<uint64_t> ko;
            kb.ensure(P * K);
            ko.ensure(P + 1);
            launch(KC_TABLE, k_kmer_batch, P, P, K, B, sym, kb.p, ko.p, (uint64_t)1, (uint64_t)0);
            res.ensure(P); ovf_orig.ensure(P);
            zero(stats.p, kStatSlots * 8);
            Capture c;
            c.K = K; c.B = B; c.budget = budget;
            cap = &c;
            const bool was_count_only = count_only;
            count_only = true;
            uint64_t abase = 0;
            try {
                levels2(kb.p, ko.p, P, false, res.p, abase, ovf_orig.p);
            } catch (const TooBig&) {
                // a depth past the budget outgrew 32-bit counts: keep what was captured
            }
            cap = nullptr;
            count_only = was_count_only;
            st = edsbwt_stats{};
            HIPCHK(hipStreamSynchronize(stream));
            if (c.depth < kKtabMinDepth || c.n == 0) {
                release_workspace();
                return;
            }
            const uint64_t E = pw(c.depth);
            n = c.n;
            DBuf<uint64_t> k1, k2;
            DBuf<uint32_t> e2;
            k1.ensure(n); k2.ensure(n); e2.ensure(n);
            launch(KC_TABLE, k_ktab_keys, n, n, (const uint32_t*)c.k.p, (const uint32_t*)c.b.p, k1.p);
            size_t tb = 0;
            const int endbit = 32 + (int)bits_for(E);
            HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k1.p, k2.p, c.e.p, e2.p, cub_n(n), 0, endbit, stream));
            tmp.ensure(tb);
            HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, k1.p, k2.p, c.e.p, e2.p, cub_n(n), 0, endbit, stream));
            sync_check(nullptr, "hipcub call in build_ktab");
            ktab_off.ensure(E + 2);  // [E, E+1): the empty list of D-mers outside the alphabet (direct start)
            ktab_b.ensure(n);
            ktab_e.ensure(n);
            launch(KC_TABLE, k_ktab_bounds, E + 1, E, (const uint64_t*)k2.p, n, ktab_off.p);
            HIPCHK(hipMemcpyAsync(ktab_off.p + E + 1, ktab_off.p + E, 4, hipMemcpyDeviceToDevice, stream));
            launch(KC_TABLE, k_ktab_split, n, n, (const uint64_t*)k2.p, ktab_b.p);
            HIPCHK(hipMemcpyAsync(ktab_e.p, e2.p, n * 4, hipMemcpyDeviceToDevice, stream));
            depth = c.depth;
        }
        const uint64_t E = pw(depth);
        if (N < 0x80000000u) {  // inline single intervals need bit 63 free
            kt1_pos = have_text && gpos.p && N < 0x40000000u && tlen < 0x80000000ull && env_double("EDSBWT_KT1_POS", 1) != 0;
            // the wide form when a one-row entry can carry its sample and text window (dense
            // samples, the text) and HBM holds 32 B per D-mer with room to spare (C3: 4^15 D-mers,
            // 34 GB); EDSBWT_KT1_WIDE=0: the 8-B entries
            // (EDSBWT_KT1_LINK=1: 64 B per D-mer when HBM also holds that, a one-row entry then carrying
            // the link ranks of its word's segment, KIdx::kt1_ws — C3 1.434-1.446 against 1.438-1.475 ms
            // for 34 GB more index, profiles/r05_ab_c3_kt1_link.txt: the segment rows mostly hit the
            // cache; off by default)
            size_t fb = 0, tb_ = 0;
            fb = hbm_free(&tb_);
            const KIdx X0 = kidx();
            const bool link = sigma <= 5 && X0.segtab && env_double("EDSBWT_KT1_LINK", 0) != 0 &&
                              (double)fb > kKt1WideHbmShare * (double)((E + 1) * 64);
            kt1_ws = link ? 4u : 2u;
            const uint64_t wide_b = (E + 1) * 16 * kt1_ws;
            const bool wide = kt1_pos && have_samples && samp_shift == 0 && samples.p && rtext.p &&
                              (double)fb > kKt1WideHbmShare * (double)wide_b && env_double("EDSBWT_KT1_WIDE", 1) != 0;
            if (wide) {
                ktab_wide.ensure((size_t)kt1_ws * (E + 1));
                launch(KC_TABLE, k_ktab_wide, E + 1, E, (const uint32_t*)ktab_off.p, (const uint32_t*)ktab_b.p,
                       (const uint32_t*)ktab_e.p, (const uint32_t*)gpos.p, (const uint4*)samples.p, (const uint64_t*)rtext.p,
                       (uint64_t)tlen, ktab_wide.p, kt1_ws, X0.segtab, X0.seg_stride, X0.seg_hi, (uint32_t)sigma);
                device_bytes += wide_b;
            } else {
                ktab_one.ensure(E + 1);
                launch(KC_TABLE, k_ktab_one, E + 1, E, (const uint32_t*)ktab_off.p, (const uint32_t*)ktab_b.p,
                       (const uint32_t*)ktab_e.p, ktab_one.p, kt1_pos ? (const uint32_t*)gpos.p : (const uint32_t*)nullptr);
                device_bytes += (E + 1) * 8;
            }
        }
        HIPCHK(hipStreamSynchronize(stream));
        ktab_depth = depth;
        ktab_items = n;
        ktab_entries = E;
        device_bytes += (E + 1) * 4 + n * 8;
        release_workspace();
        if (trace) std::fprintf(stderr, "[edsbwt] k-mer start table: depth %u, %llu D-mers, %llu intervals\n", ktab_depth,
                                (unsigned long long)E, (unsigned long long)n);
    }

    // The k-mer start table at depth K in G = B^2 groups — the K-mers sharing their last two
    // characters, one level walk of B^K / G patterns each (k_kmer_batch with stride G), captured at
    // depth K and sorted by (D-mer, row) per group — then concatenated into the table's layout
    // (k_ktab_group_lens, a scan, k_ktab_group_copy): the same table as the whole-table walk's, with
    // 1/G of its transient workspace.  Returns K when built; else the deepest depth the failing
    // group's walk reached within its share of the budget (nothing built).
    uint32_t build_ktab_grouped(uint32_t K, uint64_t budget, uint64_t sym) {
        const uint32_t B = sigma - 1;
        auto pw = [&](uint32_t k) { uint64_t v = 1; for (uint32_t t = 0; t < k; t++) v *= B; return v; };
        const uint32_t G = (uint32_t)pw(2);
        const uint64_t E = pw(K), EG = E / G;
        // a group walk past 2/G of the budget at any depth ends the attempt (the groups are alike)
        const uint64_t gbudget = std::max<uint64_t>(1, 2 * budget / G);
        DBuf<uint32_t> goff;
        goff.ensure((size_t)G * (EG + 1));
        std::vector<DBuf<uint32_t>> gb(G), ge(G);
        uint64_t tot = 0;
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t g = 0; g < G; g++) {
            Capture c;
            {
                DBuf<uint8_t> kb;
                DBuf<uint64_t> ko;
                kb.ensure(EG * K);
                ko.ensure(EG + 1);
                launch(KC_TABLE, k_kmer_batch, EG, EG, K, B, sym, kb.p, ko.p, (uint64_t)G, (uint64_t)g);
                res.ensure(EG); ovf_orig.ensure(EG);
                zero(stats.p, kStatSlots * 8);
                c.K = K; c.B = B; c.only_last = true; c.budget = gbudget;
                cap = &c;
                const bool was_count_only = count_only;
                count_only = true;
                uint64_t abase = 0;
                try {
                    levels2(kb.p, ko.p, EG, false, res.p, abase, ovf_orig.p);
                } catch (const TooBig&) {
                    c.depth = 0;
                }
                cap = nullptr;
                count_only = was_count_only;
                st = edsbwt_stats{};
                HIPCHK(hipStreamSynchronize(stream));
            }
            tot += c.n;
            if (c.depth != K || (double)tot > (double)budget) {
                if (trace) std::fprintf(stderr, "[edsbwt] k-mer table depth %u, group %u: reached depth %u within %llu items\n", K, g,
                                        c.reached, (unsigned long long)gbudget);
                release_workspace();
                return std::min(c.reached, K - 1);
            }
            const uint64_t n = c.n;
            gb[g].ensure(n);
            ge[g].ensure(n);
            uint32_t* go = goff.p + (size_t)g * (EG + 1);
            if (n) {
                DBuf<uint64_t> k1, k2;
                DBuf<uint32_t> e2;
                k1.ensure(n); k2.ensure(n); e2.ensure(n);
                launch(KC_TABLE, k_ktab_keys, n, n, (const uint32_t*)c.k.p, (const uint32_t*)c.b.p, k1.p);
                c.k.release(); c.b.release();
                size_t tb = 0;
                const int endbit = 32 + (int)bits_for(EG);
                HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k1.p, k2.p, c.e.p, e2.p, cub_n(n), 0, endbit, stream));
                tmp.ensure(tb);
                HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, k1.p, k2.p, c.e.p, e2.p, cub_n(n), 0, endbit, stream));
                sync_check(nullptr, "hipcub call in build_ktab_grouped");
                k1.release();
                c.e.release();
                launch(KC_TABLE, k_ktab_split, n, n, (const uint64_t*)k2.p, gb[g].p);
                HIPCHK(hipMemcpyAsync(ge[g].p, e2.p, n * 4, hipMemcpyDeviceToDevice, stream));
                launch(KC_TABLE, k_ktab_bounds, EG + 1, EG, (const uint64_t*)k2.p, n, go);
                HIPCHK(hipStreamSynchronize(stream));
            } else {
                zero(go, (EG + 1) * 4);
            }
        }
        release_workspace();
        // the groups' lists in D-mer order: lengths, their scan (the table's offsets), the copy
        std::vector<const uint32_t*> pb(G), pe(G);
        for (uint32_t g = 0; g < G; g++) { pb[g] = gb[g].p; pe[g] = ge[g].p; }
        DBuf<const uint32_t*> dpb, dpe;
        dpb.ensure(G); dpe.ensure(G);
        HIPCHK(hipMemcpy(dpb.p, pb.data(), G * sizeof(void*), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(dpe.p, pe.data(), G * sizeof(void*), hipMemcpyHostToDevice));
        DBuf<uint32_t> len;
        len.ensure(E);
        launch(KC_TABLE, k_ktab_group_lens, E, E, G, EG, (const uint32_t*)goff.p, len.p);
        ktab_off.ensure(E + 2);  // [E, E+1): the empty list of D-mers outside the alphabet (direct start)
        const uint32_t n = scan_u32(len.p, ktab_off, E);
        len.release();
        if ((uint64_t)n != tot) throw Fail(EDSBWT_E_DEVICE, "k-mer table groups: list total mismatch");
        HIPCHK(hipMemcpyAsync(ktab_off.p + E + 1, ktab_off.p + E, 4, hipMemcpyDeviceToDevice, stream));
        ktab_b.ensure(std::max<uint64_t>(tot, 1));
        ktab_e.ensure(std::max<uint64_t>(tot, 1));
        launch(KC_TABLE, k_ktab_group_copy, E, E, G, EG, (const uint32_t*)goff.p, (const uint32_t* const*)dpb.p,
               (const uint32_t* const*)dpe.p, (const uint32_t*)ktab_off.p, ktab_b.p, ktab_e.p);
        HIPCHK(hipStreamSynchronize(stream));
        ktab_items = tot;
        if (trace)
            std::fprintf(stderr, "[edsbwt] k-mer start table built in %u groups of %llu K-mers: %llu intervals in %.2f s\n", G,
                         (unsigned long long)EG, (unsigned long long)tot,
                         std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        return K;
    }

    // Locate samples: one (word, offset) per row whose offset in its word is a multiple
    // of 2^kSampleShift, marked in the occ blocks' `samp` plane (sigma <= 7 frees cnt[7]
    // for their running count).  Built from the per-row table, which is then dropped.
    void build_samples() {
#if EDSBWT_OCC_ROWS == 64
        if (sigma > 7 || have_samples) return;
        const bool keep_table = have_table;
        build_table();
        const uint64_t nblk = (uint64_t)N / kOccRows + 1;
        DBuf<uint32_t> bcnt;
        bcnt.ensure(nblk);
        const uint32_t shift = std::min(8u, (uint32_t)env_double("EDSBWT_SAMPLE_SHIFT", kSampleShift));  // tuning knob
        samp_shift = shift;
        launch(KC_TABLE, k_samp_blocks, nblk, nblk, N, (const uint32_t*)offt.p, shift, occ.p, bcnt.p);
        DBuf<uint32_t> bbase;
        const uint32_t ns = scan_u32(bcnt.p, bbase, nblk);  // bbase[0..nblk], total read back
        if (ns < W) throw Fail(EDSBWT_E_FORMAT, "locate samples: fewer sampled rows than words");
        samples.ensure(ns);
        device_bytes += (size_t)ns * sizeof(uint4);
        launch(KC_TABLE, k_samp_fill, nblk, nblk, N, (const uint32_t*)da.p, (const uint32_t*)offt.p, (const uint32_t*)bbase.p,
               (const uint32_t*)seg_of_word.p, (const uint32_t*)seg_start.p, occ.p, samples.p);
        HIPCHK(hipStreamSynchronize(stream));
        if (!keep_table) {
            da.release();
            offt.release();
            device_bytes -= (size_t)N * 8;
            have_table = false;
        }
        have_samples = true;
#endif
    }

    void build_table() {
        if (have_table) return;
        da.ensure(N);
        offt.ensure(N);
        DBuf<uint32_t> wl;
        wl.ensure(W);
        device_bytes += (size_t)N * 8;
        KIdx X = kidx();
        launch(KC_TABLE, k_table_walk, W, W, X, da.p, offt.p, wl.p);
        launch(KC_TABLE, k_table_finish, N, N, (const uint32_t*)da.p, (const uint32_t*)wl.p, offt.p);
        HIPCHK(hipStreamSynchronize(stream));
        if (!have_text && sigma >= 2 && sigma - 1 <= 4 && env_double("EDSBWT_TEXT", 1) != 0) build_text(wl);
        wl.release();
        have_table = true;
    }

    // the words' text (k_text_build) from the per-row table and the word lengths
    void build_text(DBuf<uint32_t>& wl) {
        DBuf<uint32_t> ws;
        const uint32_t* wsp = nullptr;
        {
            DBuf<uint64_t> wl64, ws64;
            wl64.ensure(W);
            launch(KC_TABLE, k_u32_to_u64, W, (const uint32_t*)wl.p, (uint64_t)W, wl64.p);
            tlen = scan_u64(wl64.p, ws64, W);
            if (tlen >= 0xFFFFFFFFull) return;  // text positions are u32
            ws.ensure(W);
            launch(KC_TABLE, k_u32_of_u64, W, (const uint64_t*)ws64.p, (uint64_t)W, ws.p);
            wsp = ws.p;
        }
        const uint64_t nw = tlen / 32 + 5;  // rtext_window(tlen) reads word tlen/32 + 1
        rtext.ensure(nw);
        zero(rtext.p, nw * 8);
        gpos.ensure(N);
        wrow.ensure(W);
        launch(KC_TABLE, k_text_build, N, N, kidx(), (const uint32_t*)da.p, (const uint32_t*)offt.p, wsp, tlen, gpos.p, wrow.p,
               (uint32_t*)rtext.p);
        HIPCHK(hipStreamSynchronize(stream));
        device_bytes += nw * 8 + (size_t)N * 4 + (size_t)W * 4;
        have_text = true;
    }

    // ------------------------------------------------------------ search
    // Reversed-pattern trie order: patterns radix-sorted by their reversed symbol
    // codes, with the common-suffix length of neighbours (lcp).  Nodes of depth D
    // are the maximal runs with lcp >= D; nodes_at[D] counts them for every depth.
    // Returns false when every pattern is empty.
    bool build_trie(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t P, uint32_t& Lmax, std::vector<unsigned long long>& hist,
                    std::vector<uint64_t>& ge, uint32_t* n_term = nullptr) {
        if (P > 0x7fffffffull) throw Fail(EDSBWT_E_UNSUPPORTED, "more than 2^31 patterns in one call");
        // ---- A. longest pattern, from the offsets: one small launch, one read
        zero(counters.p + 6, 8);
        launch_reduce(KC_TRIE, k_lmax, d_off, P, counters.p + 6);
        Lmax = (uint32_t)read_u64(counters.p + 6);
        if (Lmax == 0) return false;
        // ---- B. reversed-pattern sort (trie order) and neighbours' common suffix
        bps = sigma + 2 <= 8 ? 3u : 4u;
        const uint32_t spc = 64 / bps;
        const uint32_t nch = (Lmax + spc - 1) / spc;
        lhist.ensure(2 * (size_t)(Lmax + 2) + 3);
        zero(lhist.p, (2 * (size_t)(Lmax + 2) + 3) * 8);
        unsigned long long* d_nterm = lhist.p + 2 * (size_t)(Lmax + 2);
        len.ensure(P);
        keys.ensure((size_t)nch * P);
        if (bps == 3)
            launch(KC_TRIE, k_keys<3>, P, d_bytes, d_off, P, (const uint8_t*)code_of.p, sigma, nch, keys.p, len.p, d_nterm, 0u, 0u,
                   (uint32_t*)nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr, 0u);
        else
            launch(KC_TRIE, k_keys<4>, P, d_bytes, d_off, P, (const uint8_t*)code_of.p, sigma, nch, keys.p, len.p, d_nterm, 0u, 0u,
                   (uint32_t*)nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr, 0u);
        perm.ensure(P);
        perm2.ensure(P);
        kc.ensure(P);
        kc2.ensure(P);
        slen.ensure(P);
        lcp.ensure(P);
        if (nch > 1) skey.ensure((size_t)(nch - 1) * P);
        unsigned long long* d_ties = d_nterm + 1;  // neighbours equal in chunk 0 only (statistic)
        unsigned long long* d_big = d_nterm + 2;   // tie groups too large for k_fix_ties
        std::vector<unsigned long long> hv(2 * (size_t)(Lmax + 2) + 3);
        // Trie order.  Sort by chunk 0 (the first SPC reversed symbols) only, then order each
        // group of equal chunk 0 by the later chunks in place (k_fix_ties: groups are small —
        // patterns ending at the same place through different variant words, or duplicates).
        // Only when a group is too large does the full LSD sort over every chunk run.
        // Only the bits that hold symbols are sorted.
        auto order = [&](bool full) {
            launch(KC_TRIE, k_iota, P, perm.p, P);
            for (int c = full ? (int)nch - 1 : 0; c >= 0; c--) {
                const uint32_t nsym = std::min(spc, Lmax - (uint32_t)c * spc);
                // rocPRIM (ROCm 7.2) mis-sorts u64 keys over [begin_bit, 64) when begin_bit > 0
                // (measured: tools/diag/sort_check.hip): every chunk is sorted from bit 0 (the
                // zero digits below a partial chunk's symbols cost passes, not correctness)
                const int end_bit = (int)(bps * spc);
                const int begin_bit = 0;
                (void)nsym;
                const uint64_t* kin = keys.p + (size_t)c * P;
                if (full && c != (int)nch - 1) {  // later passes sort the chunk in the current order
                    launch(KC_TRIE, k_gather_key, P, kin, (const uint32_t*)perm.p, P, kc.p);
                    kin = kc.p;
                }
                size_t tb = 0;
                HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kin, kc2.p, perm.p, perm2.p, cub_n(P), begin_bit, end_bit, stream));
                tmp.ensure(tb);
                timed(KC_TRIE, [&] {
                    HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, kin, kc2.p, perm.p, perm2.p, cub_n(P), begin_bit, end_bit, stream));
                    sync_check(nullptr, "hipcub call at engine.hip:739");
                });
                std::swap(perm.p, perm2.p);
                std::swap(perm.cap, perm2.cap);
            }
            // sorted chunks 1.. (chunk 0 is the last pass's output, kc2)
            for (uint32_t c = 1; c < nch; c++)
                launch(KC_TRIE, k_gather_key, P, (const uint64_t*)(keys.p + (size_t)c * P), (const uint32_t*)perm.p, P, skey.p + (size_t)(c - 1) * P);
            if (!full && nch > 1) launch(KC_TRIE, k_fix_ties, P, (const uint64_t*)kc2.p, skey.p, nch, P, perm.p, d_big);
            if (bps == 3)
                launch(KC_TRIE, k_slen_lcp<3>, P, (const uint64_t*)kc2.p, (const uint64_t*)skey.p, nch, P, slen.p, lcp.p, d_ties);
            else
                launch(KC_TRIE, k_slen_lcp<4>, P, (const uint64_t*)kc2.p, (const uint64_t*)skey.p, nch, P, slen.p, lcp.p, d_ties);
            // ---- C. nodes per depth and patterns per length, read once (with the '#' count and ties)
            if (Lmax + 2 <= 1024)
                launch_reduce(KC_TRIE, k_trie_counts, (const uint32_t*)slen.p, (const uint32_t*)lcp.p, P, Lmax, lhist.p, lhist.p + (Lmax + 2));
            else
                launch(KC_TRIE, k_trie_counts_global, P, (const uint32_t*)slen.p, (const uint32_t*)lcp.p, P, lhist.p, lhist.p + (Lmax + 2));
            if (hv.size() * 8 <= kStageBytes) {
                small_copy(hstage, lhist.p, hv.size() * 8);
                HIPCHK(hipStreamSynchronize(stream));
                std::memcpy(hv.data(), hstage, hv.size() * 8);
            } else {
                HIPCHK(hipMemcpyAsync(hv.data(), lhist.p, hv.size() * 8, hipMemcpyDeviceToHost, stream));
                HIPCHK(hipStreamSynchronize(stream));
            }
        };
        order(false);
        if (hv[2 * (size_t)(Lmax + 2) + 2]) {  // a tie group too large to fix in place: sort every chunk
            zero(lhist.p, 2 * (size_t)(Lmax + 2) * 8);
            order(true);
        }
        if (n_term) *n_term = (uint32_t)hv[2 * (size_t)(Lmax + 2)];
        hist.assign(hv.begin() + (Lmax + 2), hv.begin() + (Lmax + 2) + (Lmax + 1));
        nodes_at.assign(Lmax + 2, 0);
        int64_t run = 0;
        for (uint32_t D = 0; D <= Lmax + 1; D++) {
            run += (int64_t)hv[D];
            nodes_at[D] = (uint64_t)run;
        }
        ge.assign(Lmax + 2, 0);  // patterns with length >= l
        for (int l = (int)Lmax; l >= 0; l--) ge[l] = ge[l + 1] + hist[l];
        return true;
    }

    uint32_t levels(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t P, bool allow_deep, Res* r, uint64_t& abase, uint32_t* ovf_orig) {
        const KIdx X = kidx();
        uint32_t Lmax = 0;
        std::vector<unsigned long long> hist;
        std::vector<uint64_t> ge;
        if (!build_trie(d_bytes, d_off, P, Lmax, hist, ge)) return 0;
        // ---- B. root state [(0, N-1)] (init_backward_search, :220-225)
        nid[0].ensure(P);
        nid[1].ensure(P);
        zero(nid[0].p, P * 4);
        int cur = 0;
        uint32_t Mcur = 1;  // nodes at the current depth
        uint32_t ncur = 1;  // intervals at the current depth
        ib[0].ensure(1); ie[0].ensure(1); iu[0].ensure(1); ioff[0].ensure(1); iend[0].ensure(1);
        {
            uint32_t h[5] = {0, N - 1, 0, 0, 1};
            std::memcpy(pinned, h, sizeof h);
            small_copy(ib[0].p, &pinned[0], 4);
            small_copy(ie[0].p, &pinned[1], 4);
            small_copy(iu[0].p, &pinned[2], 4);
            small_copy(ioff[0].p, &pinned[3], 4);
            small_copy(iend[0].p, &pinned[4], 4);
            HIPCHK(hipStreamSynchronize(stream));
        }
        uint32_t novf = 0;
        // ---- C. depth loop
        for (uint32_t d = 0; d < Lmax; d++) {
            const uint32_t D = d + 1;
            const int nxt = cur ^ 1;
            // children nodes at depth D
            flag.ensure(P);
            launch(KC_NODES, k_node_flags, P, (const uint32_t*)slen.p, (const uint32_t*)lcp.p, P, D, flag.p);
            const uint32_t M = scan_u32(flag.p, scan, P);
            if (M == 0) break;
            // the trie stopped sharing below depth d: finish every pattern alone (k_deep)
            if (allow_deep && d >= 1 && (double)M >= deep_share * (double)ge[D]) {
                novf = run_deep(d, M, P, ge[D], d_bytes, d_off, nid[cur].p, ioff[cur].p, iend[cur].p, ib[cur].p, ie[cur].p, r, abase, ovf_orig);
                break;
            }
            st.depths++;
            st.trie_nodes += M;
            if (trace) std::fprintf(stderr, "[edsbwt] depth %u: nodes %u, parent intervals %u\n", D, M, ncur);
            node_first.ensure(M);
            node_parent.ensure(M);
            node_char.ensure(M);
            launch(KC_NODES, bps == 3 ? k_node_build<3> : k_node_build<4>, P, P, D, (const uint32_t*)slen.p, sorted_chunk(D, P), sigma, (const uint32_t*)lcp.p,
                   (const uint32_t*)scan.p, (const uint32_t*)nid[cur].p, nid[nxt].p, node_first.p, node_parent.p, node_char.p);
            child_first.ensure(Mcur);
            child_end.ensure(Mcur);
            zero(child_first.p, (size_t)Mcur * 4);
            zero(child_end.p, (size_t)Mcur * 4);
            launch(KC_NODES, k_child_links, M, (const uint32_t*)node_parent.p, M, child_first.p, child_end.p);
            // expand current intervals: rank of every symbol at both ends
            iocb.ensure((size_t)ncur * 8);
            ioce.ensure((size_t)ncur * 8);
            launch(KC_EXPAND, k_expand, ncur, (const uint32_t*)ib[cur].p, (const uint32_t*)ie[cur].p, (uint64_t)ncur, X, iocb.p, ioce.p);
            st.bytes_kernel[KC_EXPAND] += (uint64_t)ncur * (2 * sizeof(OccBlock) + 8 + 64);
            // LINK (not before the first step, :246-258)
            uint32_t R = 0;
            doff.ensure(Mcur);
            dend.ensure(Mcur);
            zero(doff.p, (size_t)Mcur * 4);
            zero(dend.p, (size_t)Mcur * 4);
            if (d > 0) {
                hcnt.ensure(ncur);
                launch(KC_LINK, k_hash_counts, ncur, (const uint32_t*)iu[cur].p, (const uint32_t*)iocb.p, (const uint32_t*)ioce.p,
                       (const uint32_t*)child_first.p, (const uint32_t*)child_end.p, (uint64_t)ncur, hcnt.p);
                const uint32_t Hn = scan_u32(hcnt.p, hoff, ncur);
                st.link_hash_rows += Hn;
                if (Hn) {
                    lkeys.ensure(Hn);
                    lkeys2.ensure(Hn);
                    zero(counters.p, 8);
                    launch(KC_LINK, k_link_emit, Hn, (uint64_t)Hn, (const uint32_t*)hoff.p, (uint64_t)ncur, (const uint32_t*)iocb.p,
                           (const uint32_t*)iu[cur].p, (const uint32_t*)eof_seg.p, lkeys.p, counters.p);
                    st.bytes_kernel[KC_LINK] += (uint64_t)Hn * 12;
                    const uint32_t V = (uint32_t)read_u64(counters.p);
                    if (V) {
                        size_t tb = 0;
                        // sentinels (~0) sort last; only the first V keys are used
                        HIPCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, lkeys.p, lkeys2.p, cub_n(Hn), 0, 64, stream));
                        tmp.ensure(tb);
                        timed(KC_LINKSORT, [&] { HIPCHK(hipcub::DeviceRadixSort::SortKeys(tmp.p, tb, lkeys.p, lkeys2.p, cub_n(Hn), 0, 64, stream)); });
                        sync_check(nullptr, "hipcub call at engine.hip:862");
                        rflag.ensure(V);
                        launch(KC_LINK, k_run_flags, V, (const uint64_t*)lkeys2.p, (uint64_t)V, (const uint32_t*)seg_lo.p, 32u, rflag.p,
                               (const uint32_t*)seg_chain.p, 0u);
                        R = scan_u32(rflag.p, rscan, V);
                        rb.ensure(R); re.ensure(R); ru.ensure(R);
                        launch(KC_LINK, k_run_build, V, (const uint64_t*)lkeys2.p, (uint64_t)V, (const uint32_t*)rflag.p, (const uint32_t*)rscan.p,
                               (const uint32_t*)seg_lo.p, (const uint32_t*)seg_start.p, 32u, rb.p, re.p, ru.p, (uint32_t*)nullptr);
                        launch(KC_LINK, k_bounds, R, (const uint32_t*)ru.p, (uint64_t)R, doff.p, dend.p);
                        docb.ensure((size_t)R * 8);
                        doce.ensure((size_t)R * 8);
                        launch(KC_EXPAND, k_expand, R, (const uint32_t*)rb.p, (const uint32_t*)re.p, (uint64_t)R, X, docb.p, doce.p);
                        st.bytes_kernel[KC_EXPAND] += (uint64_t)R * (2 * sizeof(OccBlock) + 8 + 64);
                        st.link_ranges += R;
                    }
                }
            }
            // STEP every child over [dollar ranges, own intervals] of its parent
            tcnt.ensure(M);
            launch(KC_STEP, k_task_counts, M, M, (const uint32_t*)node_parent.p, (const uint32_t*)doff.p, (const uint32_t*)dend.p,
                   (const uint32_t*)ioff[cur].p, (const uint32_t*)iend[cur].p, tcnt.p);
            const uint32_t T = scan_u32(tcnt.p, toff, M);
            st.intervals_stepped += T;
            if (trace) std::fprintf(stderr, "[edsbwt]   link ranges %u, step tasks %u\n", R, T);
            uint32_t R2 = 0;
            if (T) {
                tb.ensure(T); te.ensure(T); tu.ensure(T); tflag.ensure(T);
                launch(KC_STEP, k_step, T, (uint64_t)T, (const uint32_t*)toff.p, M, (const uint32_t*)node_parent.p, (const uint8_t*)node_char.p,
                       (const uint32_t*)doff.p, (const uint32_t*)dend.p, (const uint32_t*)ioff[cur].p, (const uint32_t*)docb.p,
                       (const uint32_t*)doce.p, (const uint32_t*)iocb.p, (const uint32_t*)ioce.p, X, tb.p, te.p, tu.p, tflag.p);
                st.bytes_kernel[KC_STEP] += (uint64_t)T * (8 + 16 + 16);
                const uint32_t V2 = scan_u32(tflag.p, tscan, T);
                if (V2) {
                    cb.ensure(V2); ce.ensure(V2); cu.ensure(V2);
                    launch(KC_MERGE, k_compact3, T, (uint64_t)T, (const uint32_t*)tflag.p, (const uint32_t*)tscan.p, (const uint32_t*)tb.p,
                           (const uint32_t*)te.p, (const uint32_t*)tu.p, cb.p, ce.p, cu.p);
                    mflag.ensure(V2);
                    launch(KC_MERGE, k_merge_flags, V2, (uint64_t)V2, (const uint32_t*)cb.p, (const uint32_t*)ce.p, (const uint32_t*)cu.p, mflag.p);
                    R2 = scan_u32(mflag.p, mscan, V2);
                    ib[nxt].ensure(R2); ie[nxt].ensure(R2); iu[nxt].ensure(R2);
                    launch(KC_MERGE, k_merge_build, V2, (uint64_t)V2, (const uint32_t*)mflag.p, (const uint32_t*)mscan.p, (const uint32_t*)cb.p,
                           (const uint32_t*)ce.p, (const uint32_t*)cu.p, ib[nxt].p, ie[nxt].p, iu[nxt].p);
                }
            }
            ioff[nxt].ensure(M);
            iend[nxt].ensure(M);
            zero(ioff[nxt].p, (size_t)M * 4);
            zero(iend[nxt].p, (size_t)M * 4);
            launch(KC_MERGE, k_bounds, R2, (const uint32_t*)iu[nxt].p, (uint64_t)R2, ioff[nxt].p, iend[nxt].p);
            // FINISH patterns of length D: archive their node's list
            fcnt.ensure(M);
            launch(KC_FINISH, k_fin_counts, M, M, D, (const uint32_t*)node_first.p, (const uint32_t*)slen.p, (const uint32_t*)ioff[nxt].p,
                   (const uint32_t*)iend[nxt].p, fcnt.p);
            const uint32_t F = scan_u32(fcnt.p, foff, M);
            node_occ.ensure(M);
            zero(node_occ.p, (size_t)M * 4);
            if (F) {
                ab.grow_keep(abase + F, stream);
                ae.grow_keep(abase + F, stream);
                launch(KC_FINISH, k_archive, R2, (uint64_t)R2, (const uint32_t*)iu[nxt].p, (const uint32_t*)ib[nxt].p, (const uint32_t*)ie[nxt].p,
                       (const uint32_t*)ioff[nxt].p, (const uint32_t*)fcnt.p, (const uint32_t*)foff.p, abase, ab.p, ae.p, node_occ.p);
            }
            if (hist[D])
                launch(KC_FINISH, k_finish, P, P, D, (const uint32_t*)slen.p, (const uint32_t*)nid[nxt].p, (const uint32_t*)perm.p,
                       (const uint32_t*)foff.p, (const uint32_t*)fcnt.p, (const uint32_t*)node_occ.p, abase, r);
            abase += F;
            cur = nxt;
            Mcur = M;
            ncur = R2;
            if (R2 == 0) break;  // every deeper suffix has an empty list
        }
        return novf;
    }

    // Finish every pattern longer than d with k_deep, starting from the lists of its
    // depth-d node ([goff[u], gend[u]) in gb/ge).  Returns the overflow count.
    uint32_t run_deep(uint32_t d, uint32_t M, uint64_t P, uint64_t active, const uint8_t* d_bytes, const uint64_t* d_off,
                      const uint32_t* nid_d, const uint32_t* goff, const uint32_t* gend, const uint32_t* gb, const uint32_t* gee,
                      Res* r, uint64_t& abase, uint32_t* ovf_orig,
                      const uint64_t* k0 = nullptr, const uint64_t* krest = nullptr, const uint32_t* lens = nullptr, uint32_t ind = 0,
                      const uint64_t* pv = nullptr) {
        // k0/krest/lens/ind: the direct start's input-order key chunks and lengths (ind: read
        // through perm); by default the trie's sorted chunks and slen.  pv: the packed direct
        // start (k_keys), from which k_deep_fast also writes perm
        const KIdx X = kidx();
        const uint32_t D = d + 1;
        DBuf<uint32_t>& ovf = tflag;  // flag_push list of sorted patterns k_deep could not hold
        ovf.ensure(P + 1);
        if (!defer) zero(ovf.p, 4);
        const uint32_t K = deep_k;
        ab.grow_keep(abase + (uint64_t)P * K, stream);
        ae.grow_keep(abase + (uint64_t)P * K, stream);
        // single-interval walks first; patterns needing lists or links are queued for k_deep
        const size_t qcap = std::max<size_t>(shard_bound(P, 1), 1024);
        dq.ensure(qcap * NSHARD);
        if (pv) dq2.ensure(qcap * NSHARD);
        dqpre.ensure(NSHARD + 1);
        lcnt.ensure(NSHARD * 32 + 32);
        if (!defer) zero(lcnt.p, NSHARD * 32 * 4);
        // the patterns' remaining symbols come from the sorted key chunks (chunk 0, then skey)
        if (!k0) {
            k0 = sorted_chunk(1, P);
            krest = skey.p;
            lens = slen.p;
        }
        // direct start from the k-mer table: its 8-B entries, or the wide ones (entry + a one-row
        // entry's sample and text window)
        const bool dstart = goff == ktab_off.p;
        const uint64_t* kt1 = dstart && ktab_one.p ? (const uint64_t*)ktab_one.p : (const uint64_t*)nullptr;
        const uint4* kt1w = dstart && ktab_wide.p ? (const uint4*)ktab_wide.p : (const uint4*)nullptr;
        const bool kdd = pv && kt1w && !X.rent3 && deep_direct;
        if (!kdd) settle_res(r);  // (k_deep_direct writes every result; the other walks need zeros)
        // fused counts: only on the deferred direct start (its three kernels write every final count)
        uint32_t* fc = kdd && defer ? fc_counts : nullptr;
        if (fc) fc_done = true;
        const uint32_t np = kdd && fk_now.on && defer && deep_pieces > 1 && P >= deep_piece_min && K == 4 && bps == 3 &&
                                    !X.eofrow && deepq_waves >= 5
                                ? deep_pieces : 1u;
        if (np > 1) {
            run_deep_pieces(np, d, P, nid_d, goff, gend, gb, gee, lens, k0, krest, ind, X, abase, K, r, kt1w, fc);
        } else if (kdd && fk_now.on) {
            // the fused direct start: keys from the pattern bytes inside k_deep_direct (nid_d is
            // written there, for k_deep and k_deep_wave)
            auto kd0 = direct_waves >= 8 ? (direct_back ? (deep_stats ? k_deep_direct<8, true> : k_deep_direct<8, true, false>)
                                                        : (deep_stats ? k_deep_direct<8, true, true, false> : k_deep_direct<8, true, false, false>))
                     : direct_waves >= 7 ? (deep_stats ? k_deep_direct<7, true> : k_deep_direct<7, true, false>)
                     : direct_waves >= 6 ? k_deep_direct<6, true> : k_deep_direct<1, true>;
            launch(KC_DEEP, kd0, P, P, d, nid_d, X, abase, K, r, dq.p, (uint32_t)qcap, lcnt.p, stats.p, pv, perm.p, kt1w, dq2.p,
                   fk_now.bytes, fk_now.off, len.p, const_cast<uint32_t*>(nid_d), fk_now.n_term, fk_now.E, fk_now.lmin, fk_now.lmax, fc, 0u);
            fk_now.on = false;
        } else if (kdd) {
            auto kd0 = direct_waves >= 8 ? k_deep_direct<8> : direct_waves >= 7 ? k_deep_direct<7> : direct_waves >= 6 ? k_deep_direct<6>
                                                                                                        : k_deep_direct<1>;
            launch(KC_DEEP, kd0, P, P, d, nid_d, X, abase, K, r, dq.p, (uint32_t)qcap, lcnt.p, stats.p, pv, perm.p, kt1w, dq2.p,
                   (const uint8_t*)nullptr, (const uint64_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr, (unsigned long long*)nullptr, 0u,
                   0u, 0u, fc, 0u);
        } else {
            auto kf = bps == 4 ? k_deep_fast<4> : deep_waves >= 8 ? k_deep_fast<3, 8> : deep_waves >= 6 ? k_deep_fast<3, 6> : k_deep_fast<3>;
            launch(KC_DEEP, kf, P, P, d, lens, (const uint32_t*)perm.p, k0, krest, ind,
                   nid_d, goff, gend, gb, gee, X, abase, K, ab.p, ae.p, r, dq.p, (uint32_t)qcap, lcnt.p, stats.p, pv, perm.p, kt1,
                   pv ? dq2.p : (uint64_t*)nullptr, kt1w);
        }
        if (trace) {  // (k_deep sums the shard counters itself; the trace line below reads the total)
            hipLaunchKernelGGL(k_queue_prefix, dim3(1), dim3(64), 0, stream, (const uint32_t*)lcnt.p, dqpre.p);
            HIPCHK(hipGetLastError());
        }
        const bool unb = deepq_waves <= 1;
        if (np > 1) {
            // (run_deep_pieces walked every piece's queue)
        } else {
        auto kd = K == 2   ? (bps == 3 ? k_deep<2, 3> : k_deep<2, 4>)
                  : K == 3 ? (bps == 3 ? k_deep<3, 3> : k_deep<3, 4>)
                  : K == 4 ? (bps == 3 ? (X.eofrow ? (unb ? k_deep<4, 3, 1, true> : k_deep<4, 3, 5, true>)
                                          : unb ? k_deep<4, 3, 1> : deepq_waves >= 6 ? (deep_stats ? k_deep<4, 3, 6> : k_deep<4, 3, 6, false, false>) : deep_stats ? k_deep<4, 3, 5> : k_deep<4, 3, 5, false, false>)
                                       : unb ? k_deep<4, 4, 1> : k_deep<4, 4, 5>)
                           : (bps == 3 ? k_deep<8, 3> : k_deep<8, 4>);
        // the packed direct start's queue: the build without the key-chunk reader and the perm /
        // slen reads (PACKED: 77 VGPRs and no scratch at 6 waves per SIMD, against 80 + 40 B of
        // scratch; EDSBWT_DEEPQ_PACKED=0: the generic build; EDSBWT_DEEPQ_WAVES=7: 7 waves)
        if (pv && deepq_packed && K == 4 && bps == 3 && !X.eofrow && !unb && deepq_waves >= 6)
            kd = deepq_waves >= 7 ? (deep_stats ? k_deep<4, 3, 7, false, true, true> : k_deep<4, 3, 7, false, false, true>)
                                  : (deep_stats ? k_deep<4, 3, 6, false, true, true> : k_deep<4, 3, 6, false, false, true>);
        launch(KC_DEEPQ, kd, P, (const uint4*)dq.p, (const uint32_t*)lcnt.p, (uint32_t)qcap, d, lens,
               (const uint32_t*)perm.p, k0, krest, ind, P, nid_d, goff, gend, gb, gee, X, abase, ab.p, ae.p, r, ovf.p, stats.p,
               pv ? (const uint64_t*)dq2.p : (const uint64_t*)nullptr, kt1w, fc, deepq_pairs);
        tag_queue((const uint4*)dq.p, (const uint32_t*)lcnt.p, (uint32_t)qcap, EDSBWT_PATH_DEEP);
        }
        abase += (uint64_t)P * K;
        st.deep_from_depth = D;
        if (trace)
            std::fprintf(stderr, "[edsbwt] deep from depth %u: nodes %u, patterns %llu, queued for k_deep %u\n", D, M, (unsigned long long)active,
                         read_u32(dqpre.p + NSHARD));
        st.bytes_kernel[KC_DEEP] += (uint64_t)P * 24;  // + interval steps and '#' rows, folded at the end of search()
        // lists that outgrew k_deep's registers: retry those patterns with wide lists
        if (defer) {
            // no read-back: k_deep_wide takes the list's length from the device, up to
            // kWideCap patterns; a longer list, or any pattern the wide lists cannot hold
            // either, fails search()'s final check and the batch is searched again
            DBuf<uint32_t>& ovf2 = hcnt;
            const uint32_t wcap = (uint32_t)std::min<uint64_t>(P, wide_cap);
            ovf2.ensure((size_t)wcap + 1);  // (count zeroed by search())
            if (!no_wide) {
                ab.grow_keep(abase + (uint64_t)wcap * kDeepWide, stream);
                ae.grow_keep(abase + (uint64_t)wcap * kDeepWide, stream);
                // the record-offset tiles of every other pattern beside k_deep_wave (early_counts: a
                // located direct start; the results are final but for k_deep_wave's patterns)
                if (deep_wave && early_counts && in_direct && r == res.p) {
                    const uint64_t nwords = (P + 31) / 32;
                    if (wbits_words < nwords) {
                        wbits.ensure(nwords);
                        zero(wbits.p, nwords * 4);
                        wbits_words = nwords;
                    }
                    tile_sum.ensure((P + 63) / 64);
                    if (!stream2) HIPCHK(hipStreamCreateWithFlags(&stream2, hipStreamNonBlocking));
                    if (!tiles_ev) HIPCHK(hipEventCreateWithFlags(&tiles_ev, hipEventDisableTiming));
                    if (!tiles_ev0) HIPCHK(hipEventCreateWithFlags(&tiles_ev0, hipEventDisableTiming));
                    HIPCHK(hipEventRecord(tiles_ev0, stream));
                    HIPCHK(hipStreamWaitEvent(stream2, tiles_ev0, 0));
                    std::swap(stream, stream2);  // (launch() and its timing events on the second stream)
                    launch(KC_FINISH, k_mark_wide, wcap, (const uint32_t*)ovf.p, wcap, (const uint32_t*)perm.p, wbits.p);
                    launch(KC_FINISH, k_count_tiles, P, (const Res*)res.p, P, early_counts, stats.p, (unsigned long long*)tile_sum.p, wbits.p);
                    std::swap(stream, stream2);
                    HIPCHK(hipEventRecord(tiles_ev, stream2));
                    tiles_early = true;
                    early_ovf = ovf.p;
                    early_cap = wcap;
                }
                // (the waves stride over the list: 2048 of them, not one per possible pattern)
                if (deep_wave)
                    launch(KC_DEEPW, k_deep_wave, (size_t)std::min<uint32_t>(wcap, kWaveGrid) * 64, P, d, (const uint32_t*)(ovf.p + 1), wcap, lens, (const uint32_t*)perm.p, ind,
                           d_off, d_bytes, (const uint8_t*)code_of.p, nid_d, goff, gend, gb, gee, X, abase, ab.p, ae.p, r, ovf2.p,
                           (const uint32_t*)ovf.p, stats.p, fc);
                else
                    launch(KC_DEEPW, k_deep_wide<kDeepWide>, wcap, P, d, (const uint32_t*)(ovf.p + 1), wcap, lens, (const uint32_t*)perm.p, ind,
                           d_off, d_bytes, (const uint8_t*)code_of.p, nid_d, goff, gend, gb, gee, X, abase, ab.p, ae.p, r, ovf2.p,
                           (const uint32_t*)ovf.p);
                abase += (uint64_t)wcap * kDeepWide;
                tag_list(ovf.p, wcap, EDSBWT_PATH_WIDE);
            }
            defer_ovf2 = no_wide ? ovf.p : ovf2.p;  // gathered by finish_deferred
            defer_wide_cap = no_wide ? 0 : wcap;
            return 0;
        }
        const uint32_t nw = read_u32(ovf.p);
        uint32_t novf = nw;
        const uint32_t* list = ovf.p + 1;
        if (nw && !no_wide) {
            DBuf<uint32_t>& ovf2 = hcnt;  // ... and those the wide lists could not hold either
            ovf2.ensure((size_t)nw + 1);
            zero(ovf2.p, 4);
            ab.grow_keep(abase + (uint64_t)nw * kDeepWide, stream);
            ae.grow_keep(abase + (uint64_t)nw * kDeepWide, stream);
            if (deep_wave)
                launch(KC_DEEPW, k_deep_wave, (size_t)std::min<uint32_t>(nw, kWaveGrid) * 64, P, d, list, nw, lens, (const uint32_t*)perm.p, ind,
                       d_off, d_bytes, (const uint8_t*)code_of.p, nid_d, goff, gend, gb, gee, X, abase, ab.p, ae.p, r, ovf2.p,
                       (const uint32_t*)nullptr, stats.p, (uint32_t*)nullptr);
            else
                launch(KC_DEEPW, k_deep_wide<kDeepWide>, nw, P, d, list, nw, lens, (const uint32_t*)perm.p, ind,
                       d_off, d_bytes, (const uint8_t*)code_of.p, nid_d, goff, gend, gb, gee, X, abase, ab.p, ae.p, r, ovf2.p,
                       (const uint32_t*)nullptr);
            abase += (uint64_t)nw * kDeepWide;
            st.deep_overflow += nw;
            novf = read_u32(ovf2.p);
            list = ovf2.p + 1;
            tag_list(ovf.p, nw, EDSBWT_PATH_WIDE);
        }
        tag_list(list - 1, novf, EDSBWT_PATH_LEVELS);
        if (novf) {
            zero(ovf_orig, P * 4);
            launch(KC_MERGE, k_ovf_mark, novf, novf, list, (const uint32_t*)perm.p, ovf_orig);
        }
        if (no_wide) st.deep_overflow += nw;
        st.deep_level_rerun += novf;
        return novf;
    }

    // The fused, deferred direct start in np pieces of the batch (EDSBWT_DEEP_PIECES): piece j's
    // k_deep_direct on the library stream, then an event, and k_deep over piece j's own queue on a
    // second stream, so it runs beside piece j + 1's k_deep_direct; the library stream waits for the
    // last k_deep before what follows (k_deep_wave, locate).  Each piece has its own queue slots and
    // shard counters (pcnt), its k_deep the queue's capacity of its piece; results, counts, the
    // overflow list and the statistics are shared (device atomics).  Same work, same results as one
    // piece: only the order in which the GPU runs it changes
    void run_deep_pieces(uint32_t np, uint32_t d, uint64_t P, const uint32_t* nid_d, const uint32_t* goff, const uint32_t* gend,
                         const uint32_t* gb, const uint32_t* gee, const uint32_t* lens, const uint64_t* k0, const uint64_t* krest,
                         uint32_t ind, const KIdx& X, uint64_t abase, uint32_t K, Res* r, const uint4* kt1w, uint32_t* fc) {
        if (!stream2) HIPCHK(hipStreamCreateWithFlags(&stream2, hipStreamNonBlocking));
        while (piece_ev.size() < np + 1) {
            hipEvent_t e;
            HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            piece_ev.push_back(e);
        }
        DBuf<uint32_t>& ovf = tflag;
        const size_t pq = std::max<size_t>(shard_bound((P + np - 1) / np, 1), 1024);  // each piece's queue capacity per shard
        dq.ensure(pq * NSHARD * np);
        dq2.ensure(pq * NSHARD * np);
        pcnt.ensure((size_t)NSHARD * 32 * np);
        // stream2 starts after everything already on the library stream (the zeroing, the keys' inputs)
        HIPCHK(hipEventRecord(piece_ev[np], stream));
        HIPCHK(hipStreamWaitEvent(stream2, piece_ev[np], 0));
        auto kd0 = direct_waves >= 8 ? (direct_back ? (deep_stats ? k_deep_direct<8, true> : k_deep_direct<8, true, false>)
                                                    : (deep_stats ? k_deep_direct<8, true, true, false> : k_deep_direct<8, true, false, false>))
                 : direct_waves >= 7 ? (deep_stats ? k_deep_direct<7, true> : k_deep_direct<7, true, false>)
                 : direct_waves >= 6 ? k_deep_direct<6, true> : k_deep_direct<1, true>;
        auto kd = deepq_waves >= 6 ? (deep_stats ? k_deep<4, 3, 6> : k_deep<4, 3, 6, false, false>)
                                   : (deep_stats ? k_deep<4, 3, 5> : k_deep<4, 3, 5, false, false>);
        if (deepq_packed && deepq_waves >= 6)  // (the pieces are the packed start's: see run_deep)
            kd = deepq_waves >= 7 ? (deep_stats ? k_deep<4, 3, 7, false, true, true> : k_deep<4, 3, 7, false, false, true>)
                                  : (deep_stats ? k_deep<4, 3, 6, false, true, true> : k_deep<4, 3, 6, false, false, true>);
        for (uint32_t j = 0; j < np; j++) {
            const uint64_t lo = P * j / np, hi = P * (j + 1) / np;
            uint4* qj = (uint4*)dq.p + (size_t)j * pq * NSHARD;
            uint64_t* q2j = dq2.p + (size_t)j * pq * NSHARD;
            uint32_t* cj = pcnt.p + (size_t)j * NSHARD * 32;
            launch(KC_DEEP, kd0, hi - lo, hi, d, nid_d, X, abase, K, r, qj, (uint32_t)pq, cj, stats.p, (const uint64_t*)nullptr, perm.p,
                   kt1w, q2j, fk_now.bytes, fk_now.off, len.p, const_cast<uint32_t*>(nid_d), fk_now.n_term, fk_now.E, fk_now.lmin,
                   fk_now.lmax, fc, (uint32_t)lo);
            HIPCHK(hipEventRecord(piece_ev[j], stream));
            HIPCHK(hipStreamWaitEvent(stream2, piece_ev[j], 0));
            std::swap(stream, stream2);  // (launch() and its timing events on the second stream)
            launch(KC_DEEPQ, kd, hi - lo, (const uint4*)qj, (const uint32_t*)cj, (uint32_t)pq, d, lens, (const uint32_t*)perm.p, k0,
                   krest, ind, P, nid_d, goff, gend, gb, gee, X, abase, ab.p, ae.p, r, ovf.p, stats.p, (const uint64_t*)q2j, kt1w, fc,
                   deepq_pairs);
            std::swap(stream, stream2);
            tag_queue((const uint4*)qj, (const uint32_t*)cj, (uint32_t)pq, EDSBWT_PATH_DEEP);
        }
        fk_now.on = false;
        HIPCHK(hipEventRecord(piece_ev[np], stream2));
        HIPCHK(hipStreamWaitEvent(stream, piece_ev[np], 0));
    }

    // Direct start: when every pattern is longer than the k-mer table's depth D0 and the
    // table's lists are short on average, no trie is built.  Each pattern (in input order)
    // takes its D0-mer's list straight from the table and k_deep walks it from there: the
    // sharing a trie would add past depth D0 is small (nodes ~ patterns), and the sort,
    // node build and list copy it needs cost more than the deep walk saves.  Returns
    // kNotDirect when the batch does not qualify (nothing was written), kNeedOrdered for
    // patterns holding '#', else k_deep's overflow count as run_deep.
    static constexpr uint32_t kNotDirect = 0xFFFFFFFEu;
    // buckets of the direct start's grouping (0: the radix sort path or no direct start)
    uint64_t direct_buckets() const {
        if (!ktab_depth || !use_buckets || sort_bits() <= 0) return 0;
        const uint64_t E = ktab_entries;
        const int shift = std::max(0, (int)bits_for(E) - sort_bits());
        const uint64_t nb = (E >> shift) + 1;
        return nb <= (1u << 22) ? nb : 0;
    }
    uint32_t direct(const uint64_t* d_off, const uint8_t* d_bytes, uint64_t P, Res* r,
                    uint64_t& abase, uint32_t* ovf_orig) {
        if (cap || !use_ktab || !use_direct || !ktab_depth || (double)ktab_items > direct_items * (double)ktab_entries) return kNotDirect;
        if (P > 0x7fffffffull) throw Fail(EDSBWT_E_UNSUPPORTED, "more than 2^31 patterns in one call");
        const uint32_t D0 = ktab_depth;
        if (!defer_call) zero(counters.p + 8, 24);
        uint32_t Lmax, Lmin;
        bool unmeasured = false;
        if (known_len) {  // the host pipeline measured the chunk's lines beside the previous search
            Lmax = known_lmax;
            Lmin = known_lmin;
        } else if (defer_call && len_guess && acgt_alpha && keys_packed && keys_swar && use_packed && direct_sort && !use_buckets && sigma == 5) {
            // deferred: assume the packed start's lengths (D0 + 1 .. D0 + 16) and let k_keys_acgt
            // count the patterns outside them with the '#' check (no read-back here)
            Lmin = D0 + 1;
            Lmax = D0 + 16;
            unmeasured = true;
            guessed_len = true;
        } else {
            launch_reduce(KC_TRIE, k_lminmax, d_off, P, counters.p + 8);
            small_copy(pinned, counters.p + 8, 16);
            HIPCHK(hipStreamSynchronize(stream));
            uint64_t mm[2];
            std::memcpy(mm, pinned, 16);
            Lmax = (uint32_t)mm[0];
            Lmin = ~(uint32_t)mm[1];
        }
        if (Lmin <= D0) return kNotDirect;
        bps = sigma + 2 <= 8 ? 3u : 4u;
        const uint32_t nch = (Lmax + 64 / bps - 1) / (64 / bps);
        len.ensure(P);
        keys.ensure((size_t)nch * P);
        unsigned long long* d_nterm = counters.p + 10;
        nid[0].ensure(P);
        perm.ensure(P);
        const uint32_t E = (uint32_t)ktab_entries;
        if (direct_sort) {
            nid[1].ensure(P);
            perm2.ensure(P);
        }
        uint32_t* kid = direct_sort ? nid[1].p : nid[0].p;
        // packed start: each pattern's input index and remaining symbols travel through the
        // D-mer sort as its value, so k_deep_fast reads no key chunks or lengths at random
        const bool packed = direct_sort && use_packed && sigma - 1 <= 4 && Lmax - D0 <= 16 && bps == 3;
        if (packed) {
            pv_in.ensure(P);
            pv_out.ensure(P);
        }
        // the packed start's grouping by the D-mer's leading bits: a bucket histogram from k_keys,
        // a scan, one scatter (EDSBWT_BUCKETS=0: hipcub radix sort over those bits instead)
        const int endbit_e = (int)bits_for(E);
        const int direct_sort_bits = sort_bits();
        const uint32_t hshift = (uint32_t)std::max(0, endbit_e - direct_sort_bits);
        const uint64_t nbkt = direct_buckets();
        const bool buckets = packed && nbkt;
        if (buckets && !defer_call) {
            bhist.ensure(nbkt + 1);
            zero(bhist.p, (nbkt + 1) * 4);
        }
        // fused: the deferred, input-ordered packed start with the wide entries (C3's path) computes
        // the keys inside k_deep_direct (run_deep); its '#' / length check is deferred as k_keys_acgt's
        const bool in_order = direct_sort_bits <= 0 || P < direct_sort_min;
        fk_now = FusedKeys{};
        if (fused_keys && defer_call && packed && !buckets && keys_packed && acgt_alpha && keys_swar && in_order && ktab_wide.p &&
            !kidx().rent3 && deep_direct) {
            fk_now.on = true;
            fk_now.bytes = d_bytes;
            fk_now.off = d_off;
            fk_now.n_term = d_nterm;
            fk_now.E = E;
            fk_now.lmin = unmeasured ? D0 + 1 : 0u;
            fk_now.lmax = unmeasured ? D0 + 16 : 0u;
        }
        // key chunks (k_deep's queue reads them), D-mer ids and packed starts in one pass; the
        // packed start needs no chunks (EDSBWT_KEYS_PACKED=0: k_keys for it too)
        if (fk_now.on) {
            // (k_deep_direct computes them)
        } else if (packed && !buckets && keys_packed && acgt_alpha && keys_swar)
            launch(KC_TRIE, k_keys_acgt, P, d_bytes, d_off, P, len.p, d_nterm, D0, E, kid, pv_in.p, unmeasured ? D0 + 1 : 0u,
                   unmeasured ? D0 + 16 : 0u);
        else if (packed && !buckets && keys_packed)
            launch(KC_TRIE, k_keys_packed, P, d_bytes, d_off, P, (const uint8_t*)code_of.p, sigma, len.p, d_nterm, D0, E, kid, pv_in.p);
        else if (bps == 3)
            launch(KC_TRIE, k_keys<3>, P, d_bytes, d_off, P, (const uint8_t*)code_of.p, sigma, nch, keys.p, len.p, d_nterm, D0, E, kid,
                   packed ? pv_in.p : (uint64_t*)nullptr, buckets ? bhist.p : (uint32_t*)nullptr, hshift);
        else
            launch(KC_TRIE, k_keys<4>, P, d_bytes, d_off, P, (const uint8_t*)code_of.p, sigma, nch, keys.p, len.p, d_nterm, D0, E, kid,
                   (uint64_t*)nullptr, (uint32_t*)nullptr, 0u);
        // '#' in a pattern: lists may overlap, use levels().  Deferred: read with the final check
        // (a batch holding '#' is then searched again on the ordered path)
        defer = defer_call && packed;
        if (!defer && read_u64(d_nterm)) return kNeedOrdered;
        // input order (EDSBWT_DIRECT_SORT_BITS=0, or a batch too small for the grouping to pay:
        // its ~20 sort launches cost more than the locality saves below EDSBWT_DIRECT_SORT_MIN)
        if (packed && (direct_sort_bits <= 0 || P < direct_sort_min)) {
            st.start_depth = D0;
            return run_deep(D0, (uint32_t)std::min<uint64_t>(P, 0xffffffffu), P, P, d_bytes, d_off, kid, ktab_off.p, ktab_off.p + 1,
                            ktab_b.p, ktab_e.p, r, abase, ovf_orig, keys.p, keys.p + P, len.p, 1u, pv_in.p);
        }
        if (buckets) {
            bscan.ensure(nbkt + 1);
            exclusive_scan(bhist.p, bscan.p, nbkt);
            hmark("bucket scan");
            launch(KC_TRIE, k_bucket_scatter, P, (uint64_t)P, (const uint32_t*)kid, (const uint64_t*)pv_in.p, hshift, bscan.p, nid[0].p, pv_out.p);
            st.start_depth = D0;
            return run_deep(D0, (uint32_t)std::min<uint64_t>(P, 0xffffffffu), P, P, d_bytes, d_off, nid[0].p, ktab_off.p, ktab_off.p + 1,
                            ktab_b.p, ktab_e.p, r, abase, ovf_orig, keys.p, keys.p + P, len.p, 1u, pv_out.p);
        }
        if (packed) {
            // the order only buys locality (neighbouring lanes read neighbouring table entries and
            // rows): the D-mer's first direct_sort_bits bits (its leading symbols) are enough
            size_t tb = 0;
            const int endbit = (int)bits_for(E);
            const int beginbit = std::max(0, endbit - direct_sort_bits);
            HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kid, nid[0].p, pv_in.p, pv_out.p, cub_n(P), beginbit, endbit, stream));
            tmp.ensure(tb);
            timed(KC_TRIE, [&] {
                HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, kid, nid[0].p, pv_in.p, pv_out.p, cub_n(P), beginbit, endbit, stream));
            });
            sync_check(nullptr, "hipcub call in direct() (packed)");
            st.start_depth = D0;
            return run_deep(D0, (uint32_t)std::min<uint64_t>(P, 0xffffffffu), P, P, d_bytes, d_off, nid[0].p, ktab_off.p, ktab_off.p + 1,
                            ktab_b.p, ktab_e.p, r, abase, ovf_orig, keys.p, keys.p + P, len.p, 1u, pv_out.p);
        }
        launch(KC_NODES, k_iota, P, direct_sort ? perm2.p : perm.p, P);
        if (direct_sort) {
            // patterns ordered by D-mer: a wave's lanes share their table lists and the rows of
            // their first steps (their lengths and key chunks stay in input order, read via perm)
            size_t tb = 0;
            const int endbit = (int)bits_for(E);
            HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kid, nid[0].p, perm2.p, perm.p, cub_n(P), 0, endbit, stream));
            tmp.ensure(tb);
            timed(KC_TRIE, [&] { HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, kid, nid[0].p, perm2.p, perm.p, cub_n(P), 0, endbit, stream)); });
            sync_check(nullptr, "hipcub call in direct()");
        }
        st.start_depth = D0;
        if (trace)
            std::fprintf(stderr, "[edsbwt] direct start at depth %u from the k-mer table: %llu patterns%s\n", D0, (unsigned long long)P,
                         direct_sort ? ", sorted by D-mer" : "");
        // chunk c of input pattern j is keys[c*P + j]: chunk 0 and then chunks 1.. as k_deep reads them
        return run_deep(D0, (uint32_t)std::min<uint64_t>(P, 0xffffffffu), P, P, d_bytes, d_off, nid[0].p, ktab_off.p, ktab_off.p + 1,
                        ktab_b.p, ktab_e.p, r, abase, ovf_orig, keys.p, keys.p + P, len.p, direct_sort ? 1u : 0u);
    }

    // Order-free level walk (default): a depth's lists are unordered (node, b, e)
    // items; k_lvl_items steps every item by every child symbol and emits its
    // '#' rows in the same pass; link keys are sorted per node into previous-segment
    // runs (k_run_*), which k_lvl_dollar steps.  Same outputs as levels() for
    // patterns without '#' (finished lists are sorted by row before archiving).
    uint32_t levels2(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t P, bool allow_deep, Res* r, uint64_t& abase, uint32_t* ovf_orig) {
        const KIdx X = kidx();
        uint32_t Lmax = 0, n_term = 0;
        std::vector<unsigned long long> hist;
        std::vector<uint64_t> ge;
        if (!build_trie(d_bytes, d_off, P, Lmax, hist, ge, &n_term)) return 0;
        if (n_term) return kNeedOrdered;  // '#' in a pattern: lists may overlap, use levels()
        nid[0].ensure(P);
        nid[1].ensure(P);
        flag.ensure(P);
        scan.ensure(P + 1);
        node_first.ensure(P);
        node_parent.ensure(P);
        node_char.ensure(P);
        lcnt.ensure(NSHARD * 32 + 32);
        uint32_t* d_runs = lcnt.p + NSHARD * 32;  // link runs of the current depth (device count)
        zero(nid[0].p, P * 4);
        int cur = 0;
        uint32_t Mcur = 1, ncur = 1;
        ib[0].ensure(1); ie[0].ensure(1); iu[0].ensure(1);
        {
            uint32_t* h = pinned;
            h[0] = 0; h[1] = N - 1; h[2] = 0;
            small_copy(ib[0].p, &h[0], 4);
            small_copy(ie[0].p, &h[1], 4);
            small_copy(iu[0].p, &h[2], 4);
        }
        uint32_t novf = 0;
        // text items (count-only walks with the per-row text entries): no new ones once a deep
        // cutover may come, and no cutover while any is alive (they carry no row)
        const bool titems = text_items && count_only && fuse_finish && !cap && X.srow && N < 0x80000000u && (uint64_t)S + 2 < kTextSeg;
        bool text_stop = false;
        uint32_t text_alive = 0;
        bool in_sharded = false;  // current items in fu/fb/fe shards (prefix fpre, capacity fcap)
        size_t fcap = 0;
        auto pack_items = [&](int dst) {  // shards -> iu/ib/ie[dst]
            iu[dst].ensure(ncur); ib[dst].ensure(ncur); ie[dst].ensure(ncur);
            if (ncur)
                launch(KC_MERGE, k_unshard<uint32_t, uint32_t, uint32_t>, ncur, ncur, (const uint32_t*)fpre.p, (uint32_t)fcap,
                       (const uint32_t*)fu.p, (const uint32_t*)fb.p, (const uint32_t*)fe.p, iu[dst].p, ib[dst].p, ie[dst].p);
            in_sharded = false;
        };
        // k-mer start table: when every pattern is longer than its depth d0, the items of
        // depth d0 are the table's lists of the depth-d0 nodes' d0-mers (no steps 1..d0)
        uint32_t d0 = 0;
        bool from_lt = false;  // ... or from the deep level table, when every pattern is >= its depth
        if (!cap && use_ktab && (ktab_depth || lt_depth)) {
            uint32_t lmin = 0;
            while (lmin <= Lmax && hist[lmin] == 0) lmin++;
            if (use_ltab && lt_depth && lmin >= lt_depth) {
                d0 = lt_depth;
                from_lt = true;
            } else if (ktab_depth && lmin > ktab_depth) {
                d0 = ktab_depth;
            }
        }
        if (from_lt) {
            const uint32_t M0 = (uint32_t)nodes_at[d0];
            node_scan(d0, P);
            launch(KC_NODES, bps == 3 ? k_node_build<3> : k_node_build<4>, P, P, d0, (const uint32_t*)slen.p, sorted_chunk(d0, P), sigma,
                   (const uint32_t*)lcp.p, (const uint32_t*)scan.p, (const uint32_t*)nid[0].p, nid[1].p, node_first.p, node_parent.p, node_char.p);
            kt_kid.ensure(M0);
            kt_cnt.ensure(M0);
            zero(lt_total.p, 8);
            launch(KC_NODES, bps == 3 ? k_ltab_count<3> : k_ltab_count<4>, M0, M0, d0, sigma - 1, (const uint32_t*)node_first.p,
                   sorted_chunk(1, P), (const uint32_t*)lt_off.p, lt_G, lt_EG, kt_kid.p, kt_cnt.p, lt_total.p);
            // a batch whose start items pass 2^31 (a whole C5 batch: ~9G) is searched in trie-subtree groups
            if (read_u64(lt_total.p) > lt_start_max) throw TooBig("level table start over 2^31 items");
            const uint32_t n0 = scan_u32(kt_cnt.p, kt_pos, M0);
            iu[1].ensure(n0); ib[1].ensure(n0); ie[1].ensure(n0);
            if (n0) {
                const uint64_t waves = ((uint64_t)n0 + 64 * kLtabR - 1) / (64 * kLtabR);
                launch_blocks(KC_NODES, k_ltab_emit, (size_t)std::min<uint64_t>((waves + 3) / 4, 1u << 20), n0, M0, (const uint32_t*)kt_kid.p,
                              (const uint32_t*)kt_pos.p, (const uint32_t*)lt_off.p, lt_G, lt_EG, (const uint32_t* const*)lt_pb.p,
                              (const uint32_t* const*)lt_pe.p, iu[1].p, ib[1].p, ie[1].p);
            }
            cur = 1;
            Mcur = M0;
            ncur = n0;
            st.start_depth = d0;
            st.trie_nodes += M0;
            if (trace) std::fprintf(stderr, "[edsbwt] start at depth %u from the level table: nodes %u, items %u\n", d0, M0, n0);
            if (ncur == 0) return 0;
            if (hist[d0] && !count_only && lt_fin_direct) {
                // patterns of length d0 end at the start, and their nodes' lists come out of the
                // table sorted by row: the items go to the archive as they are (C5's 8-mers:
                // ~1.5e5 intervals each, which the finisher path would append and radix-sort)
                // (only the finishing nodes' lists go to the archive: a batch with few patterns of
                // length d0 among many longer ones archives few of the start's ~10^9 items)
                node_occ.ensure(M0); foff.ensure(M0 + 1); fend.ensure(M0); fin.ensure(M0); fcnt.ensure(M0);
                launch(KC_FINISH, k_fin_lt_cnt, M0, M0, d0, (const uint32_t*)node_first.p, (const uint32_t*)slen.p, (const uint32_t*)kt_cnt.p,
                       fin.p, fcnt.p);
                const uint32_t F = scan_u32(fcnt.p, foff, M0);
                ab.grow_keep(abase + F, stream);
                ae.grow_keep(abase + F, stream);
                launch_grid(KC_FINISH, k_fin_lt, (unsigned)std::min<uint64_t>(((uint64_t)M0 + 3) / 4, 65536), M0, (const uint8_t*)fin.p,
                            (const uint32_t*)kt_pos.p, (const uint32_t*)kt_cnt.p, (const uint32_t*)ib[1].p, (const uint32_t*)ie[1].p,
                            (const uint32_t*)foff.p, fend.p, node_occ.p, abase, ab.p, ae.p);
                launch(KC_FINISH, k_finish2, P, P, d0, (const uint32_t*)slen.p, (const uint32_t*)nid[1].p, (const uint32_t*)perm.p,
                       (const uint32_t*)foff.p, (const uint32_t*)fend.p, (const uint32_t*)node_occ.p, abase, r);
                abase += F;
            } else if (hist[d0]) {
                // patterns of length d0 end at the start: their nodes' lists (sorted by row in the
                // table) are finished as a depth's finishers are — k_fin_emit over the packed items
                node_occ.ensure(M0); foff.ensure(M0); fend.ensure(M0); fin.ensure(M0);
                launch(KC_NODES, k_zero4, 3 * (size_t)M0, node_occ.p, (uint64_t)M0, foff.p, (uint64_t)M0, fend.p, (uint64_t)M0,
                       (uint32_t*)nullptr, (uint64_t)0);
                zero(lcnt.p, (NSHARD * 32 + 32) * 4);
                launch(KC_FINISH, k_fin_flags, M0, M0, d0, (const uint32_t*)node_first.p, (const uint32_t*)slen.p, fin.p);
                const size_t cap_fin = count_only ? 0 : shard_bound(n0, 1);
                if (!count_only) { efk.ensure(cap_fin * NSHARD); efv.ensure(cap_fin * NSHARD); }
                launch(KC_FINISH, k_fin_emit, n0, n0, (const uint32_t*)iu[1].p, (const uint32_t*)ib[1].p, (const uint32_t*)ie[1].p,
                       (const uint8_t*)fin.p, lcnt.p, count_only ? (uint64_t*)nullptr : efk.p, count_only ? (uint32_t*)nullptr : efv.p,
                       (uint32_t)cap_fin, node_occ.p, X.rowbits, (const uint32_t*)nullptr, 0u);
                uint32_t F = 0;
                if (!count_only) {
                    fetch_shards();
                    F = shard_total(4);
                }
                fk.ensure(F); fv.ensure(F);
                if (F) {
                    unshard2(4, cap_fin, efk.p, efv.p, fk.p, fv.p, F);
                    fk2.ensure(F); fv2.ensure(F);
                    const int endbit = (int)std::min<uint32_t>(64, X.rowbits + bits_for(M0));
                    size_t tb = 0;
                    HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, fk.p, fk2.p, fv.p, fv2.p, cub_n(F), 0, endbit, stream));
                    tmp.ensure(tb);
                    timed(KC_FINISH, [&] { HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, fk.p, fk2.p, fv.p, fv2.p, cub_n(F), 0, endbit, stream)); });
                    sync_check(nullptr, "hipcub call in levels2 (level table finishers)");
                    launch(KC_FINISH, k_fin_bounds, F, F, (const uint64_t*)fk2.p, X.rowbits, foff.p, fend.p);
                    ab.grow_keep(abase + F, stream);
                    ae.grow_keep(abase + F, stream);
                    launch(KC_FINISH, k_fin_archive, F, F, (const uint64_t*)fk2.p, (const uint32_t*)fv2.p, abase, X.rowbits, ab.p, ae.p);
                }
                launch(KC_FINISH, k_finish2, P, P, d0, (const uint32_t*)slen.p, (const uint32_t*)nid[1].p, (const uint32_t*)perm.p,
                       (const uint32_t*)foff.p, (const uint32_t*)fend.p, (const uint32_t*)node_occ.p, abase, r);
                abase += F;
            }
        } else if (d0) {
            const uint32_t M0 = (uint32_t)nodes_at[d0];
            node_scan(d0, P);
            launch(KC_NODES, bps == 3 ? k_node_build<3> : k_node_build<4>, P, P, d0, (const uint32_t*)slen.p, sorted_chunk(d0, P), sigma,
                   (const uint32_t*)lcp.p, (const uint32_t*)scan.p, (const uint32_t*)nid[0].p, nid[1].p, node_first.p, node_parent.p, node_char.p);
            kt_kid.ensure(M0);
            kt_cnt.ensure(M0);
            launch(KC_NODES, bps == 3 ? k_ktab_count<3> : k_ktab_count<4>, M0, M0, d0, sigma - 1, (const uint32_t*)node_first.p,
                   sorted_chunk(1, P), (const uint32_t*)ktab_off.p, kt_kid.p, kt_cnt.p);
            const uint32_t n0 = scan_u32(kt_cnt.p, kt_pos, M0);
            iu[1].ensure(n0); ib[1].ensure(n0); ie[1].ensure(n0);
            if ((uint64_t)n0 > 256ull * M0)  // few nodes, long lists: one thread per item
                launch(KC_NODES, k_ktab_emit_flat, n0, n0, M0, (const uint32_t*)kt_kid.p, (const uint32_t*)kt_pos.p, (const uint32_t*)ktab_off.p,
                       (const uint32_t*)ktab_b.p, (const uint32_t*)ktab_e.p, iu[1].p, ib[1].p, ie[1].p);
            else
                launch(KC_NODES, k_ktab_emit, ((size_t)M0 + 63) / 64 * 64, M0, (const uint32_t*)kt_kid.p, (const uint32_t*)kt_pos.p,
                       (const uint32_t*)ktab_off.p, (const uint32_t*)ktab_b.p, (const uint32_t*)ktab_e.p, iu[1].p, ib[1].p, ie[1].p);
            cur = 1;
            Mcur = M0;
            ncur = n0;
            st.start_depth = d0;
            st.trie_nodes += M0;
            if (trace) std::fprintf(stderr, "[edsbwt] start at depth %u from the k-mer table: nodes %u, items %u\n", d0, M0, n0);
            if (ncur == 0) return 0;  // no pattern's last d0 characters occur
        }
        for (uint32_t d = d0; d < Lmax; d++) {
            const uint32_t D = d + 1;
            const int nxt = cur ^ 1;
            const uint32_t M = (uint32_t)nodes_at[D];
            if (M == 0) break;
            const bool cut_static = !cap && allow_deep && d >= 1 && (double)M >= deep_share * (double)ge[D];
            // no new text items once the lists near the cutover's density (a text item walks at most
            // 16 more characters, so the cutover waits that long at most); C5 from the level table
            // starts where the cutover is already possible but lists are ~10^5 items per node
            if (cut_static && (double)ncur <= text_stop_items * (double)Mcur) text_stop = true;
            if (cut_static && text_alive == 0 && (double)ncur <= deep_items * (double)Mcur) {
                gend.ensure(Mcur);
                if (d0 && d == d0) {
                    // the table's items are already grouped by node: [kt_pos[u], + kt_cnt[u])
                    launch(KC_MERGE, k_group_end, Mcur, Mcur, (const uint32_t*)kt_pos.p, (const uint32_t*)kt_cnt.p, gend.p);
                    novf = run_deep(d, M, P, ge[D], d_bytes, d_off, nid[cur].p, kt_pos.p, gend.p, ib[cur].p, ie[cur].p, r, abase,
                                    ovf_orig);
                    break;
                }
                if (in_sharded) pack_items(cur);
                // group the unordered items by node, then finish patterns one per thread
                gcnt.ensure(Mcur); gfill.ensure(Mcur); goff.ensure(Mcur);
                launch(KC_MERGE, k_zero4, 2 * (size_t)Mcur, gcnt.p, (uint64_t)Mcur, gfill.p, (uint64_t)Mcur, (uint32_t*)nullptr, (uint64_t)0,
                       (uint32_t*)nullptr, (uint64_t)0);
                launch(KC_MERGE, k_group_count, ncur, ncur, (const uint32_t*)iu[cur].p, gcnt.p);
                exclusive_scan(gcnt.p, goff.p, Mcur);
                gb.ensure(ncur); gee.ensure(ncur);
                launch(KC_MERGE, k_group_scatter, ncur, ncur, (const uint32_t*)iu[cur].p, (const uint32_t*)ib[cur].p, (const uint32_t*)ie[cur].p,
                       (const uint32_t*)goff.p, gfill.p, gb.p, gee.p);
                launch(KC_MERGE, k_group_end, Mcur, Mcur, (const uint32_t*)goff.p, (const uint32_t*)gcnt.p, gend.p);
                novf = run_deep(d, M, P, ge[D], d_bytes, d_off, nid[cur].p, goff.p, gend.p, gb.p, gee.p, r, abase, ovf_orig);
                break;
            }
            st.depths++;
            st.trie_nodes += M;
            const bool finishing = hist[D] != 0;
            // count only: the step itself sums the finishing children's occurrences (child_info
            // marks them), so no finisher pass reads this depth's items again
            const bool fuse_fin = finishing && count_only && !cap && fuse_finish;
            // one zeroing launch: shard counters, child links of the parents, finisher tables
            child_info.ensure(Mcur);
            if (finishing) { node_occ.ensure(M); foff.ensure(M); fend.ensure(M); fin.ensure(M); }
            launch(KC_NODES, k_zero4, (size_t)NSHARD * 32 + 32 + 2 * (size_t)Mcur, lcnt.p, (uint64_t)NSHARD * 32 + 32,
                   (uint32_t*)child_info.p, 2 * (uint64_t)Mcur, (uint32_t*)nullptr, (uint64_t)0, (uint32_t*)nullptr, (uint64_t)0);
            if (finishing)
                launch(KC_NODES, k_zero4, 3 * (size_t)M, node_occ.p, (uint64_t)M, foff.p, (uint64_t)M, fend.p, (uint64_t)M, (uint32_t*)nullptr,
                       (uint64_t)0);
            // children nodes at depth D (node count known from build_trie: no read-back)
            node_scan(D, P);
            launch(KC_NODES, bps == 3 ? k_node_build<3> : k_node_build<4>, P, P, D, (const uint32_t*)slen.p, sorted_chunk(D, P), sigma, (const uint32_t*)lcp.p,
                   (const uint32_t*)scan.p, (const uint32_t*)nid[cur].p, nid[nxt].p, node_first.p, node_parent.p, node_char.p);
            launch(KC_NODES, k_child_info, M, M, (const uint32_t*)node_parent.p, (const uint8_t*)node_char.p, child_info.p, D,
                   fuse_fin ? (const uint32_t*)node_first.p : (const uint32_t*)nullptr, (const uint32_t*)slen.p);
            // fused step + '#'-row emission over the current items (sharded appends)
            size_t cap_next = std::max<size_t>(shard_bound(ncur, 2), 4096);
            size_t cap_keys = std::max<size_t>(shard_bound(ncur, 1), 4096);
            size_t cap_chunks = std::max<size_t>(shard_bound(ncur, 1) / 8, 1024);
            // use what earlier depths / calls already allocated: no regrow-and-redo in steady state
            cap_next = std::max(cap_next, std::min({eu.cap, eb.cap, ee.cap}) / NSHARD);
            cap_keys = std::max(cap_keys, ekeys.cap / NSHARD);
            cap_chunks = std::max(cap_chunks, std::min({eck_u.cap, eck_k.cap, eck_e.cap}) / NSHARD);
            for (bool first = true;; first = false) {
                eu.ensure(cap_next * NSHARD); eb.ensure(cap_next * NSHARD); ee.ensure(cap_next * NSHARD);
                ekeys.ensure(cap_keys * NSHARD);
                eck_u.ensure(cap_chunks * NSHARD); eck_k.ensure(cap_chunks * NSHARD); eck_e.ensure(cap_chunks * NSHARD);
                if (!first) zero(lcnt.p, NSHARD * 32 * 4);
                if (d > 0)
                    launch(KC_STEP, lvl_waves >= 8 ? k_lvl_items<true, 8> : lvl_waves >= 7 ? k_lvl_items<true, 7> : k_lvl_items<true>, ncur, ncur, (const uint32_t*)(in_sharded ? fu.p : iu[cur].p),
                           (const uint32_t*)(in_sharded ? fb.p : ib[cur].p), (const uint32_t*)(in_sharded ? fe.p : ie[cur].p),
                           (const uint64_t*)child_info.p, X, eu.p, eb.p, ee.p, (uint32_t)cap_next, lcnt.p, ekeys.p, (uint32_t)cap_keys, eck_u.p,
                           eck_k.p, eck_e.p, (uint32_t)cap_chunks, stats.p, (const uint32_t*)(in_sharded ? fpre.p : nullptr), (uint32_t)fcap,
                           fuse_fin && first ? node_occ.p : (uint32_t*)nullptr, titems ? (text_stop ? 1u : 3u) : 0u);
                else  // no link before the first step (:246-258)
                    launch(KC_STEP, lvl_waves >= 8 ? k_lvl_items<false, 8> : lvl_waves >= 7 ? k_lvl_items<false, 7> : k_lvl_items<false>, ncur, ncur, (const uint32_t*)(in_sharded ? fu.p : iu[cur].p),
                           (const uint32_t*)(in_sharded ? fb.p : ib[cur].p), (const uint32_t*)(in_sharded ? fe.p : ie[cur].p),
                           (const uint64_t*)child_info.p, X, eu.p, eb.p, ee.p, (uint32_t)cap_next, lcnt.p, ekeys.p, (uint32_t)cap_keys, eck_u.p,
                           eck_k.p, eck_e.p, (uint32_t)cap_chunks, stats.p, (const uint32_t*)(in_sharded ? fpre.p : nullptr), (uint32_t)fcap,
                           fuse_fin && first ? node_occ.p : (uint32_t*)nullptr, titems ? (text_stop ? 1u : 3u) : 0u);
                fetch_shards();  // sync A
                const uint32_t m0 = shard_max(0), m1 = shard_max(1), m2 = shard_max(2);
                if (m0 <= cap_next && m1 <= cap_keys && m2 <= cap_chunks) break;
                cap_next = std::max<size_t>(cap_next, m0 + m0 / 4 + 1024);
                cap_keys = std::max<size_t>(cap_keys, m1 + m1 / 4 + 1024);
                cap_chunks = std::max<size_t>(cap_chunks, m2 + m2 / 4 + 256);
            }
            text_alive = titems ? shard_total(5) : 0u;
            const uint32_t nchunks = shard_total(2);
            st.intervals_stepped += ncur;
            const std::vector<uint32_t> keep_keys = shard_counts(1);
            if (nchunks) {  // long '#'-row ranges: pack, then one chunk per thread
                ck_u.ensure(nchunks); ck_k.ensure(nchunks); ck_e.ensure(nchunks);
                unshard3(2, cap_chunks, eck_u.p, eck_k.p, eck_e.p, ck_u.p, ck_k.p, ck_e.p, nchunks);
                for (;;) {
                    launch(KC_LINK, k_lvl_chunks, (size_t)nchunks * 64, nchunks, (const uint32_t*)ck_u.p, (const uint32_t*)ck_k.p, (const uint32_t*)ck_e.p, X,
                           lcnt.p, ekeys.p, (uint32_t)cap_keys);
                    fetch_shards();
                    const uint32_t m1 = shard_max(1);
                    if (m1 <= cap_keys) break;
                    // grow the key shards keeping what k_lvl_items wrote, then redo the chunks
                    DBuf<uint64_t> nk;
                    const size_t ncap = m1 + m1 / 4 + 1024;
                    nk.ensure(ncap * NSHARD);
                    for (uint32_t sh = 0; sh < NSHARD; sh++)
                        HIPCHK(hipMemcpyAsync(nk.p + sh * ncap, ekeys.p + sh * cap_keys, (size_t)keep_keys[sh] * 8, hipMemcpyDeviceToDevice, stream));
                    HIPCHK(hipStreamSynchronize(stream));
                    std::swap(nk.p, ekeys.p);
                    std::swap(nk.cap, ekeys.cap);
                    nk.release();
                    for (uint32_t sh = 0; sh < NSHARD; sh++) hsh[sh * 32 + 1] = keep_keys[sh];
                    std::memcpy(pinned_big, hsh.data(), NSHARD * 32 * 4);
                    small_copy(lcnt.p, pinned_big, NSHARD * 32 * 4);
                    cap_keys = ncap;
                }
            }
            const uint32_t nkeys = shard_total(1);
            st.link_hash_rows += nkeys;
            uint32_t nnext = shard_total(0);
            if (nkeys) {
                // link: sort (node, segment), maximal runs of previous-segment ranges, step them
                lkeys.ensure(nkeys);
                lkeys2.ensure(nkeys);
                unshard1(1, cap_keys, ekeys.p, lkeys.p, nkeys);
                const int endbit = (int)std::min<uint32_t>(64, X.segbits + X.link_cb + bits_for(Mcur));
                sort_link_keys(lkeys.p, lkeys2.p, nkeys, endbit);
                rflag.ensure(nkeys);
                rscan.ensure(nkeys);
                launch(KC_LINK, k_run_flags, nkeys, (const uint64_t*)lkeys2.p, (uint64_t)nkeys, (const uint32_t*)seg_lo.p, X.segbits, rflag.p,
                       (const uint32_t*)seg_chain.p, X.link_cb);
                exclusive_scan(rflag.p, rscan.p, nkeys);
                rb.ensure(nkeys); re.ensure(nkeys); ru.ensure(nkeys);
                launch(KC_LINK, k_run_build_seg, nkeys, (const uint64_t*)lkeys2.p, (uint64_t)nkeys, (const uint32_t*)rflag.p,
                       (const uint32_t*)rscan.p, X.segbits, rb.p, re.p, ru.p, d_runs, X.link_cb);
                const std::vector<uint32_t> keep_items = shard_counts(0);
                for (bool dfirst = true;; dfirst = false) {
                    // (a redo after a regrow adds no counts: the first launch counted every item)
                    launch(KC_STEP, lvl_waves >= 8 ? k_lvl_dollar<8> : k_lvl_dollar<1>, nkeys, (const uint32_t*)d_runs, (const uint32_t*)ru.p, (const uint32_t*)rb.p, (const uint32_t*)re.p,
                           (const uint64_t*)child_info.p, X, eu.p, eb.p, ee.p,
                           (uint32_t)cap_next, lcnt.p, stats.p, fuse_fin && dfirst ? node_occ.p : (uint32_t*)nullptr,
                           titems ? (text_stop ? 1u : 3u) : 0u);
                    fetch_shards();  // sync B
                    const uint32_t m0 = shard_max(0);
                    if (m0 <= cap_next) break;
                    // grow the item shards keeping k_lvl_items' output, then redo the dollar step
                    const size_t ncap = m0 + m0 / 4 + 1024;
                    regrow3(eu, eb, ee, cap_next, ncap, keep_items);
                    for (uint32_t sh = 0; sh < NSHARD; sh++) hsh[sh * 32 + 0] = keep_items[sh];
                    std::memcpy(pinned_big, hsh.data(), NSHARD * 32 * 4);
                    small_copy(lcnt.p, pinned_big, NSHARD * 32 * 4);
                    cap_next = ncap;
                }
                // the dollar step makes text items too (KIdx::segtext): the count after it (a redo
                // after a regrow counts some twice, which only delays the cutover)
                if (titems) text_alive = shard_total(5);
                const uint32_t R = hsh[NSHARD * 32];
                st.link_ranges += R;
                st.intervals_stepped += R;
                st.bytes_kernel[KC_STEP] += (uint64_t)R * 12;  // the runs read (their lines: ST_STEP_BLOCKS)
                nnext = shard_total(0);
            }
            // the item streams (12 B read per item, 12 B written per next item, 8 B per link key);
            // the random lines the step kernels gather are counted by them (ST_STEP_BLOCKS, 64 B
            // each, added in finish_stats): a text item reads none, a single row one, an interval
            // whose ends share a line one (round 3 charged every item 2 x 64 B: C5's model then
            // exceeded its DRAM traffic)
            st.bytes_kernel[KC_STEP] += (uint64_t)ncur * 12 + (uint64_t)nnext * 12 + (uint64_t)nkeys * 8;
            if (trace) {
                // single-row items and lines read by this depth's step (stats so far, less the last depth's)
                small_copy(pinned_stats, stats.p, kStatSlots * 8);
                HIPCHK(hipStreamSynchronize(stream));
                const std::vector<uint64_t> sv = fold_pinned_stats();
                std::fprintf(stderr, "[edsbwt] depth %u: nodes %u, items %u (single-row %llu), link keys %u, link ranges %u, next items %u, "
                                     "step lines %llu\n", D, M, ncur, (unsigned long long)(sv[ST_LVL_SINGLE] - trace_single),
                             nkeys, nkeys ? hsh[NSHARD * 32] : 0u, nnext, (unsigned long long)(sv[ST_STEP_BLOCKS] - trace_lines));
                trace_single = sv[ST_LVL_SINGLE];
                trace_lines = sv[ST_STEP_BLOCKS];
            }
            // hand the item shards to the next depth as they are (k_lvl_items reads them in
            // place); they are packed only for the finishers below or the deep cutover
            {
                uint32_t* pre = pinned_big + kCnt + NSHARD + 8;  // own staging: upload_prefix uses pinned_big + kCnt
                pre[0] = 0;
                for (uint32_t sh = 0; sh < NSHARD; sh++) pre[sh + 1] = pre[sh] + hsh[sh * 32 + 0];
                fpre.ensure(NSHARD + 1);
                small_copy(fpre.p, pre, (NSHARD + 1) * 4);
                std::swap(fu, eu); std::swap(fb, eb); std::swap(fe, ee);
                fcap = cap_next;
                in_sharded = true;
            }
            if (cap) {  // table build: keep this depth's items as (D-mer, b, e) while they fit
                if (nnext > cap->budget) break;
                cap->reached = D;
                if (cap->only_last && D < cap->K) {  // the level table keeps depth K only
                    if (nnext == 0) { cap->depth = cap->K; cap->n = 0; break; }  // no K-mer of this group occurs
                    cur = nxt;
                    Mcur = M;
                    ncur = nnext;
                    continue;
                }
                cap->k.ensure(nnext); cap->b.ensure(nnext); cap->e.ensure(nnext);
                if (nnext) {
                    launch(KC_TABLE, k_unshard<uint32_t, uint32_t, uint32_t>, nnext, nnext, (const uint32_t*)fpre.p, (uint32_t)fcap,
                           (const uint32_t*)fu.p, (const uint32_t*)fb.p, (const uint32_t*)fe.p, cap->k.p, cap->b.p, cap->e.p);
                    uint64_t BD = 1;
                    for (uint32_t t = 0; t < D; t++) BD *= cap->B;
                    launch(KC_TABLE, k_ktab_capture_map, nnext, (uint64_t)nnext, cap->k.p, (const uint32_t*)node_first.p, (const uint32_t*)perm.p, BD);
                }
                cap->depth = D;
                cap->n = nnext;
                if (D >= cap->K || nnext == 0) break;
                cur = nxt;
                Mcur = M;
                ncur = nnext;
                continue;
            }
            // finish patterns of length D: their node's items, sorted by row
            if (finishing) {
                // the items stay in their shards (k_fin_emit reads them in place, as the next
                // depth's k_lvl_items does)
                const size_t cap_fin = count_only ? 0 : shard_bound(nnext, 1);
                if (!count_only) { efk.ensure(cap_fin * NSHARD); efv.ensure(cap_fin * NSHARD); }
                if (!fuse_fin) launch(KC_FINISH, k_fin_flags, M, M, D, (const uint32_t*)node_first.p, (const uint32_t*)slen.p, fin.p);
                // count only: per-node occurrence sums, no interval archive (C5-scale batches
                // finish billions of intervals); fused into the step unless EDSBWT_FUSE_FINISH=0
                if (!fuse_fin) launch(KC_FINISH, k_fin_emit, nnext, nnext, (const uint32_t*)fu.p, (const uint32_t*)fb.p, (const uint32_t*)fe.p,
                       (const uint8_t*)fin.p, lcnt.p, count_only ? (uint64_t*)nullptr : efk.p, count_only ? (uint32_t*)nullptr : efv.p,
                       (uint32_t)cap_fin, node_occ.p, X.rowbits, (const uint32_t*)fpre.p, (uint32_t)fcap);
                uint32_t F = 0;
                if (!count_only) {
                    fetch_shards();
                    F = shard_total(4);
                }
                fk.ensure(F); fv.ensure(F);
                if (F) {
                    unshard2(4, cap_fin, efk.p, efv.p, fk.p, fv.p, F);
                    fk2.ensure(F); fv2.ensure(F);
                    const int endbit = (int)std::min<uint32_t>(64, X.rowbits + bits_for(M));
                    size_t tb = 0;
                    HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, fk.p, fk2.p, fv.p, fv2.p, cub_n(F), 0, endbit, stream));
                    tmp.ensure(tb);
                    timed(KC_FINISH, [&] { HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, fk.p, fk2.p, fv.p, fv2.p, cub_n(F), 0, endbit, stream)); });
                    sync_check(nullptr, "hipcub call at engine.hip:1257");
                    launch(KC_FINISH, k_fin_bounds, F, F, (const uint64_t*)fk2.p, X.rowbits, foff.p, fend.p);
                    ab.grow_keep(abase + F, stream);
                    ae.grow_keep(abase + F, stream);
                    launch(KC_FINISH, k_fin_archive, F, F, (const uint64_t*)fk2.p, (const uint32_t*)fv2.p, abase, X.rowbits, ab.p, ae.p);
                }
                launch(KC_FINISH, k_finish2, P, P, D, (const uint32_t*)slen.p, (const uint32_t*)nid[nxt].p, (const uint32_t*)perm.p,
                       (const uint32_t*)foff.p, (const uint32_t*)fend.p, (const uint32_t*)node_occ.p, abase, r);
                abase += F;
            }
            cur = nxt;
            Mcur = M;
            ncur = nnext;
            if (ncur == 0) break;
        }
        return novf;
    }

    // One batch: the trie walk (order-free unless patterns hold '#'), then the patterns
    // k_deep could not hold re-run through the unbounded level path.
    void run_batch(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t P, bool allow_deep, bool ordered, Res* r, uint64_t& abase) {
        uint32_t novf = kNotDirect;
        if (!ordered && allow_deep) {
            in_direct = true;
            try {
                novf = direct(d_off, d_bytes, P, r, abase, ovf_orig.p);
            } catch (...) {
                in_direct = false;
                throw;
            }
            in_direct = false;
        }
        if (novf == kNotDirect || novf == kNeedOrdered) settle_res(r);
        if (novf == kNeedOrdered) ordered = true;
        if (!ordered && novf == kNotDirect) {
            novf = levels2(d_bytes, d_off, P, allow_deep, r, abase, ovf_orig.p);
            if (novf == kNeedOrdered) ordered = true;
        }
        if (ordered) novf = levels(d_bytes, d_off, P, allow_deep, r, abase, ovf_orig.p);
        if (!novf) return;
        // patterns k_deep could not hold: gather them and run the unbounded level path
        const uint32_t n = scan_u32(ovf_orig.p, ovf_scan, P);
        sub_map.ensure(n);
        sub_len.ensure(n + 1);
        launch(KC_MERGE, k_sub_build, P, P, (const uint32_t*)ovf_orig.p, (const uint32_t*)ovf_scan.p, (const uint32_t*)len.p, sub_map.p, sub_len.p);
        const uint64_t nbytes = scan_u64(sub_len.p, sub_off, n);
        sub_bytes.ensure(nbytes + 1);
        launch(KC_MERGE, k_sub_bytes, n, (uint64_t)n, (const uint32_t*)sub_map.p, d_off, (const uint64_t*)sub_off.p, d_bytes, sub_bytes.p);
        sub_res.ensure(n);
        zero(sub_res.p, (size_t)n * sizeof(Res));
        if (ordered) levels(sub_bytes.p, sub_off.p, n, false, sub_res.p, abase, ovf_orig.p);
        else levels2(sub_bytes.p, sub_off.p, n, false, sub_res.p, abase, ovf_orig.p);
        launch(KC_MERGE, k_sub_scatter, n, (uint64_t)n, (const uint32_t*)sub_map.p, (const Res*)sub_res.p, r);
    }

    // The batch as separate trie subtrees: patterns grouped by their last k characters
    // (the first k levels of the reversed-pattern trie), each group one run_batch, so a
    // depth's items split over the groups.  Results land in res_* as for one batch.
    void run_grouped(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t P, bool allow_deep, bool ordered, uint32_t k, uint64_t& abase) {
        abase = 0;
        zero(res.p, P * sizeof(Res));
        res_unzeroed = false;
        glen.ensure(P);
        gid.ensure(P);
        gflag.ensure(P);
        launch(KC_TRIE, k_lens, P, d_off, P, glen.p);
        launch(KC_TRIE, k_pattern_group, P, d_bytes, d_off, P, (const uint8_t*)code_of.p, sigma, k, gid.p);
        uint32_t G = 1;
        for (uint32_t t = 0; t < k; t++) G *= sigma + 2;
        for (uint32_t g = 0; g < G; g++) {
            launch(KC_TRIE, k_eq_flag, P, (const uint32_t*)gid.p, P, g, gflag.p);
            const uint32_t n = scan_u32(gflag.p, gscan, P);
            if (!n) continue;
            g_map.ensure(n);
            g_len.ensure(n + 1);
            launch(KC_TRIE, k_sub_build, P, P, (const uint32_t*)gflag.p, (const uint32_t*)gscan.p, (const uint32_t*)glen.p, g_map.p, g_len.p);
            const uint64_t nbytes = scan_u64(g_len.p, g_off, n);
            g_bytes.ensure(nbytes + 1);
            launch(KC_TRIE, k_sub_bytes, n, (uint64_t)n, (const uint32_t*)g_map.p, d_off, (const uint64_t*)g_off.p, d_bytes, g_bytes.p);
            g_res.ensure(n);
            zero(g_res.p, (size_t)n * sizeof(Res));
            tag_map = g_map.p;
            struct MapReset { const uint32_t*& m; ~MapReset() { m = nullptr; } } mr{tag_map};
            run_batch(g_bytes.p, g_off.p, n, allow_deep, ordered, g_res.p, abase);
            launch(KC_TRIE, k_sub_scatter, n, (uint64_t)n, (const uint32_t*)g_map.p, (const Res*)g_res.p, res.p);
        }
        st.search_groups = G;
    }

    // reorder rec[0..n) into the legacy engine's order (k_legacy_keys)
    void legacy_order(uint64_t n, uint64_t P, uint32_t first_id) {
        if (n > 0x7fffffffull) throw Fail(EDSBWT_E_UNSUPPORTED, "legacy order over >2^31 records");
        const uint32_t kbits = bits_for(W), obits = bits_for(N);
        if (kbits + obits > 64) throw Fail(EDSBWT_E_UNSUPPORTED, "legacy order key wider than 64 bits");
        lk.ensure(n); lk2.ensure(n); lp.ensure(n); lp2.ensure(n); li.ensure(n); li2.ensure(n);
        launch(KC_LOCATE, k_legacy_keys, n, (uint64_t)n, (const edsbwt_occ*)rec.p, (const uint32_t*)kpos.p, kbits, lk.p, lp.p, li.p);
        size_t tb = 0;
        HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, lk.p, lk2.p, li.p, li2.p, cub_n(n), 0, (int)(kbits + obits), stream));
        tmp.ensure(tb);
        HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, lk.p, lk2.p, li.p, li2.p, cub_n(n), 0, (int)(kbits + obits), stream));
        sync_check(nullptr, "hipcub call at engine.hip:1351");
        // stable by pattern: gather the pattern ids in key order, then sort them carrying the indices
        launch(KC_LOCATE, k_gather_u32, n, (const uint32_t*)lp.p, (const uint32_t*)li2.p, (uint64_t)n, lp2.p);
        const int pbits = (int)bits_for((uint64_t)first_id + P);
        tb = 0;
        HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, lp2.p, lp.p, li2.p, li.p, cub_n(n), 0, pbits, stream));
        tmp.ensure(tb);
        HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, lp2.p, lp.p, li2.p, li.p, cub_n(n), 0, pbits, stream));
        sync_check(nullptr, "hipcub call at engine.hip:1358");
        rec2.ensure(n);
        launch(KC_LOCATE, k_gather_rec, n, (uint64_t)n, (const uint32_t*)li.p, (const edsbwt_occ*)rec.p, rec2.p);
        std::swap(rec.p, rec2.p);
        std::swap(rec.cap, rec2.cap);
    }

    // d_bytes/d_off/d_counts are device pointers; returns number of records
    uint64_t search(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t P, uint32_t first_id, uint32_t flags, uint32_t* d_counts) {
        t_search0 = std::chrono::steady_clock::now();
        st = edsbwt_stats{};
        trace_single = trace_lines = 0;
        guessed_len = false;
        prof = (flags & (EDSBWT_PROFILE | EDSBWT_PROFILE_LIGHT)) != 0;
        prof_mask = (flags & EDSBWT_PROFILE) ? ~0u
                                             : ((1u << KC_STEP) | (1u << KC_DEEP) | (1u << KC_DEEPQ) | (1u << KC_DEEPW) | (1u << KC_LOCATE) |
                                                (1u << KC_LINKSORT));
        deep_stats = deep_stats_env && !(flags & EDSBWT_NO_COUNTERS);
        const bool locate = (flags & EDSBWT_LOCATE) && !(flags & EDSBWT_COUNT_ONLY);
        const bool use_table = locate && (flags & EDSBWT_LOCATE_TABLE);
        count_only = !locate;
        const int loc_mode = use_table ? 1 : ((flags & EDSBWT_LOCATE_WALK) || !have_samples) ? 0 : 2;
        const bool allow_deep = !(flags & EDSBWT_NO_DEEP);
        no_wide = (flags & EDSBWT_NO_WIDE) != 0;
        use_ktab = (flags & EDSBWT_NO_KTAB) == 0;
        use_ltab = use_ktab && env_double("EDSBWT_NO_LTAB", 0) == 0;
        use_pairs = (flags & EDSBWT_NO_PAIRS) == 0 && env_double("EDSBWT_NO_PAIRS", 0) == 0;
        use_direct = (flags & EDSBWT_NO_DIRECT) == 0 && env_double("EDSBWT_NO_DIRECT", 0) == 0;
        // the single-row text compare answers with (word, offset): the reference walk and table
        // locate modes keep their row-based records
        text_on = (flags & (EDSBWT_NO_TEXT | EDSBWT_LOCATE_WALK | EDSBWT_LOCATE_TABLE)) == 0 && env_double("EDSBWT_NO_TEXT", 0) == 0;
        if (use_table) build_table();
        st.patterns = P;
        defer = false;
        defer_call = defer_ok && !(flags & (kFlagNoDefer | EDSBWT_LEGACY_ORDER)) && !force_groups && !sticky_groups;
        fc_done = false;
        fc_counts = nullptr;
        // (count-only; the per-pattern locate writes them in k_count_tiles or k_locate_pp instead, finish_deferred)
        // (located: only when finish_deferred takes the per-pattern locate with record-offset tiles —
        // the path whose k_tile_sums reads these counts; every other located path sums them itself)
        const bool loc_tiles = locate && loc_mode == 2 && have_samples && samp_shift == 0 && locate_pp && !locate_counts && tile_scan;
        if (defer_call && fused_counts && (deep_wave || no_wide) && (!locate || (loc_fc && loc_tiles))) fc_counts = d_counts;
        // (the early tiles: exactly the path finish_deferred takes k_count_tiles on)
        early_counts = defer_call && loc_tiles && !fc_counts && deep_wave && !no_wide && wave_tiles ? d_counts : nullptr;
        join_early();  // (a previous search that failed after queueing them)
        in_direct = false;
        if (P == 0) return 0;
        struct EvPair {  // released on every exit, including exceptions
            hipEvent_t a = nullptr, b = nullptr;
            ~EvPair() { if (a) (void)hipEventDestroy(a); if (b) (void)hipEventDestroy(b); }
        } ep;
        HIPCHK(hipEventCreate(&ep.a));
        HIPCHK(hipEventCreate(&ep.b));
        hipEvent_t e0 = ep.a, e1 = ep.b;
        HIPCHK(hipEventRecord(e0, stream));
        hmark("events");
        // a search that throws leaves no timing events behind for the next call
        struct EvRecycle {
            Engine* E;
            bool done = false;
            ~EvRecycle() { if (!done) E->discard_attempt(); }
        } recycle{this};
        const KIdx X = kidx();
        res.ensure(P);
        ovf_orig.ensure(P);
        if (defer_call) {
            // one zeroing launch for everything the deferred direct start counts into (see
            // direct(), run_deep(), finish_deferred(); they skip their own zeroing when defer)
            tflag.ensure(P + 1);
            hcnt.ensure((size_t)std::min<uint64_t>(P, wide_cap) + 1);
            lcnt.ensure(NSHARD * 32 + 32);
            oscan.ensure(P + 1);
            const uint64_t nb = direct_buckets();
            if (nb) bhist.ensure(nb + 1);
            lbig.ensure(P + 1);  // (the per-pattern locate's big list: its counter is zeroed here)
            // (the result array only when the search does not turn out to be k_deep_direct's, which
            // writes every result: res_unzeroed, settled by run_batch / run_deep)
            if (deep_pieces > 1) pcnt.ensure((size_t)NSHARD * 32 * deep_pieces);
            zero_many({{stats.p, kStatSlots * 8}, {counters.p, 24 * 8}, {tflag.p, 4}, {hcnt.p, 4},
                       {lcnt.p, NSHARD * 32 * 4}, {oscan.p, 8}, {bhist.p, nb ? (nb + 1) * 4 : 0}, {lbig.p, 4},
                       {pcnt.p, deep_pieces > 1 ? (size_t)NSHARD * 32 * deep_pieces * 4 : 0}});
            res_unzeroed = true;
        } else {
            zero(res.p, P * sizeof(Res));
            zero(stats.p, kStatSlots * 8);
            res_unzeroed = false;
        }
        uint64_t abase = 0;
        // patterns holding '#' make the reference's lists overlap: they take the ordered path
        const bool ordered = (flags & EDSBWT_ORDERED) != 0;
        try {
            const uint32_t g0 = force_groups ? force_groups : sticky_groups;
            if (g0) run_grouped(d_bytes, d_off, P, allow_deep, ordered, g0, abase);
            else run_batch(d_bytes, d_off, P, allow_deep, ordered, res.p, abase);
        } catch (const TooBig&) {
            join_early();  // (the early tiles of the failed attempt, if queued, end before anything is reused)
            // a depth outgrew 32-bit counts (e.g. a 1 Gchar EDS with many empty words):
            // search the batch as separate trie subtrees, grouped by the last k characters;
            // later batches on this index start grouped (sticky_groups)
            for (uint32_t k = std::max(2u, sticky_groups + 1);; k++) {
                try {
                    // the failed attempt's counters and timings are not this search's
                    discard_attempt();
                    defer_call = defer = false;
                    st = edsbwt_stats{};
                    trace_single = trace_lines = 0;
                    st.patterns = P;
                    zero(res.p, P * sizeof(Res));
                    res_unzeroed = false;
                    zero(stats.p, kStatSlots * 8);
                    abase = 0;
                    run_grouped(d_bytes, d_off, P, allow_deep, ordered, k, abase);
                    sticky_groups = k;
                    break;
                } catch (const TooBig&) {
                    if (k >= 4) throw;
                }
            }
        }
        if (defer) {
            const uint64_t n = finish_deferred(P, first_id, locate, loc_mode, d_counts, e1);
            if (n != kRedo) {
                recycle.done = true;
                return finish_stats(P, locate, use_table, loc_mode, n, e0, e1);
            }
            // a deferred check failed: the batch again on the checked path (inputs are untouched)
            if (guessed_len) len_guess = false;
            discard_attempt();
            recycle.done = true;
            const uint64_t m = search(d_bytes, d_off, P, first_id, flags | kFlagNoDefer, d_counts);
            st.redo_searches++;
            if (tag_now) {
                hipLaunchKernelGGL(k_tag_all, dim3((unsigned)std::min<uint64_t>(65535, (P + 255) / 256)), dim3(256), 0, stream, ptag.p, P,
                                   (uint32_t)EDSBWT_PATH_REDO);
                HIPCHK(hipGetLastError());
            }
            return m;
        }
        // ---- D. counts (backwardSearch's return value) and locate; one read-back for the sizes
        last_locate_pp = false;
        zero(counters.p + 1, 8);
        zero(counters.p + 12, 16);
        if (locate) occ64.ensure(P);
        // counts, found, totals and (locate) the packed scan input in one pass over the results
        launch_reduce(KC_FINISH, k_count_found, (const Res*)res.p, P, d_counts, counters.p + 1, counters.p + 12,
                      locate ? occ64.p : (uint64_t*)nullptr);
        emit_c8(P, d_counts);
        if (locate) inclusive_scan_u64(occ64.p, oscan, P);  // occurrence and task offsets: one scan of both
        small_copy(pinned, counters.p + 1, 8);
        small_copy(pinned + 2, counters.p + 12, 16);
        HIPCHK(hipStreamSynchronize(stream));
        uint64_t rb3[3];
        std::memcpy(rb3, pinned, 24);
        st.found = rb3[0];
        st.not_found = P - st.found;
        uint64_t OCC = 0;
        if (locate) {
            OCC = rb3[1];
            const uint64_t TT = rb3[2];
            const uint64_t* tsc = nullptr;
            if (OCC >> 32 || TT >> 32 || split_scans) {  // totals past 32 bits: the two scans apart
                tc64.ensure(P);
                launch(KC_LOCPREP, k_res_scan_in, P, (const Res*)res.p, P, occ64.p, tc64.p);
                inclusive_scan_u64(occ64.p, oscan, P);
                inclusive_scan_u64(tc64.p, tscan64, P);
                tsc = tscan64.p;
            }
            if (OCC && loc_mode == 2 && X.samp_dense && locate_lists) {
                // dense samples: each pattern's records straight from its list (k_locate_lists), no tasks
                rec.ensure(OCC);
                launch_grid(KC_LOCATE, k_locate_lists, (unsigned)std::min<uint64_t>((P + 3) / 4, 65536), P, (const Res*)res.p,
                            (const uint64_t*)oscan.p, tsc ? 0u : 1u, first_id, pat_ids, X, (const uint32_t*)ab.p, (const uint32_t*)ae.p,
                            rec.p, stats.p);
                if (flags & EDSBWT_LEGACY_ORDER) legacy_order(OCC, P, first_id);
            } else if (OCC) {
                trow.ensure(TT); tout.ensure(TT); tpat.ensure(TT);
                blk_first.ensure(OCC / kLocRun + 1);
                if (TT <= 0x7fffffffull && (tasks_wave == 2 || (tasks_wave == 1 && TT > kTasksWaveRatio * P))) {
                    // long lists (C5's 8-mers): tasks one wave per pattern, their offsets one scan
                    tc64.ensure(TT);
                    launch_grid(KC_LOCPREP, k_tasks_wave, (unsigned)std::min<uint64_t>((P + 3) / 4, 65536), P, (const Res*)res.p, tsc,
                                (const uint64_t*)oscan.p, (const uint32_t*)ab.p, (const uint32_t*)ae.p, trow.p, tc64.p, tpat.p);
                    size_t tb = 0;
                    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, tc64.p, tout.p, cub_n(TT), stream));
                    tmp.ensure(tb);
                    timed(KC_LOCPREP, [&] { HIPCHK(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb, tc64.p, tout.p, cub_n(TT), stream)); });
                    sync_check(nullptr, "hipcub call (task offsets)");
                    const uint64_t nblk = (OCC + kLocRun - 1) / kLocRun;
                    launch(KC_LOCPREP, k_blk_first, nblk, nblk, (const uint64_t*)tout.p, TT, blk_first.p);
                } else {
                    launch(KC_LOCPREP, k_tasks, P, P, (const Res*)res.p, tsc,
                           (const uint64_t*)oscan.p, (const uint32_t*)ab.p, (const uint32_t*)ae.p, trow.p, tout.p, tpat.p, blk_first.p,
                           ~0ull, ~0ull, (uint32_t*)(counters.p + 20));
                }
                rec.ensure(OCC);
                launch(KC_LOCATE, k_locate, OCC, OCC, TT, (const uint64_t*)tout.p, (const uint32_t*)trow.p, (const uint32_t*)tpat.p,
                       (const uint64_t*)blk_first.p, first_id, pat_ids, X, loc_mode, rec.p, stats.p, (const Res*)res.p,
                       (const unsigned long long*)nullptr, (const uint32_t*)nullptr);
                if (flags & EDSBWT_LEGACY_ORDER) legacy_order(OCC, P, first_id);  // (refused with pat_ids)
            }
        }
        small_copy(pinned_stats, stats.p, kStatSlots * 8);
        HIPCHK(hipEventRecord(e1, stream));
        HIPCHK(hipStreamSynchronize(stream));
        recycle.done = true;
        return finish_stats(P, locate, use_table, loc_mode, OCC, e0, e1);
    }

    // the end of search(): device statistics (already copied to pinned_stats), timings
    bool last_locate_pp = false;  // finish_deferred took the per-pattern locate (bytes model in finish_stats)
    uint64_t finish_stats(uint64_t P, bool locate, bool use_table, int loc_mode, uint64_t OCC, hipEvent_t e0, hipEvent_t e1) {
        {
            const std::vector<uint64_t> sv = fold_pinned_stats();
#ifdef EDSBWT_DEBUG_CHECKS
            // the debug build's device invariant checks (kernels.hip DBG_CHECK): a failed one is an error
            if (sv[ST_DBG_QUEUE] | sv[ST_DBG_PACKED] | sv[ST_DBG_WIDE] | sv[ST_DBG_LIST])
                throw Fail(EDSBWT_E_DEVICE, "debug checks failed: queue " + std::to_string(sv[ST_DBG_QUEUE]) + ", packed start " +
                                                std::to_string(sv[ST_DBG_PACKED]) + ", wide entry " + std::to_string(sv[ST_DBG_WIDE]) +
                                                ", list " + std::to_string(sv[ST_DBG_LIST]));
#endif
            st.intervals_stepped += sv[ST_DEEP_STEPS] + sv[ST_DEEPQ_STEPS];
            st.link_hash_rows += sv[ST_DEEP_HASH];
            // the 64-B lines the deep kernels gather (occ blocks or the 16-B rank entries' lines; a
            // narrow interval's two ends in one block count once) and the '#'-row reads; + P * 24
            // record bytes above (k_deep_fast).  k_deep_wide's lines are not counted.
            st.bytes_kernel[KC_DEEP] += sv[ST_DEEP_BLOCKS] * 64;
            st.lines_kernel[KC_DEEP] += sv[ST_DEEP_BLOCKS];
            // k_deep: its rank / segment / text lines, one line per '#' row it links from (eofrow, or
            // eof_seg: its segment's table row is then among ST_DEEPQ_BLOCKS), and its queue entries
            // (16 + 8 B streamed per queued pattern)
            st.bytes_kernel[KC_DEEPQ] += (sv[ST_DEEPQ_BLOCKS] + sv[ST_DEEP_HASH]) * 64 + sv[ST_DEEPQ_PATS] * 24;
            st.lines_kernel[KC_DEEPQ] += sv[ST_DEEPQ_BLOCKS] + sv[ST_DEEP_HASH];
            st.bytes_kernel[KC_DEEPW] += sv[ST_DW_BLOCKS] * 64;  // k_deep_wave (k_deep_wide counts none)
            st.lines_kernel[KC_DEEPW] += sv[ST_DW_BLOCKS];
            st.intervals_stepped += sv[ST_DW_STEPS];
            st.lines_kernel[KC_STEP] += sv[ST_STEP_BLOCKS];
            st.bytes_kernel[KC_STEP] += sv[ST_STEP_BLOCKS] * 64;
            st.locate_lf_steps = sv[ST_LOC_STEPS];
            st.text_chars = sv[ST_TEXT_CHARS];
            st.text_rows = sv[ST_TEXT_ROWS];
            st.locate_offsets = sv[ST_LOC_OFFSETS];
            if (trace && sv[ST_DF_WAVE_ROUNDS])
                std::fprintf(stderr, "[edsbwt] k_deep_fast: %llu dependent load rounds over the lanes' patterns, %llu lane slots: lane utilisation %.3f\n",
                             (unsigned long long)sv[ST_DF_LANE_ROUNDS], (unsigned long long)sv[ST_DF_WAVE_ROUNDS],
                             (double)sv[ST_DF_LANE_ROUNDS] / (double)sv[ST_DF_WAVE_ROUNDS]);
            if (trace && (sv[ST_CLK_DD_ONE] | sv[ST_CLK_DD_SROW]))
                std::fprintf(stderr, "[edsbwt] k_deep_direct loads: one-row D-mer entries %llu, per-row text entries %llu, segment rows %llu, "
                                     "whole-word rows %llu, rank-entry lines %llu, interval steps %llu, text rows %llu\n",
                             (unsigned long long)sv[ST_CLK_DD_ONE], (unsigned long long)sv[ST_CLK_DD_SROW], (unsigned long long)sv[ST_CLK_DD_SEG],
                             (unsigned long long)sv[ST_CLK_DD_WROW], (unsigned long long)sv[ST_DEEP_PAIR_LINES],
                             (unsigned long long)sv[ST_DEEP_STEPS], (unsigned long long)sv[ST_TEXT_ROWS]);
            if (trace && sv[ST_CLK_STEPS])
                std::fprintf(stderr, "[edsbwt] k_deep lane-steps %llu (with '#' rows %llu): cycles/step rank+link %.0f, runs %.0f, rest %.0f\n",
                             (unsigned long long)sv[ST_CLK_STEPS], (unsigned long long)sv[ST_CLK_HASH_STEPS],
                             (double)sv[ST_CLK_RANK] / sv[ST_CLK_STEPS], (double)sv[ST_CLK_RUNS] / sv[ST_CLK_STEPS],
                             (double)sv[ST_CLK_REST] / sv[ST_CLK_STEPS]);
            // one line per walk position, plus the sample read
            if (locate && !use_table && !last_locate_pp) st.lines_kernel[KC_LOCATE] += st.locate_lf_steps + OCC + (loc_mode == 2 ? OCC : 0);
            // per-pattern locate (k_locate_pp / k_locate_big): at most one sample line per record
            // (none for a text-compare result), the 20-B record stores, the pattern's result and offset
            if (locate && last_locate_pp) st.lines_kernel[KC_LOCATE] += OCC;
        }
        if (locate && OCC && last_locate_pp) {
            st.bytes_kernel[KC_LOCATE] += OCC * (64 + sizeof(edsbwt_occ)) + P * (sizeof(Res) + 4);
        } else if (locate && OCC) {
            st.bytes_kernel[KC_LOCATE] += st.locate_lf_steps * sizeof(OccBlock) + OCC * (sizeof(OccBlock) + 8 + 8 + 4 + 4 + 4 + sizeof(edsbwt_occ)) +
                                          (loc_mode != 0 ? OCC * 8 : 0);
        }
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, e0, e1));
        st.ms_total = ms;
        if (prof) {
            for (auto& e : evs) {
                float t = 0;
                HIPCHK(hipEventElapsedTime(&t, e.a, e.b));
                st.ms_kernel[e.k] += t;
                ev_pool.push_back(e);
            }
            evs.clear();
        }
        st.occurrences = OCC;
        return OCC;
    }

    // Deferred checks (direct start): counts, and with locate the tasks and records into
    // buffers sized from earlier batches (at least 2 per pattern), then ONE read-back of
    // everything the search postponed.  Returns the record count, or kRedo when a check
    // failed ('#' in a pattern, more overflow patterns than k_deep_wide's launch covered or
    // lists longer than its limit, totals past the buffers).
    static constexpr uint64_t kRedo = ~0ull;
    // the host pipeline's byte-wide counts (k_counts_u8), queued with the search that makes
    // the counts so they are ready when it returns (c8_out.c8 null: none)
    struct C8Out {
        uint8_t* c8 = nullptr;
        uint2* exc = nullptr;
        uint32_t* ne = nullptr;
    } c8_out;
    void emit_c8(uint64_t P, const uint32_t* d_counts) {
        if (!c8_out.c8 || !P) return;
        zero(c8_out.ne, 8);
        hipLaunchKernelGGL(k_counts_u8, dim3((unsigned)std::min<uint64_t>(2048, (P + 1023) / 1024)), dim3(256), 0, stream, d_counts, P,
                           c8_out.c8, c8_out.exc, c8_out.ne);
        HIPCHK(hipGetLastError());
    }
    uint64_t finish_deferred(uint64_t P, uint32_t first_id, bool locate, int loc_mode, uint32_t* d_counts, hipEvent_t e1) {
        const KIdx X = kidx();
        // (counters, the scan's first slot and the check words were zeroed by search())
        // (< 2^32 - 1: a fused occurrence sum saturates there)
        uint64_t occ_cap = std::min<uint64_t>(0xfffffffeull, std::max<uint64_t>({rec.cap, 2 * P + 65536, (uint64_t)(occ_per_pat * 1.25 * (double)P)}));
        uint64_t task_cap = std::min<uint64_t>(0xffffffffull, std::max<uint64_t>({trow.cap, 2 * P + 65536, (uint64_t)(tasks_per_pat * 1.25 * (double)P)}));
        if (defer_cap) occ_cap = task_cap = defer_cap;
        // dense samples: records straight from each pattern's result (k_locate_pp / k_locate_big),
        // no tasks (EDSBWT_LOCATE_TASKS=1: the task path as for every other search)
        const bool per_pattern = locate && loc_mode == 2 && X.samp_dense && locate_pp;
        last_locate_pp = per_pattern;
        if (locate && !per_pattern) occ64.ensure(P);
        // fused counts: written by the deep kernels (count-only) or by k_locate_pp (per-pattern
        // locate, whose offsets scan reads the results), their sums folded by k_gather_checks
        // (EDSBWT_LOCATE_COUNTS=1: the per-pattern locate's counts from k_locate_pp, its scan over the
        // results — C3 1.608 / 1.620 against 1.617 ms with k_count_found, profiles/r04_ab4_c3_*.json: the
        // scan reading 16-B results and the locate kernel's count stores cost what the pass saves)
        const bool loc_counts = per_pattern && fused_counts && locate_counts;
        // per-pattern locate: record offsets per 64-pattern tile (k_count_tiles, a scan over tiles,
        // the offsets inside a tile in k_locate_pp) instead of a scan over every pattern's count
        // (EDSBWT_TILE_SCAN=0: the latter; C3 1.607 / 1.610 against 1.635 ms with 256-pattern
        // tiles, profiles/r04_ab5_c3_*.json)
        const bool tiles = per_pattern && !loc_counts && tile_scan;
        if (tiles_early && !tiles) {
            join_early();
            throw std::logic_error("early record-offset tiles without the tile path");
        }
        const uint64_t ntile = (P + 63) / 64;
        if (tiles) {
            tile_sum.ensure(ntile);
            tile_pre.ensure(ntile);
            if (tiles_early) {  // (summed beside k_deep_wave: join them, add k_deep_wave's patterns)
                if (fc_done || d_counts != early_counts) throw std::logic_error("early record-offset tiles on another path");
                join_early();
                launch_grid(KC_FINISH, k_tile_fix, std::max(1u, std::min(grid_for(early_cap), 64u)), early_ovf, early_cap, (const uint32_t*)perm.p,
                            (const Res*)res.p, d_counts, stats.p, (unsigned long long*)tile_sum.p);
            } else if (fc_done)  // (the deep kernels wrote every count and their sums)
                launch(KC_FINISH, k_tile_sums, P, (const uint32_t*)d_counts, P, (unsigned long long*)tile_sum.p);
            else
                launch(KC_FINISH, k_count_tiles, P, (const Res*)res.p, P, d_counts, stats.p, (unsigned long long*)tile_sum.p, (uint32_t*)nullptr);
        } else if (!fc_done && !loc_counts)
            launch_reduce(KC_FINISH, k_count_found, (const Res*)res.p, P, d_counts, counters.p + 1, counters.p + 12,
                          locate && !per_pattern ? occ64.p : (uint64_t*)nullptr);
        if (!loc_counts) emit_c8(P, d_counts);
        uint32_t* oflow = reinterpret_cast<uint32_t*>(counters.p + 20);
        if (per_pattern) {
            // record offsets: a u32 scan of the counts themselves (a total past 2^32 fails the
            // occ_cap check below); o32[0] = 0 from search()'s zeroing of oscan's first 8 bytes
            oscan.ensure(P + 1);
            uint32_t* o32 = reinterpret_cast<uint32_t*>(oscan.p);
            size_t tb = 0;
            if (tiles) {
                HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, tile_sum.p, tile_pre.p, cub_n(ntile), stream));
                tmp.ensure(tb);
                timed(KC_SCAN, [&] { HIPCHK(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb, tile_sum.p, tile_pre.p, cub_n(ntile), stream)); });
            } else if (loc_counts) {  // the counts straight from the results (k_locate_pp writes them)
                using It = hipcub::TransformInputIterator<uint32_t, ResOcc, const Res*>;
                const It in((const Res*)res.p, ResOcc{});
                HIPCHK(hipcub::DeviceScan::InclusiveSum(nullptr, tb, in, o32 + 1, cub_n(P), stream));
                tmp.ensure(tb);
                timed(KC_SCAN, [&] { HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp.p, tb, in, o32 + 1, cub_n(P), stream)); });
            } else {
                HIPCHK(hipcub::DeviceScan::InclusiveSum(nullptr, tb, d_counts, o32 + 1, cub_n(P), stream));
                tmp.ensure(tb);
                timed(KC_SCAN, [&] { HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp.p, tb, d_counts, o32 + 1, cub_n(P), stream)); });
            }
            hmark("locate scan");
            rec.ensure(occ_cap);
            lbig.ensure(P + 1);  // (its counter zeroed with the others at the search's start)
            // (k_locate_pp's waves are k_count_tiles' tiles: both start every block at a multiple of 256)
            // (EDSBWT_LOC_BLOCKS: a smaller grid, so small tests take the kernel's later block-rounds)
            // (EDSBWT_LOC_PPT: patterns per thread and block-round, 1 or 2)
            const uint64_t lppt = loc_ppt >= 2 ? 2 : 1;
            const unsigned lgrid = grid_for((P + lppt - 1) / lppt);
            launch_grid(KC_LOCATE, loc_stage <= 512 ? (lppt == 2 ? k_locate_pp<512, 2> : k_locate_pp<512>)
                                                    : (lppt == 2 ? k_locate_pp<kLocStage, 2> : k_locate_pp<kLocStage>),
                        loc_blocks ? std::min<unsigned>(lgrid, loc_blocks) : lgrid, P, (const Res*)res.p, o32, first_id, pat_ids, X,
                   (const uint32_t*)ab.p,
                   (const uint32_t*)ae.p, rec.p, occ_cap, lbig.p, oflow, stats.p, loc_counts ? d_counts : (uint32_t*)nullptr,
                   tiles ? (const unsigned long long*)tile_pre.p : (const unsigned long long*)nullptr);
            timed(KC_LOCATE, [&] {
                hipLaunchKernelGGL(k_locate_big, dim3(256), dim3(256), 0, stream, (const uint32_t*)lbig.p, (const Res*)res.p,
                                   (const uint32_t*)o32, first_id, pat_ids, X, (const uint32_t*)ab.p, (const uint32_t*)ae.p, rec.p, stats.p);
            });
            HIPCHK(hipGetLastError());
            task_cap = ~0ull;  // no task buffers in this path
            if (loc_counts) emit_c8(P, d_counts);
        } else if (locate) {
            inclusive_scan_u64(occ64.p, oscan, P, false);  // packed: occurrences << 32 | tasks (totals checked below)
            hmark("locate scan");
            trow.ensure(task_cap); tout.ensure(task_cap); tpat.ensure(task_cap);
            blk_first.ensure(occ_cap / kLocRun + 2);
            rec.ensure(occ_cap);
            launch(KC_LOCPREP, k_tasks, P, P, (const Res*)res.p, (const uint64_t*)nullptr, (const uint64_t*)oscan.p, (const uint32_t*)ab.p,
                   (const uint32_t*)ae.p, trow.p, tout.p, tpat.p, blk_first.p, occ_cap, task_cap, oflow);
            launch(KC_LOCATE, k_locate, occ_cap, occ_cap, task_cap, (const uint64_t*)tout.p, (const uint32_t*)trow.p, (const uint32_t*)tpat.p,
                   (const uint64_t*)blk_first.p, first_id, pat_ids, X, loc_mode, rec.p, stats.p, (const Res*)res.p,
                   (const unsigned long long*)(counters.p + 12), (const uint32_t*)oflow);
        }
        uint32_t* ck = chk();
        hipLaunchKernelGGL(k_gather_checks, dim3(kStatSlots / 256), dim3(256), 0, stream, (const unsigned long long*)counters.p,
                           (const uint32_t*)tflag.p, defer_ovf2, (const unsigned long long*)stats.p, kStatSlots,
                           (uint32_t*)dev_alias(ck), (unsigned long long*)dev_alias(pinned_stats));
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(e1, stream));
        hmark("gather queued");
        HIPCHK(hipStreamSynchronize(stream));
        hmark("synced");
        uint64_t term, found, sums[2];
        std::memcpy(&term, ck + kChkTerm, 8);
        std::memcpy(&found, ck + kChkFound, 8);
        std::memcpy(sums, ck + kChkSums, 16);
        const bool ok = term == 0 && ck[kChkOvf] <= defer_wide_cap && ck[kChkOvf2] == 0 && ck[kChkOflow] == 0 &&
                        (!locate || (sums[0] <= occ_cap && sums[1] <= task_cap && sums[1] < (1ull << 32)));
        if (trace)
            std::fprintf(stderr, "[edsbwt] deferred checks: '#' %llu, overflow %u (wide cap %u), wide overflow %u, buffers %s -> %s\n",
                                    (unsigned long long)term, ck[kChkOvf], defer_wide_cap, ck[kChkOvf2], ck[kChkOflow] ? "short" : "ok", ok ? "ok" : "redo");
        if (!ok) return kRedo;
        const uint32_t nw = ck[kChkOvf];
        st.deep_overflow += nw;
        st.found = found;
        st.not_found = P - found;
        const uint64_t OCC = locate ? sums[0] : 0;
        if (locate) {
            occ_per_pat = std::max(occ_per_pat, (double)sums[0] / (double)P);
            tasks_per_pat = std::max(tasks_per_pat, (double)sums[1] / (double)P);
        }
        return OCC;
    }

    // ------------------------------------------------------------ host pipeline
    static bool host_pinned(const void* p) {
        if (!p) return false;
        hipPointerAttribute_t a{};
        if (hipPointerGetAttributes(&a, p) != hipSuccess) { (void)hipGetLastError(); return false; }
        return a.type == hipMemoryTypeHost;
    }
    // host memcpy on up to 16 threads (staging pageable caller memory)
    static void par_copy(void* dst, const void* src, size_t n) {
        const size_t kPer = 8u << 20;
        const unsigned T = (unsigned)std::min<size_t>(16, std::max<size_t>(1, n / kPer));
        if (T <= 1) { if (n) std::memcpy(dst, src, n); return; }
        std::vector<std::thread> th;
        for (unsigned t = 0; t < T; t++)
            th.emplace_back([=] {
                const size_t a = n * t / T, b = n * (t + 1) / T;
                std::memcpy((char*)dst + a, (const char*)src + a, b - a);
            });
        for (auto& x : th) x.join();
    }
    void pipe_init() {
        if (up) return;
        pool.start((unsigned)std::max(0.0, env_double("EDSBWT_HOST_THREADS", 12) - 1));
        cpool.start((unsigned)std::max(0.0, env_double("EDSBWT_COUNT_THREADS", 4) - 1));
        HIPCHK(hipStreamCreateWithFlags(&up, hipStreamNonBlocking));
        // downloads: hipMemcpyAsync into page-locked host memory runs as a blit kernel that fills
        // every CU with waves waiting on PCIe stores, and the search kernels beside it then wait
        // for CUs (measured: a 4-byte zeroing kernel took 0.56 ms behind a 34 MB download).  The
        // download stream is therefore confined to a few CUs spread over the XCDs
        // (EDSBWT_DOWN_CUS, 0: no mask)
        {
            hipDeviceProp_t prop{};
            HIPCHK(hipGetDeviceProperties(&prop, device));
            const int ncu = prop.multiProcessorCount;
            const int want = (int)env_double("EDSBWT_DOWN_CUS", 32);
            if (want > 0 && want < ncu) {
                std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
                const bool spread = env_double("EDSBWT_DOWN_CU_SPREAD", 1) != 0;
                const int stride = std::max(1, ncu / want);
                int got = 0;
                for (int i = 0; i < ncu && got < want; i++)
                    if (!spread || i % stride == 0) { mask[i / 32] |= 1u << (i % 32); got++; }
                HIPCHK(hipExtStreamCreateWithCUMask(&down, (uint32_t)mask.size(), mask.data()));
            } else {
                HIPCHK(hipStreamCreateWithFlags(&down, hipStreamNonBlocking));
            }
        }
        for (int k = 0; k < kSlots; k++) {
            HIPCHK(hipEventCreateWithFlags(&up_done[k], hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&comp_done[k], hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&down_done[k], hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&prep_done[k], hipEventDisableTiming));
        }
    }
    // host -> device on `up` (staged through page-locked memory when src is pageable)
    void upload(void* dst, const void* src, size_t n, bool pinned_src, Pinned& stage, int slot) {
        if (!n) return;
        if (pinned_src) {
            HIPCHK(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, up));
            return;
        }
        HIPCHK(hipEventSynchronize(up_done[slot]));  // the slot's previous upload has left the staging buffer
        stage.ensure(n);
        par_copy(stage.p, src, n);
        HIPCHK(hipMemcpyAsync(dst, stage.p, n, hipMemcpyHostToDevice, up));
    }
    void arena_ensure(size_t n) {  // keep the records received so far (down stream synced)
        if (n <= arena_cap && arena) return;
        HIPCHK(hipStreamSynchronize(down));
        std::lock_guard<std::mutex> g(arena_mx);
        const size_t c = std::max<size_t>({n, arena_cap + arena_cap / 2, (size_t)1 << 16});
        edsbwt_occ* q = nullptr;
        if (hipHostMalloc((void**)&q, c * sizeof(edsbwt_occ), hipHostMallocDefault) != hipSuccess)
            throw Fail(EDSBWT_E_NOMEM, "hipHostMalloc of the occurrence records failed");
        if (arena) {
            pool.parallel_copy(q, arena, arena_cap * sizeof(edsbwt_occ));
            arena_release();
        }
        arena = q;
        arena_cap = c;
        arena_dev = nullptr;
        void* d = nullptr;
        if (hipHostGetDevicePointer(&d, arena, 0) == hipSuccess) arena_dev = static_cast<edsbwt_occ*>(d);
        else (void)hipGetLastError();
        arena_register();
    }
    // compact downloads: per record only (word, offset) crosses PCIe; the host rebuilds
    // (pat, word, segment, word in segment, offset) from the counts and the segment tables
    std::vector<uint32_t> h_seg_of_word, h_seg_start;
    DBuf<uint2> hrec8[kSlots];
    uint2* arena8 = nullptr;  // page-locked landing area of the compact records
    size_t arena8_cap = 0;
    std::mutex arena_mx;      // arena / arena8 growth vs the expander thread
    void arena8_ensure(size_t n) {
        if (n <= arena8_cap && arena8) return;
        HIPCHK(hipStreamSynchronize(down));
        const size_t c = std::max<size_t>({n, arena8_cap + arena8_cap / 2, (size_t)1 << 16});
        uint2* q = nullptr;
        if (hipHostMalloc((void**)&q, c * sizeof(uint2), hipHostMallocDefault) != hipSuccess)
            throw Fail(EDSBWT_E_NOMEM, "hipHostMalloc of the compact records failed");
        std::lock_guard<std::mutex> g(arena_mx);
        if (arena8) {
            pool.parallel_copy(q, arena8, arena8_cap * sizeof(uint2));
            (void)hipHostFree(arena8);
        }
        arena8 = q;
        arena8_cap = c;
    }
    // a few persistent host threads (EDSBWT_HOST_THREADS, default 12: bench.py on C3 5.74 ms against 6.0 with 16 — more threads than the 16-CPU share throttles; an in-process A/B had favoured 16) for staging copies and
    // record expansion, so the pipeline never pays thread start-up per chunk
    struct Pool {
        std::vector<std::thread> th;
        std::mutex m;
        std::condition_variable cv, done_cv;
        std::function<void(unsigned)> fn;
        unsigned todo = 0, next = 0, running = 0;
        uint64_t gen = 0;
        bool stop = false;
        std::mutex run_mx;  // one run at a time (the upload thread packs while this thread may grow the arena)
        unsigned size() const { return (unsigned)th.size() + 1; }
        void start(unsigned n) {
            for (unsigned i = 0; i < n; i++)
                th.emplace_back([this] {
                    uint64_t seen = 0;
                    for (;;) {
                        std::unique_lock<std::mutex> lk(m);
                        cv.wait(lk, [&] { return stop || (gen != seen && next < todo); });
                        if (stop) return;
                        seen = gen;
                        while (next < todo) {
                            const unsigned t = next++;
                            running++;
                            lk.unlock();
                            fn(t);
                            lk.lock();
                            running--;
                        }
                        done_cv.notify_all();
                    }
                });
        }
        // fn(t) for t < n on the pool and the calling thread; returns when all are done
        void run(unsigned n, const std::function<void(unsigned)>& f) {
            if (n <= 1 || th.empty()) { for (unsigned t = 0; t < n; t++) f(t); return; }
            std::lock_guard<std::mutex> one(run_mx);
            std::unique_lock<std::mutex> lk(m);
            fn = f;
            todo = n;
            next = 0;
            gen++;
            cv.notify_all();
            while (next < todo) {
                const unsigned t = next++;
                running++;
                lk.unlock();
                fn(t);
                lk.lock();
                running--;
            }
            done_cv.wait(lk, [&] { return running == 0; });
            todo = 0;
        }
        void parallel_copy(void* dst, const void* src, size_t n) {
            const size_t kPer = 4u << 20;
            const unsigned T = (unsigned)std::min<size_t>(size(), std::max<size_t>(1, n / kPer));
            run(T, [&](unsigned t) {
                const size_t a = n * t / T, b = n * (t + 1) / T;
                std::memcpy((char*)dst + a, (const char*)src + a, b - a);
            });
        }
        ~Pool() {
            {
                std::lock_guard<std::mutex> g(m);
                stop = true;
            }
            cv.notify_all();
            for (auto& x : th) x.join();
        }
    } pool, cpool;  // cpool: the counts thread's (expand_c8)
    // the host pipeline's upload, download and counts threads, kept for the engine's life: a call
    // hands each its closure and waits for it (C2's one-chunk call: no thread creation on its
    // critical path)
    struct Worker {
        std::thread th;
        std::mutex m;
        std::condition_variable cv;
        std::function<void()> job;
        bool busy = false, stop = false;
        void run(std::function<void()> f) {
            if (!th.joinable())
                th = std::thread([this] {
                    for (;;) {
                        std::function<void()> g;
                        {
                            std::unique_lock<std::mutex> lk(m);
                            cv.wait(lk, [&] { return stop || (busy && job); });
                            if (stop) return;
                            g = std::move(job);
                            job = nullptr;
                        }
                        g();
                        {
                            std::lock_guard<std::mutex> lk(m);
                            busy = false;
                        }
                        cv.notify_all();
                    }
                });
            {
                std::lock_guard<std::mutex> lk(m);
                job = std::move(f);
                busy = true;
            }
            cv.notify_all();
        }
        void wait() {
            std::unique_lock<std::mutex> lk(m);
            cv.wait(lk, [&] { return !busy; });
        }
        ~Worker() {
            {
                std::lock_guard<std::mutex> lk(m);
                stop = true;
            }
            cv.notify_all();
            if (th.joinable()) th.join();
        }
    } w_up, w_down, w_cnt;
    // With records the counts cross PCIe as one byte each (k_counts_u8: most are small), the
    // few of 255 and more as (pattern, count) pairs, and a host thread widens them into the
    // caller's counts while the next chunk downloads: a quarter of the counts' PCIe bytes.
    // EDSBWT_SMALL_COUNTS=0: 4 bytes each.
    // Only beside records: a count-only call's counts go straight to the caller's page-locked array
    // as u32 (C2: 4 MB in ~0.07 ms, against 1 MB of bytes plus their widening on the host, ~0.1 ms
    // and a thread wake-up on the critical path).  EDSBWT_SMALL_COUNTS=0: never, 2: count-only too.
    int small_counts = (int)env_double("EDSBWT_SMALL_COUNTS", 1);
    static uint64_t c8_bytes(uint64_t P) { return (P + 7) / 8 * 8 + 8; }  // bytes, then the exception count (u32)
    void expand_c8(uint32_t* c, const uint8_t* c8, uint64_t P, const uint2* exc, uint32_t nexc) {
        const unsigned T = (unsigned)std::min<uint64_t>(cpool.size(), std::max<uint64_t>(1, P / 262144));
        cpool.run(T, [&](unsigned t) {
            for (uint64_t p = P * t / T, e = P * (t + 1) / T; p < e; p++) c[p] = c8[p];
        });
        for (uint32_t i = 0; i < nexc; i++) {
            if (exc[i].x >= P) throw Fail(EDSBWT_E_DEVICE, "counts: an exception outside the chunk");
            c[exc[i].x] = exc[i].y;
        }
    }
    // expand one chunk's compact records: pattern ids from the counts, segment and word in
    // segment from the segment tables (MOVE_EDSBWTSearch.cpp:361-363's rank1/select1)
    void expand_chunk(const uint32_t* counts, uint64_t p0, uint64_t P, uint64_t r0, uint64_t n, uint32_t first_id) {
        std::lock_guard<std::mutex> g(arena_mx);
        const unsigned T = (unsigned)std::min<uint64_t>(pool.size(), std::max<uint64_t>(1, n / 32768));
        std::vector<uint64_t> start(T + 1, 0);
        pool.run(T, [&](unsigned t) {
            uint64_t sum = 0;
            for (uint64_t p = P * t / T; p < P * (t + 1) / T; p++) sum += counts[p0 + p];
            start[t + 1] = sum;
        });
        for (unsigned t = 0; t < T; t++) start[t + 1] += start[t];
        if (start[T] != n) throw Fail(EDSBWT_E_DEVICE, "record expansion: counts do not add up to the records");
        const uint32_t* sow = h_seg_of_word.data();
        const uint32_t* sst = h_seg_start.data();
        pool.run(T, [&](unsigned t) {
            uint64_t r = r0 + start[t];
            for (uint64_t p = P * t / T; p < P * (t + 1) / T; p++) {
                const uint32_t c = counts[p0 + p], pid = first_id + (uint32_t)(p0 + p);
                for (uint32_t q = 0; q < c; q++, r++) {
                    const uint2 v = arena8[r];
                    const uint32_t sg = sow[v.x];
                    arena[r] = edsbwt_occ{pid, v.x, sg, v.x - sst[sg], v.y};
                }
            }
        });
    }
    edsbwt_occ* arena_dev = nullptr;  // the arena as the device sees it (kernel-written downloads)
    // blocks of the download kernel: few, so its PCIe stores do not crowd out the search's memory traffic
    size_t d2h_blocks = (size_t)std::max(1.0, env_double("EDSBWT_D2H_BLOCKS", 32));
    // device view of page-locked caller memory (nullptr: not mapped)
    static void* host_dev_ptr(void* p) {
        void* d = nullptr;
        if (!p || hipHostGetDevicePointer(&d, p, 0) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
        return d;
    }
    // device -> mapped host memory by a kernel on `down`: the copy engines take the uploads, so the
    // downloads go over PCIe as kernel stores and both directions stream at once
    void download(void* dst_dev, const void* src, size_t bytes) {
        if (!bytes) return;
        const size_t n4 = bytes / 4;
        const unsigned blocks = (unsigned)std::min<size_t>(d2h_blocks, (n4 + 255) / 256);
        hipLaunchKernelGGL(k_copy_out, dim3(blocks), dim3(256), 0, down, (const uint32_t*)src, (uint32_t*)dst_dev, (uint64_t)n4);
        HIPCHK(hipGetLastError());
    }
    void arena_register();
    void arena_release();
    void arena_checkout();
    void arena_checkin();
    bool arena_checked_out();

    struct Chunk { uint64_t b0, b1, p0, p1, dpos; };  // byte range; pattern range (offsets mode); device place (eager)
    // chunk prep on `up` (after its upload into slot sl): lines mode splits the raw bytes into
    // (bytes, offsets) — k_nl_count, a scan, k_nl_compact — and k_line_fin writes the pattern
    // count, the unterminated last line's end and the longest / shortest line; offsets mode
    // rebases the offsets and measures the lengths.  Results land in prep_host(sl).
    void prep(const Chunk& c, int sl, bool lines, const uint8_t* text) {
        prep_mm[sl].ensure(4);
        zero_on(prep_mm[sl].p, 32, up);
        if (lines) {
            const uint64_t nb = c.b1 - c.b0;
            const uint64_t nblk = std::max<uint64_t>(1, (nb + kLineBlk - 1) / kLineBlk);
            const uint32_t tail = (nb && text[c.b1 - 1] != '\n') ? 1u : 0u;
            nlcnt_s[sl].ensure(nblk + 1);
            nlpre_s[sl].ensure(nblk + 1);
            hbytes[sl].ensure(nb + 16);
            hoffs[sl].ensure(nb + 2);  // at most one line per byte, plus the unterminated last line
            zero_on(nlpre_s[sl].p, 4, up);
            zero_on(hoffs[sl].p, 8, up);
            if (nb) {
                hipLaunchKernelGGL(k_nl_count, dim3((unsigned)nblk), dim3(256), 0, up, (const uint8_t*)hraw[sl].p, nb, nlcnt_s[sl].p);
                HIPCHK(hipGetLastError());
                size_t tb = 0;
                HIPCHK(hipcub::DeviceScan::InclusiveSum(nullptr, tb, nlcnt_s[sl].p, nlpre_s[sl].p + 1, cub_n(nblk), up));
                ptmp[sl].ensure(tb);
                HIPCHK(hipcub::DeviceScan::InclusiveSum(ptmp[sl].p, tb, nlcnt_s[sl].p, nlpre_s[sl].p + 1, cub_n(nblk), up));
                hipLaunchKernelGGL(k_nl_compact, dim3((unsigned)nblk), dim3(256), 0, up, (const uint8_t*)hraw[sl].p, nb,
                                   (const uint32_t*)nlpre_s[sl].p, hbytes[sl].p, hoffs[sl].p);
                HIPCHK(hipGetLastError());
                hipLaunchKernelGGL(k_line_fin, dim3(kReduceBlocks), dim3(256), 0, up, hoffs[sl].p, (const uint32_t*)(nlpre_s[sl].p + nblk), tail,
                                   nb, prep_mm[sl].p);
                HIPCHK(hipGetLastError());
            }
        } else {
            const uint64_t P = c.p1 - c.p0;
            if (c.b0) {
                hipLaunchKernelGGL(k_rebase, dim3(grid_for(P + 1)), dim3(256), 0, up, hoffs[sl].p, P + 1, c.b0);
                HIPCHK(hipGetLastError());
            }
            if (P) {  // (offsets mode knows P: prep_host's count slot stays 0)
                hipLaunchKernelGGL(k_lminmax, dim3(kReduceBlocks), dim3(256), 0, up, (const uint64_t*)hoffs[sl].p, P, prep_mm[sl].p + 1);
                HIPCHK(hipGetLastError());
            }
        }
        small_copy_on(prep_host(sl), prep_mm[sl].p, 24, up);
    }
    // a chunk of fixed-length A/C/G/T lines packed to 2 bits per base on the host (format.cpp),
    // into stage_pack[sl]: returns its lines (0: the chunk is not of that form; send the bytes).
    // EDSBWT_PACK_LINES=0 turns it off.
    bool pack_lines = env_double("EDSBWT_PACK_LINES", 1) != 0;
    bool pack_single = env_double("EDSBWT_PACK_SINGLE", 1) != 0;
    // one-chunk batches packed in sub-blocks, each uploaded when ready (pack_chunk_streamed): off by
    // default — C2's 5 MB upload is shorter than the packing, 0.661 against 0.639 ms median call with
    // the whole chunk packed first (profiles/r05_ab_c2_counts_pack_*.json); EDSBWT_PACK_STREAMED=1
    bool pack_streamed = env_double("EDSBWT_PACK_STREAMED", 0) != 0;
    uint64_t pack_threads = 64;  // per call: EDSBWT_PACK_THREADS (at most the pool's)
    uint64_t pack_chunk(const uint8_t* s, uint64_t nb, const uint8_t* end, int sl, uint32_t* L_out) {
        if (!pack_lines) return 0;
        uint32_t L = 0;
        const uint64_t P = edsbwt_lines_fixed(s, nb, &L);
        if (!P) return 0;
        const uint64_t S = (L + 3) / 4;
        stage_pack[sl].ensure(P * S + 16);
        uint8_t* out = static_cast<uint8_t*>(stage_pack[sl].p);
        const unsigned T = (unsigned)std::min<uint64_t>(std::min<uint64_t>(pool.size(), pack_threads), std::max<uint64_t>(1, P / 16384));
        std::atomic<int> bad{0};
        pool.run(T, [&](unsigned t) {
            if (!edsbwt_pack_lines(s, nb, L, P * t / T, P * (t + 1) / T, end, out)) bad.store(1, std::memory_order_relaxed);
        });
        if (bad.load()) return 0;
        *L_out = L;
        return P;
    }
    // pack_chunk for a one-chunk batch, in kPackSub line blocks each sent on the up engine as soon as
    // it is packed (C2: the 5 MB of packed lines cross PCIe while the later blocks are packed, instead
    // of after the whole chunk).  Returns P (0: not fixed-length A/C/G/T lines — every copy started
    // has finished; the caller sends the chunk raw); the copies are complete when it returns.
    static constexpr int kPackSub = 4;
    uint64_t pack_chunk_streamed(const uint8_t* s, uint64_t nb, const uint8_t* end, int sl, uint32_t* L_out, hsa_signal_t* sigs) {
        if (!pack_lines) return 0;
        uint32_t L = 0;
        const uint64_t P = edsbwt_lines_fixed(s, nb, &L);
        if (!P) return 0;
        const uint64_t S = (L + 3) / 4;
        stage_pack[sl].ensure(P * S + 16);
        hpack[sl].ensure(P * S + 16);
        uint8_t* out = static_cast<uint8_t*>(stage_pack[sl].p);
        int started = 0;
        bool ok = true;
        for (int j = 0; j < kPackSub && ok; j++) {
            const uint64_t p0 = P * j / kPackSub, p1 = P * (j + 1) / kPackSub;
            if (p1 == p0) continue;
            const uint64_t n = p1 - p0;
            const unsigned T = (unsigned)std::min<uint64_t>(std::min<uint64_t>(pool.size(), pack_threads), std::max<uint64_t>(1, n / 16384));
            std::atomic<int> bad{0};
            pool.run(T, [&](unsigned t) {
                if (!edsbwt_pack_lines(s, nb, L, p0 + n * t / T, p0 + n * (t + 1) / T, end, out)) bad.store(1, std::memory_order_relaxed);
            });
            if (bad.load()) { ok = false; break; }
            hsa_copy_start(hpack[sl].p + p0 * S, out + p0 * S, n * S, false, eng_up, sigs[started++]);
        }
        for (int j = 0; j < started; j++) hsa_wait(sigs[j]);
        if (!ok) return 0;
        *L_out = L;
        return P;
    }
    // prep of a packed chunk on `up`: its bytes and offsets back (k_unpack_lines), P and the
    // line length into prep_host(sl) as prep() leaves them
    void prep_packed(int sl, uint64_t nb, uint64_t P, uint32_t L) {
        prep_mm[sl].ensure(4);
        hbytes[sl].ensure(nb + 16);
        hoffs[sl].ensure(P + 2);
        const uint64_t n16 = (P * L + 15) / 16;
        hipLaunchKernelGGL(k_unpack_lines, dim3((unsigned)std::min<uint64_t>(std::max<uint64_t>(1, (n16 + 255) / 256), 4096)), dim3(256), 0, up,
                           (const uint8_t*)hpack[sl].p, P, L, (uint32_t)((L + 3) / 4), hbytes[sl].p, hoffs[sl].p, prep_mm[sl].p);
        HIPCHK(hipGetLastError());
        small_copy_on(prep_host(sl), prep_mm[sl].p, 24, up);
    }
    DBuf<uint8_t> hin_all;                // eager uploads: every chunk of the batch
    DBuf<uint64_t> hoff_all;
    std::vector<hipEvent_t> chunk_ev;     // ... and their completion
    std::vector<hipEvent_t> chunk_down_ev;  // each chunk's downloads (compact records: the expander waits on them)

    // chunks of about EDSBWT_CHUNK_MB of pattern bytes (default 40 MB: tools/ab_calls.py on C3, 40 against 32-64), cut at line ends; the
    // first and last chunks ramp up from / down to 1/8 of that (EDSBWT_CHUNK_RAMP=0: uniform),
    // so the pipeline fills and drains fast
    std::vector<Chunk> cut_chunks(const uint8_t* text, uint64_t len, const uint64_t* offs, uint64_t npat, bool lines) {
        const uint64_t target = std::max<uint64_t>(1, (uint64_t)(env_double("EDSBWT_CHUNK_MB", 40) * 1048576.0));
        std::vector<uint64_t> sizes;
        // a batch of at most EDSBWT_CHUNK_SINGLE_MB (default 24) is one chunk: every chunk pays
        // a search's fixed cost, which small batches (C2's 21 MB, C5's 7 MB of grouped search)
        // do not win back by overlapping their transfers
        const uint64_t single = (uint64_t)(env_double("EDSBWT_CHUNK_SINGLE_MB", 24) * 1048576.0);
        if (len <= single) {
            sizes = {len};
        } else {
            const bool ramp = env_double("EDSBWT_CHUNK_RAMP", 1) != 0;
            // ramp chunks target/2^R .. target/2 (R = EDSBWT_RAMP_STEPS, default 3): the first
            // chunk's search ends early, so the downloads (the call's bound) start early
            const int R = (int)std::max(1.0, std::min(8.0, env_double("EDSBWT_RAMP_STEPS", 3)));
            std::vector<uint64_t> steps;
            for (int i = R; i >= 1; i--) steps.push_back(std::max<uint64_t>(1, target >> i));
            uint64_t rsum = 0;
            for (uint64_t x : steps) rsum += x;
            if (ramp && len > 2 * rsum) {
                // ramp up, uniform middle chunks of at most `target`, ramp down: the last
                // chunk's search and download (the drain) stay short
                const uint64_t mid = len - 2 * rsum, nm = (mid + target - 1) / target;
                sizes = steps;
                for (uint64_t q = 0; q < nm; q++) sizes.push_back(mid * (q + 1) / nm - mid * q / nm);
                sizes.insert(sizes.end(), steps.rbegin(), steps.rend());
            } else {
                std::vector<uint64_t> front, back;
                uint64_t covered = 0;
                for (int i = 0; covered < len; i++) {
                    const uint64_t a = std::max<uint64_t>(1, ramp && i < (int)steps.size() ? steps[i] : target);
                    front.push_back(a);
                    covered += a;
                    if (covered >= len) break;
                    back.push_back(a);
                    covered += a;
                }
                sizes = front;
                sizes.insert(sizes.end(), back.rbegin(), back.rend());
            }
        }
        std::vector<Chunk> ch;
        if (lines) {
            uint64_t b = 0;
            for (size_t q = 0; b < len; q++) {
                uint64_t e = q + 1 < sizes.size() ? std::min(len, b + sizes[q]) : len;
                if (e < len) {
                    const void* nl = std::memchr(text + e - 1, '\n', len - (e - 1));
                    e = nl ? (uint64_t)((const uint8_t*)nl - text) + 1 : len;
                }
                ch.push_back({b, e, 0, 0, 0});
                b = e;
            }
        } else {
            if (npat && offs[0] != 0) throw Fail(EDSBWT_E_ARG, "pat_offsets[0] must be 0");
            uint64_t p = 0;
            for (size_t q = 0; p < npat; q++) {
                // the chunk's last pattern: the first whose end passes the target
                uint64_t lo = p + 1, hi = npat;
                const uint64_t want = q + 1 < sizes.size() ? offs[p] + sizes[q] : offs[npat];
                while (lo < hi) { const uint64_t m = (lo + hi) / 2; if (offs[m] < want) lo = m + 1; else hi = m; }
                ch.push_back({offs[p], offs[lo], p, lo, 0});
                p = lo;
            }
        }
        return ch;
    }

    // ---- bulk transfers on explicit SDMA engines: uploads on one, downloads on another, each
    // driven by its own host thread.  Through hipMemcpyAsync the runtime gave both directions
    // the same engine here, which then served them in turn (tools/hsa_duplex.hip on MI355X:
    // 56 GB/s on one engine, 95 GB/s on two).  EDSBWT_HSA_COPY=0: the HIP-stream pipeline.
    bool hsa_tried = false, hsa_ok = false;
    hsa_agent_t hsa_gpu{}, hsa_cpu{};
    uint32_t eng_up = 0, eng_down = 0;
    bool hsa_init() {
        if (hsa_tried) return hsa_ok;
        hsa_tried = true;
        if (env_double("EDSBWT_HSA_COPY", 1) == 0) return false;
        struct Ctx {
            int bus = -1, dev = -1, dom = -1;
            hsa_agent_t gpu{}, cpu{};
            bool g = false, c = false;
        } cx;
        if (hipDeviceGetAttribute(&cx.bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
            hipDeviceGetAttribute(&cx.dev, hipDeviceAttributePciDeviceId, device) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (hipDeviceGetAttribute(&cx.dom, hipDeviceAttributePciDomainId, device) != hipSuccess) { (void)hipGetLastError(); cx.dom = -1; }
        auto cb = [](hsa_agent_t a, void* d) -> hsa_status_t {
            Ctx* c = static_cast<Ctx*>(d);
            hsa_device_type_t t;
            if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
            if (t == HSA_DEVICE_TYPE_CPU && !c->c) { c->cpu = a; c->c = true; }
            if (t == HSA_DEVICE_TYPE_GPU && !c->g) {
                uint32_t bdf = 0, domain = 0;
                if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
                (void)hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &domain);
                if ((int)((bdf >> 8) & 0xff) == c->bus && (int)((bdf >> 3) & 0x1f) == c->dev && (c->dom < 0 || (int)domain == c->dom)) {
                    c->gpu = a;
                    c->g = true;
                }
            }
            return HSA_STATUS_SUCCESS;
        };
        if (hsa_iterate_agents(cb, &cx) != HSA_STATUS_SUCCESS || !cx.g || !cx.c) return false;
        uint32_t m_up = 0, m_down = 0;
        if (hsa_amd_memory_copy_engine_status(cx.gpu, cx.cpu, &m_up) != HSA_STATUS_SUCCESS ||
            hsa_amd_memory_copy_engine_status(cx.cpu, cx.gpu, &m_down) != HSA_STATUS_SUCCESS)
            return false;
        // engines 2 and 3: measured fastest for this pair on MI355X (0 and 1 also carry the runtime's own
        // copies; 4 and up reach the host at a fraction of the rate: tools/gpu_ab.sh sweeps)
        const uint32_t want_up = (uint32_t)env_double("EDSBWT_SDMA_UP", 0x4), want_down = (uint32_t)env_double("EDSBWT_SDMA_DOWN", 0x8);
        auto pick = [](uint32_t avail, uint32_t want, uint32_t avoid) -> uint32_t {
            if (want && (avail & want) && want != avoid && !(want & (want - 1))) return want;
            for (uint32_t b = 1; b && b <= 0x8000u; b <<= 1)
                if ((avail & b) && b != avoid) return b;
            return 0;
        };
        eng_up = pick(m_up, want_up, 0);
        eng_down = pick(m_down, want_down, eng_up);
        if (!eng_up || !eng_down) return false;
        hsa_gpu = cx.gpu;
        hsa_cpu = cx.cpu;
        hsa_ok = true;
        if (trace) std::fprintf(stderr, "[edsbwt] host pipeline: SDMA engine 0x%x up, 0x%x down\n", eng_up, eng_down);
        return true;
    }
    // n bytes on engine `eng`, waiting for the copy (the caller is that direction's thread)
    void hsa_copy(void* dst, const void* src, size_t n, bool to_host, uint32_t eng, hsa_signal_t sig) {
        if (!n) return;
        hsa_copy_start(dst, src, n, to_host, eng, sig);
        hsa_wait(sig);
    }
    void hsa_wait(hsa_signal_t sig) {
        while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE) >= 1) {}
    }
    void hsa_copy_start(void* dst, const void* src, size_t n, bool to_host, uint32_t eng, hsa_signal_t sig) {
        hsa_signal_store_relaxed(sig, 1);
        const hsa_status_t r = hsa_amd_memory_async_copy_on_engine(dst, to_host ? hsa_cpu : hsa_gpu, src, to_host ? hsa_gpu : hsa_cpu, n, 0, nullptr,
                                                                   sig, (hsa_amd_sdma_engine_id_t)eng, true);
        if (r != HSA_STATUS_SUCCESS) {
            const char* m = nullptr;
            hsa_status_string(r, &m);
            throw Fail(EDSBWT_E_DEVICE, std::string("hsa_amd_memory_async_copy_on_engine: ") + (m ? m : "?"));
        }
    }

    // search_host over explicit SDMA engines: an upload thread (chunk k+ahead: copy, then its prep
    // on `up`), this thread (chunk k's search on `stream`), a download thread (chunk k-1's counts
    // and records).  Chunk k reuses slot k % kSlots: its upload waits for chunk k-kSlots's search,
    // its search for chunk k-kSlots's download.
    uint64_t search_host_hsa(const std::vector<Chunk>& ch, const uint8_t* text, const uint64_t* offs, bool lines, bool pin_in, bool pin_off,
                             bool pin_cnt, uint32_t first_id, uint32_t flags, uint32_t* counts, uint64_t counts_cap, bool locate,
                             edsbwt_occ** occ_out, uint64_t* npat_out, std::chrono::steady_clock::time_point t0) {
        const size_t nch = ch.size();
        const size_t ahead = (size_t)std::max(1.0, std::min<double>(kSlots - 2, env_double("EDSBWT_AHEAD", 3)));
        std::mutex m;
        std::condition_variable cv;
        size_t uploaded = 0, searched = 0, downloaded = 0;
        bool stop = false, closed = false;
        std::exception_ptr err;
        struct Job {
            size_t k;
            uint64_t P, n, pats, total;
            uint32_t nexc;  // small counts: the chunk's counts of 255 and more
        };
        std::deque<Job> jobs;
        uint64_t h2d = 0, d2h = 0, packed = 0;
        // small counts (expand_c8): widened on a thread of their own, chunk by chunk as they
        // land, so the downloads never wait for it
        const bool derive_counts = small_counts == 2 || (small_counts == 1 && locate);
        size_t counted = 0;
        std::vector<Job> landed;
        const uint8_t* text_end = text + (nch ? ch.back().b1 : 0);
        const bool prepack = env_double("EDSBWT_PREPACK", 1) != 0;
        pack_threads = (uint64_t)std::max(1.0, env_double("EDSBWT_PACK_THREADS", 64));
        std::vector<std::tuple<const char*, size_t, double>> marks;
        std::mutex mark_m;
        auto mark = [&](const char* what, size_t k) {
            if (!trace) return;
            std::lock_guard<std::mutex> g(mark_m);
            marks.emplace_back(what, k, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        };
        auto fail = [&](std::exception_ptr e) {
            std::lock_guard<std::mutex> g(m);
            if (!err) err = e;
            stop = true;
            cv.notify_all();
        };
        if (arena_checked_out()) arena_release();  // the caller still holds the last records: start a new buffer
        w_up.run([&] {
            hsa_signal_t sig{};
            hsa_signal_t ssig[kPackSub] = {};  // the streamed packing's block copies
            bool have_sig = false, have_ssig = false;
            try {
                HIPCHK(hipSetDevice(device));
                if (hsa_signal_create(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) throw Fail(EDSBWT_E_DEVICE, "hsa_signal_create failed");
                have_sig = true;
                if (nch == 1 && lines && pack_streamed) {
                    int made = 0;
                    while (made < kPackSub && hsa_signal_create(1, 0, nullptr, &ssig[made]) == HSA_STATUS_SUCCESS) made++;
                    have_ssig = made == kPackSub;
                    if (!have_ssig)
                        for (int j = 0; j < made; j++) hsa_signal_destroy(ssig[j]);
                }
                size_t pre_k = ~size_t(0);  // the chunk packed ahead (pre_P lines of pre_L bases; 0: raw)
                uint64_t pre_P = 0;
                uint32_t pre_L = 0;
                for (size_t k = 0; k < nch; k++) {
                    {
                        std::unique_lock<std::mutex> lk(m);
                        cv.wait(lk, [&] { return stop || (k <= searched + ahead && k < searched + kSlots); });
                        if (stop) break;
                    }
                    const Chunk& c = ch[k];
                    const int sl = (int)(k % kSlots);
                    const uint64_t nb = c.b1 - c.b0;
                    mark("upload", k);
                    uint32_t L = 0;
                    uint64_t Pk = 0;
                    // a one-chunk batch's packing has nothing to overlap with: EDSBWT_PACK_SINGLE=0 sends
                    // it raw (C2: 21 MB raw at ~56 GB/s against packing on the host first)
                    if (lines && nch == 1 && pack_single && pack_streamed && have_ssig) {
                        // one chunk: its packed line blocks cross PCIe as they are packed
                        Pk = pack_chunk_streamed(text + c.b0, nb, text_end, sl, &L, ssig);
                        if (Pk) {
                            prep_packed(sl, nb, Pk, L);
                            HIPCHK(hipEventRecord(prep_done[sl], up));
                            mark("uploaded", k);
                            {
                                std::lock_guard<std::mutex> g(m);
                                uploaded = k + 1;
                                h2d += Pk * ((L + 3) / 4);
                                packed++;
                            }
                            cv.notify_all();
                            continue;
                        }
                    } else if (lines && (nch > 1 || pack_single))
                        Pk = pre_k == k ? (L = pre_L, pre_P) : pack_chunk(text + c.b0, nb, text_end, sl, &L);
                    pre_k = ~size_t(0);
                    if (Pk) {  // 2 bits per base over PCIe, unpacked on the device
                        const uint64_t pb = Pk * ((L + 3) / 4);
                        hpack[sl].ensure(pb + 16);
                        hsa_copy_start(hpack[sl].p, stage_pack[sl].p, pb, false, eng_up, sig);
                        if (k + 1 < nch && prepack) {
                            // the next chunk packed while this one crosses PCIe (its staging buffer's
                            // last upload has finished)
                            const Chunk& c2 = ch[k + 1];
                            pre_P = pack_chunk(text + c2.b0, c2.b1 - c2.b0, text_end, (int)((k + 1) % kSlots), &pre_L);
                            pre_k = k + 1;
                        }
                        hsa_wait(sig);
                        prep_packed(sl, nb, Pk, L);
                        HIPCHK(hipEventRecord(prep_done[sl], up));
                        mark("uploaded", k);
                        {
                            std::lock_guard<std::mutex> g(m);
                            uploaded = k + 1;
                            h2d += pb;
                            packed++;
                        }
                        cv.notify_all();
                        continue;
                    }
                    uint64_t up_bytes = nb;
                    uint8_t* dst = nullptr;
                    if (lines) {
                        hraw[sl].ensure(nb + 16);
                        dst = hraw[sl].p;
                    } else {
                        hbytes[sl].ensure(nb + 16);
                        hoffs[sl].ensure(c.p1 - c.p0 + 1);
                        dst = hbytes[sl].p;
                    }
                    const uint8_t* src = text + c.b0;
                    if (!pin_in && nb) {
                        stage_in[sl].ensure(nb);
                        par_copy(stage_in[sl].p, src, nb);
                        src = static_cast<const uint8_t*>(stage_in[sl].p);
                    }
                    hsa_copy(dst, src, nb, false, eng_up, sig);
                    if (!lines) {
                        const size_t ob = (c.p1 - c.p0 + 1) * 8;
                        const void* osrc = offs + c.p0;
                        if (!pin_off) {
                            stage_off[sl].ensure(ob);
                            par_copy(stage_off[sl].p, osrc, ob);
                            osrc = stage_off[sl].p;
                        }
                        hsa_copy(hoffs[sl].p, osrc, ob, false, eng_up, sig);
                        up_bytes += ob;
                    }
                    prep(c, sl, lines, text);
                    HIPCHK(hipEventRecord(prep_done[sl], up));
                    mark("uploaded", k);
                    {
                        std::lock_guard<std::mutex> g(m);
                        uploaded = k + 1;
                        h2d += up_bytes;
                    }
                    cv.notify_all();
                }
            } catch (...) {
                fail(std::current_exception());
            }
            if (have_sig) hsa_signal_destroy(sig);
            if (have_ssig)
                for (auto& x : ssig) hsa_signal_destroy(x);
        });
        w_down.run([&] {
            hsa_signal_t sig{};
            bool have_sig = false;
            try {
                HIPCHK(hipSetDevice(device));
                if (hsa_signal_create(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) throw Fail(EDSBWT_E_DEVICE, "hsa_signal_create failed");
                have_sig = true;
                for (;;) {
                    Job j;
                    {
                        std::unique_lock<std::mutex> lk(m);
                        cv.wait(lk, [&] { return stop || closed || !jobs.empty(); });
                        if (stop || jobs.empty()) break;
                        j = jobs.front();
                        jobs.pop_front();
                    }
                    const int sl = (int)(j.k % kSlots);
                    mark("download", j.k);
                    uint64_t dn = 0;
                    if (j.P && derive_counts) {
                        // the previous user of this slot's staging must have been widened
                        if (j.k >= (size_t)kSlots) {
                            std::unique_lock<std::mutex> lk(m);
                            cv.wait(lk, [&] { return stop || counted > j.k - kSlots; });
                            if (stop) break;
                        }
                        if (locate && j.n) {  // the records first: the byte counts were computed meanwhile
                            hsa_copy(arena + j.total, hrec[sl].p, j.n * sizeof(edsbwt_occ), true, eng_down, sig);
                            dn += j.n * sizeof(edsbwt_occ);
                            j.n = 0;
                        }
                        const uint64_t cb = c8_bytes(j.P);
                        stage_c8[sl].ensure(cb);
                        hsa_copy(stage_c8[sl].p, hc8[sl].p, cb, true, eng_down, sig);
                        dn += cb;
                        uint32_t ne = 0;
                        std::memcpy(&ne, static_cast<const uint8_t*>(stage_c8[sl].p) + cb - 8, 4);
                        if (ne > j.P) throw Fail(EDSBWT_E_DEVICE, "counts: more exceptions than patterns");
                        if (ne) {
                            stage_exc[sl].ensure((size_t)ne * 8);
                            hsa_copy(stage_exc[sl].p, hexc[sl].p, (size_t)ne * 8, true, eng_down, sig);
                            dn += (uint64_t)ne * 8;
                        }
                        j.nexc = ne;
                    } else if (j.P) {
                        if (pin_cnt) {
                            hsa_copy(counts + j.pats, hcounts[sl].p, j.P * 4, true, eng_down, sig);
                        } else {
                            stage_cnt[sl].ensure(j.P * 4);
                            hsa_copy(stage_cnt[sl].p, hcounts[sl].p, j.P * 4, true, eng_down, sig);
                            std::memcpy(counts + j.pats, stage_cnt[sl].p, j.P * 4);
                        }
                        dn += j.P * 4;
                    }
                    if (locate && j.n) {
                        hsa_copy(arena + j.total, hrec[sl].p, j.n * sizeof(edsbwt_occ), true, eng_down, sig);
                        dn += j.n * sizeof(edsbwt_occ);
                    }
                    mark("downloaded", j.k);
                    {
                        std::lock_guard<std::mutex> g(m);
                        downloaded = j.k + 1;
                        d2h += dn;
                        if (derive_counts) landed.push_back(j);
                    }
                    cv.notify_all();
                }
            } catch (...) {
                fail(std::current_exception());
            }
            if (have_sig) hsa_signal_destroy(sig);
        });
        if (derive_counts)
            w_cnt.run([&] {
                try {
                    for (size_t k = 0; k < nch; k++) {
                        Job j;
                        {
                            std::unique_lock<std::mutex> lk(m);
                            cv.wait(lk, [&] { return stop || landed.size() > k; });
                            if (stop) break;
                            j = landed[k];
                        }
                        const int sl = (int)(j.k % kSlots);
                        if (j.P)
                            expand_c8(counts + j.pats, static_cast<const uint8_t*>(stage_c8[sl].p), j.P,
                                      static_cast<const uint2*>(stage_exc[sl].p), j.nexc);
                        mark("counted", j.k);
                        {
                            std::lock_guard<std::mutex> g(m);
                            counted = k + 1;
                        }
                        cv.notify_all();
                    }
                } catch (...) {
                    fail(std::current_exception());
                }
            });
        edsbwt_stats agg{};
        uint64_t total = 0, pats = 0;
        try {
            for (size_t k = 0; k < nch; k++) {
                const Chunk& c = ch[k];
                const int sl = (int)(k % kSlots);
                {
                    std::unique_lock<std::mutex> lk(m);
                    cv.wait(lk, [&] { return stop || (uploaded > k && (k < (size_t)kSlots || downloaded > k - kSlots)); });
                    if (stop) break;
                }
                HIPCHK(hipEventSynchronize(prep_done[sl]));
                mark("search", k);
                uint64_t pm[3];
                std::memcpy(pm, prep_host(sl), 24);
                const uint64_t P = lines ? pm[0] : c.p1 - c.p0;
                known_len = P > 0;
                known_lmax = (uint32_t)pm[1];
                known_lmin = ~(uint32_t)pm[2];
                HIPCHK(hipStreamWaitEvent(stream, prep_done[sl], 0));
                if (pats + P > counts_cap) throw Fail(EDSBWT_E_ARG, "counts buffer holds " + std::to_string(counts_cap) + " patterns, the batch has more");
                if (counts_mirror && pats + P > counts_mirror_cap) throw Fail(EDSBWT_E_ARG, "device counts mirror smaller than the batch");
                hcounts[sl].ensure(P + 1);
                std::swap(rec, hrec[sl]);  // this chunk's records land in slot sl
                uint64_t n = 0;
                if (derive_counts && P) {
                    hc8[sl].ensure(c8_bytes(P));
                    hexc[sl].ensure(P);
                    c8_out = C8Out{hc8[sl].p, hexc[sl].p, reinterpret_cast<uint32_t*>(hc8[sl].p + c8_bytes(P) - 8)};
                }
                try {
                    n = search(hbytes[sl].p, hoffs[sl].p, P, first_id + (uint32_t)pats, flags, hcounts[sl].p);
                } catch (...) {
                    known_len = false;
                    c8_out = C8Out{};
                    std::swap(rec, hrec[sl]);
                    throw;
                }
                known_len = false;
                c8_out = C8Out{};
                std::swap(rec, hrec[sl]);
                mirror_counts(pats, P, hcounts[sl].p);
                mark("searched", k);
                accumulate(agg, st);
                if (locate && n && total + n > arena_cap) {
                    // the arena grows: every earlier chunk's records must have landed first
                    std::unique_lock<std::mutex> lk(m);
                    cv.wait(lk, [&] { return stop || downloaded == k; });
                    if (stop) break;
                    lk.unlock();
                    arena_ensure(total + n);
                }
                {
                    std::lock_guard<std::mutex> g(m);
                    jobs.push_back(Job{k, P, n, pats, total, 0});
                    searched = k + 1;
                }
                cv.notify_all();
                total += n;
                pats += P;
            }
            {
                std::unique_lock<std::mutex> lk(m);
                cv.wait(lk, [&] { return stop || (downloaded == nch && (!derive_counts || counted == nch)); });
                closed = true;
            }
            cv.notify_all();
        } catch (...) {
            fail(std::current_exception());
        }
        {
            std::lock_guard<std::mutex> g(m);
            closed = true;
        }
        cv.notify_all();
        w_up.wait();
        w_down.wait();
        if (derive_counts) w_cnt.wait();
        (void)hipStreamSynchronize(up);
        if (counts_mirror) (void)hipStreamSynchronize(stream);  // the mirror is complete when the call returns
        if (err) {
            (void)hipStreamSynchronize(stream);  // no kernel may still touch the slots
            std::rethrow_exception(err);
        }
        mark("drained", nch);
        if (trace) std::fprintf(stderr, "[edsbwt] host pipeline: %llu of %zu chunks went packed (2 bits per base)\n", (unsigned long long)packed, nch);
        for (auto& mk : marks) std::fprintf(stderr, "[edsbwt] t %8.3f ms  %-10s chunk %zu\n", std::get<2>(mk), std::get<0>(mk), std::get<1>(mk));
        st = agg;
        st.patterns = pats;
        st.occurrences = total;
        st.chunks = nch;
        st.bytes_h2d = h2d;
        st.bytes_d2h = d2h;
        st.ms_wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (npat_out) *npat_out = pats;
        if (occ_out) {
            *occ_out = nullptr;
            if (locate && total) {
                *occ_out = arena;
                arena_checkout();
            }
        }
        return total;
    }

    // edsbwt_prepare: the setup a host-memory batch of ~text_bytes bytes / npat lines would otherwise
    // pay inside its first call — the pipeline's threads, streams and copy-engine agents, every
    // slot's page-locked and device buffers at this batch's chunk sizes, the search workspace of a
    // chunk, and the page-locked record arena (records_hint records; 0: 1.25 per line) — done by one
    // run of the same pipeline over SYNTHETIC lines of the batch's mean length (random symbols of
    // the index's alphabet: nothing of the caller's batch is searched, and its results are dropped).
    // The reference does the index load and M_LF setup before its clock (MOVE_EDSBWTSearch.cpp:23-95,
    // 109); this is the same for the GPU pipeline, so the first real call runs at steady state.
    void prepare_lines(uint64_t text_bytes, uint64_t npat, uint64_t records_hint, uint32_t flags) {
        if (!npat || !text_bytes) return;
        const uint64_t L = std::max<uint64_t>(1, std::min<uint64_t>(255, (text_bytes + npat - 1) / npat - 1));
        const uint64_t nsyn = std::min<uint64_t>(npat, std::max<uint64_t>(1, text_bytes / (L + 1)));
        const uint64_t nb = nsyn * (L + 1);
        uint8_t* text = nullptr;
        uint32_t* counts = nullptr;
        if (hipHostMalloc((void**)&text, nb, hipHostMallocDefault) != hipSuccess) throw Fail(EDSBWT_E_NOMEM, "hipHostMalloc (prepare)");
        if (hipHostMalloc((void**)&counts, nsyn * 4, hipHostMallocDefault) != hipSuccess) {
            (void)hipHostFree(text);
            throw Fail(EDSBWT_E_NOMEM, "hipHostMalloc (prepare)");
        }
        struct Free {
            void* a;
            void* b;
            ~Free() { (void)hipHostFree(a); (void)hipHostFree(b); }
        } fr{text, counts};
        // random symbols of the alphabet (alpha[1..sigma-1]; alpha[0] is '#'), one xorshift per line
        const uint32_t B = std::max(1u, sigma - 1);
        pipe_init();
        const unsigned T = (unsigned)std::min<uint64_t>(pool.size(), std::max<uint64_t>(1, nsyn >> 16));
        pool.run(T, [&](unsigned t) {
            for (uint64_t i = nsyn * t / T; i < nsyn * (t + 1) / T; i++) {
                uint64_t x = 0x9E3779B97F4A7C15ull * (i + 1);
                uint8_t* q = text + i * (L + 1);
                for (uint64_t j = 0; j < L; j++) {
                    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
                    q[j] = alpha[1 + (uint32_t)(x % B)];
                }
                q[L] = '\n';
            }
        });
        edsbwt_occ* occ = nullptr;
        uint64_t np = 0;
        search_host(text, nb, nullptr, 0, true, 1, flags & (EDSBWT_LOCATE | EDSBWT_COUNT_ONLY | EDSBWT_LOCATE_TABLE), counts, nsyn, &occ, &np);
        if (occ) arena_checkin();  // (the synthetic records are dropped: the arena stays the engine's)
        const bool locate = (flags & EDSBWT_LOCATE) && !(flags & EDSBWT_COUNT_ONLY);
        if (locate) arena_ensure(records_hint ? records_hint : npat + npat / 4);
        st = edsbwt_stats{};
    }

    // The pattern loop of MOVE_EDSBWT (MOVE_EDSBWTSearch.cpp:97-155) over a batch in host memory,
    // timed as SURVEY §8(d) defines patterns/s: from the first H2D of the patterns to the last
    // D2H of counts and records.  lines != 0: `text` is the pattern file as it lies on disk
    // (getline semantics, :111: split at '\n', a last line without '\n' counts); else
    // text/offs is a packed (bytes, offsets[npat+1]) batch.  Returns the records (page-locked,
    // library-owned) and their number; *npat_out = patterns seen.
    uint64_t search_host(const uint8_t* text, uint64_t len, const uint64_t* offs, uint64_t npat, bool lines, uint32_t first_id,
                         uint32_t flags, uint32_t* counts, uint64_t counts_cap, edsbwt_occ** occ_out, uint64_t* npat_out) {
        const auto t0 = std::chrono::steady_clock::now();
        pipe_init();
        const bool locate = (flags & EDSBWT_LOCATE) && !(flags & EDSBWT_COUNT_ONLY);
        const bool pin_in = host_pinned(text), pin_off = lines || host_pinned(offs), pin_cnt = host_pinned(counts);
        // downloads by the copy engine (EDSBWT_D2H_KERNEL=1: kernel stores to mapped host memory;
        // measured slower on MI355X: their PCIe stores slow the search kernels running beside them)
        const bool sdma_down = env_double("EDSBWT_D2H_KERNEL", 0) == 0;
        uint32_t* counts_dev = pin_cnt ? static_cast<uint32_t*>(host_dev_ptr(counts)) : nullptr;
        // a packed batch's size is known up front: refuse it before any chunk is searched (a lines
        // batch is counted chunk by chunk, each checked before its search)
        if (!lines && counts_mirror && npat > counts_mirror_cap) throw Fail(EDSBWT_E_ARG, "device counts mirror smaller than the batch");
        std::vector<Chunk> ch = cut_chunks(text, len, offs, npat, lines);
        {
            const bool eager_req = !lines && pin_in && pin_off && env_double("EDSBWT_EAGER_UP", 0) != 0;
            const bool compact_req = locate && env_double("EDSBWT_D2H_COMPACT", 0) != 0;
            if (!eager_req && !compact_req && sdma_down && hsa_init())
                return search_host_hsa(ch, text, offs, lines, pin_in, pin_off, pin_cnt, first_id, flags, counts, counts_cap, locate, occ_out,
                                       npat_out, t0);
        }
        // page-locked inputs: every chunk's upload is queued at once, into its own 256-B aligned
        // place of one device buffer, so the copy engine never idles; pageable inputs are staged
        // through page-locked buffers slot by slot
        // (EDSBWT_EAGER_UP=1; off by default: uploads and downloads share one copy engine, which then
        // serves every upload before the first download)
        const bool eager = !lines && pin_in && pin_off && env_double("EDSBWT_EAGER_UP", 0) != 0;
        if (eager) {
            uint64_t at = 0;
            for (auto& c : ch) {
                c.dpos = at;
                at += (c.b1 - c.b0 + 16 + 255) / 256 * 256;
            }
            hin_all.ensure(at + 16);
            if (!lines) hoff_all.ensure(npat + ch.size());
            while (chunk_ev.size() < ch.size()) {
                hipEvent_t e;
                HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
                chunk_ev.push_back(e);
            }
        }
        if (arena_checked_out()) arena_release();  // the caller still holds the last records: start a new buffer
        edsbwt_stats agg{};
        uint64_t total = 0, pats = 0, h2d = 0, d2h = 0;
        // compact downloads: a host thread expands each chunk's records as soon as its download has landed
        // (EDSBWT_D2H_COMPACT=1; off by default: on the MI355X host the expansion costs more than the
        // smaller download saves)
        const bool compact = locate && env_double("EDSBWT_D2H_COMPACT", 0) != 0 && !h_seg_of_word.empty();
        while (chunk_down_ev.size() < ch.size()) {
            hipEvent_t e;
            HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            chunk_down_ev.push_back(e);
        }
        struct XJob { uint64_t p0, P, r0, n; hipEvent_t ev; };
        std::vector<XJob> xjobs;
        std::mutex xm;
        std::condition_variable xcv;
        bool xclosed = false;
        std::exception_ptr xerr;
        std::thread xth;
        auto xpost = [&](XJob j) {
            if (!xth.joinable())
                xth = std::thread([&] {
                    for (size_t q = 0;; q++) {
                        XJob jb;
                        {
                            std::unique_lock<std::mutex> lk(xm);
                            xcv.wait(lk, [&] { return xclosed || q < xjobs.size(); });
                            if (q >= xjobs.size()) return;
                            jb = xjobs[q];
                        }
                        try {
                            HIPCHK(hipEventSynchronize(jb.ev));
                            const auto tx = std::chrono::steady_clock::now();
                            expand_chunk(counts, jb.p0, jb.P, jb.r0, jb.n, first_id);
                            if (trace)
                                std::fprintf(stderr, "[edsbwt] expand chunk %zu: %llu records in %.3f ms, done at %.3f ms\n", q,
                                             (unsigned long long)jb.n,
                                             std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tx).count(),
                                             std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
                        } catch (...) {
                            std::lock_guard<std::mutex> g(xm);
                            if (!xerr) xerr = std::current_exception();
                        }
                    }
                });
            std::lock_guard<std::mutex> g(xm);
            xjobs.push_back(j);
            xcv.notify_all();
        };
        auto xfinish = [&] {
            {
                std::lock_guard<std::mutex> g(xm);
                xclosed = true;
            }
            xcv.notify_all();
            if (xth.joinable()) xth.join();
            if (xerr) std::rethrow_exception(xerr);
        };
        try {
        auto issue = [&](size_t k) {
            const Chunk& c = ch[k];
            const int sl = (int)(k % kSlots);
            const uint64_t nb = c.b1 - c.b0;
            if (eager) {
                if (nb) HIPCHK(hipMemcpyAsync(hin_all.p + c.dpos, text + c.b0, nb, hipMemcpyHostToDevice, up));
                if (!lines) {
                    HIPCHK(hipMemcpyAsync(hoff_all.p + c.p0 + k, offs + c.p0, (c.p1 - c.p0 + 1) * 8, hipMemcpyHostToDevice, up));
                    h2d += (c.p1 - c.p0 + 1) * 8;
                }
                h2d += nb;
                HIPCHK(hipEventRecord(chunk_ev[k], up));
                return;
            }
            if (lines) {
                hraw[sl].ensure(nb + 16);
                upload(hraw[sl].p, text + c.b0, nb, pin_in, stage_in[sl], sl);
            } else {
                hbytes[sl].ensure(nb + 16);
                hoffs[sl].ensure(c.p1 - c.p0 + 1);
                upload(hbytes[sl].p, text + c.b0, nb, pin_in, stage_in[sl], sl);
                upload(hoffs[sl].p, offs + c.p0, (c.p1 - c.p0 + 1) * 8, pin_off, stage_off[sl], sl);
                h2d += (c.p1 - c.p0 + 1) * 8;
            }
            h2d += nb;
            HIPCHK(hipEventRecord(up_done[sl], up));
            prep(c, sl, lines, text);
            HIPCHK(hipEventRecord(prep_done[sl], up));
        };
        // EDSBWT_TRACE: host timeline of the pipeline (printed at the end)
        std::vector<std::tuple<const char*, size_t, double>> marks;
        auto mark = [&](const char* what, size_t k) {
            if (trace) marks.emplace_back(what, k, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        };
        // uploads run two chunks ahead of the search: chunk k+2's upload and prep overlap
        // chunk k's search and chunk k-1's download
        const size_t ahead = (size_t)std::max(1.0, std::min<double>(kSlots - 2, env_double("EDSBWT_AHEAD", 2)));
        size_t issued = 0;
        if (eager) {
            for (size_t k = 0; k < ch.size(); k++) issue(k);
            issued = ch.size();
        }
        for (size_t k = 0; k < ch.size(); k++) {
            const Chunk& c = ch[k];
            const int sl = (int)(k % kSlots);
            while (issued < ch.size() && issued <= k + ahead) { mark("issue", issued); issue(issued++); }
            mark("issued", k);
            const auto tc = std::chrono::steady_clock::now();
            uint64_t P;
            const uint8_t* bytes_k = nullptr;
            uint64_t* offs_k = nullptr;
            if (eager) {
                HIPCHK(hipStreamWaitEvent(stream, chunk_ev[k], 0));
                P = c.p1 - c.p0;
                bytes_k = hin_all.p + c.dpos;
                offs_k = hoff_all.p + c.p0 + k;
                if (c.b0) launch(KC_TRIE, k_rebase, P + 1, offs_k, P + 1, c.b0);
                known_len = false;
            } else {
                // the prep's pattern count and lengths (it ran on `up` right after the upload)
                HIPCHK(hipEventSynchronize(prep_done[sl]));
                mark("prep_ready", k);
                HIPCHK(hipStreamWaitEvent(stream, prep_done[sl], 0));
                uint64_t pm[3];
                std::memcpy(pm, prep_host(sl), 24);
                P = lines ? pm[0] : c.p1 - c.p0;
                known_len = P > 0;
                known_lmax = (uint32_t)pm[1];
                known_lmin = ~(uint32_t)pm[2];
                bytes_k = hbytes[sl].p;
                offs_k = hoffs[sl].p;
            }
            HIPCHK(hipStreamWaitEvent(stream, down_done[sl], 0));  // chunk k-3's results have left the slot
            if (pats + P > counts_cap) throw Fail(EDSBWT_E_ARG, "counts buffer holds " + std::to_string(counts_cap) + " patterns, the batch has more");
            if (counts_mirror && pats + P > counts_mirror_cap) throw Fail(EDSBWT_E_ARG, "device counts mirror smaller than the batch");
            hcounts[sl].ensure(P + 1);
            std::swap(rec, hrec[sl]);  // this chunk's records land in slot sl
            uint64_t n = 0;
            try {
                n = search(bytes_k, offs_k, P, first_id + (uint32_t)pats, flags, hcounts[sl].p);
            } catch (...) {
                known_len = false;
                std::swap(rec, hrec[sl]);
                throw;
            }
            known_len = false;
            std::swap(rec, hrec[sl]);
            mirror_counts(pats, P, hcounts[sl].p);
            if (compact && locate && n) {  // (word, offset) per record for the download
                hrec8[sl].ensure(n);
                launch(KC_LOCATE, k_rec_compact, n, (const edsbwt_occ*)hrec[sl].p, n, hrec8[sl].p);
            }
            mark("searched", k);
            accumulate(agg, st);
            if (trace)
                std::fprintf(stderr, "[edsbwt] chunk %zu: %llu patterns, %llu records, search %.3f ms host / %.3f ms device, at %.3f ms\n", k,
                             (unsigned long long)P, (unsigned long long)n, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tc).count(),
                             st.ms_total, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
            // results back on `down`
            HIPCHK(hipEventRecord(comp_done[sl], stream));
            HIPCHK(hipStreamWaitEvent(down, comp_done[sl], 0));
            if (P) {
                if (counts_dev && !sdma_down) {
                    download(counts_dev + pats, hcounts[sl].p, P * 4);
                } else if (pin_cnt) {
                    HIPCHK(hipMemcpyAsync(counts + pats, hcounts[sl].p, P * 4, hipMemcpyDeviceToHost, down));
                } else {
                    HIPCHK(hipEventSynchronize(down_done[sl]));
                    stage_cnt[sl].ensure(P * 4);
                    HIPCHK(hipMemcpyAsync(stage_cnt[sl].p, hcounts[sl].p, P * 4, hipMemcpyDeviceToHost, down));
                    HIPCHK(hipStreamSynchronize(down));
                    std::memcpy(counts + pats, stage_cnt[sl].p, P * 4);
                }
                d2h += P * 4;
            }
            if (locate && n) {
                arena_ensure(total + n);
                if (compact) {
                    arena8_ensure(total + n);
                    HIPCHK(hipMemcpyAsync(arena8 + total, hrec8[sl].p, n * sizeof(uint2), hipMemcpyDeviceToHost, down));
                    d2h += n * sizeof(uint2);
                } else {
                    if (arena_dev && !sdma_down) download(arena_dev + total, hrec[sl].p, n * sizeof(edsbwt_occ));
                    else HIPCHK(hipMemcpyAsync(arena + total, hrec[sl].p, n * sizeof(edsbwt_occ), hipMemcpyDeviceToHost, down));
                    d2h += n * sizeof(edsbwt_occ);
                }
            }
            HIPCHK(hipEventRecord(down_done[sl], down));
            mark("d2h_queued", k);
            if (compact && locate && n) {
                HIPCHK(hipEventRecord(chunk_down_ev[k], down));
                xpost({pats, P, total, n, chunk_down_ev[k]});
            }
            total += n;
            pats += P;
        }
        xfinish();
        if (counts_mirror) HIPCHK(hipStreamSynchronize(stream));  // the mirror is complete when the call returns
        HIPCHK(hipStreamSynchronize(down));
        HIPCHK(hipStreamSynchronize(up));
        mark("drained", ch.size());
        for (auto& m : marks) std::fprintf(stderr, "[edsbwt] t %8.3f ms  %-10s chunk %zu\n", std::get<2>(m), std::get<0>(m), std::get<1>(m));
        } catch (...) {  // no copy may still touch the caller's buffers
            try { xfinish(); } catch (...) {}
            (void)hipStreamSynchronize(up);
            (void)hipStreamSynchronize(stream);
            (void)hipStreamSynchronize(down);
            throw;
        }
        st = agg;
        st.patterns = pats;
        st.occurrences = total;
        st.chunks = ch.size();
        st.bytes_h2d = h2d;
        st.bytes_d2h = d2h;
        st.ms_wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (npat_out) *npat_out = pats;
        if (occ_out) {
            *occ_out = nullptr;
            if (locate && total) {
                *occ_out = arena;
                arena_checkout();
            }
        }
        return total;
    }
    // edsbwt_set_counts_mirror: a chunk's u32 counts also go to the caller's device array (every
    // host-pipeline path; the capacity was checked before the chunk's search)
    void mirror_counts(uint64_t pats, uint64_t P, const uint32_t* d_counts) {
        if (!counts_mirror || !P) return;
        if (pats + P > counts_mirror_cap) throw Fail(EDSBWT_E_ARG, "device counts mirror smaller than the batch");
        HIPCHK(hipMemcpyAsync(counts_mirror + pats, d_counts, P * 4, hipMemcpyDeviceToDevice, stream));
    }
    uint64_t* pinned_u64() { return reinterpret_cast<uint64_t*>(pinned + 8); }
    template <typename K, typename... A>
    void launch_blocks(int k, K kern, size_t blocks, A... a) {
        if (!blocks) return;
        timed(k, [&] { hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, stream, a...); });
        HIPCHK(hipGetLastError());
        sync_check((const void*)kern);
        st.launches_kernel[k]++;
    }
    static void accumulate(edsbwt_stats& a, const edsbwt_stats& b) {
        a.found += b.found; a.not_found += b.not_found; a.occurrences += b.occurrences;
        a.depths = std::max(a.depths, b.depths); a.trie_nodes += b.trie_nodes; a.intervals_stepped += b.intervals_stepped;
        a.link_hash_rows += b.link_hash_rows; a.link_ranges += b.link_ranges; a.locate_lf_steps += b.locate_lf_steps;
        a.deep_from_depth = std::max(a.deep_from_depth, b.deep_from_depth); a.deep_overflow += b.deep_overflow;
        a.deep_level_rerun += b.deep_level_rerun; a.ms_total += b.ms_total;
        for (int k = 0; k < 16; k++) {
            a.ms_kernel[k] += b.ms_kernel[k]; a.launches_kernel[k] += b.launches_kernel[k];
            a.bytes_kernel[k] += b.bytes_kernel[k]; a.lines_kernel[k] += b.lines_kernel[k];
        }
        a.locate_offsets += b.locate_offsets; a.search_groups = std::max(a.search_groups, b.search_groups);
        a.start_depth = std::max(a.start_depth, b.start_depth);
        a.text_chars += b.text_chars; a.text_rows += b.text_rows; a.redo_searches += b.redo_searches;
    }

    ~Engine() {
        if (xs) (void)hipStreamSynchronize(xs);
        if (comm) (void)Rccl::get().destroy(comm);
        for (auto& g : gathers)
            if (g.ev) (void)hipEventDestroy(g.ev);
        if (xs_after) (void)hipEventDestroy(xs_after);
        if (xs) (void)hipStreamDestroy(xs);
        if (stream) (void)hipStreamSynchronize(stream);
        if (stream2) (void)hipStreamSynchronize(stream2);
        for (auto e : piece_ev) (void)hipEventDestroy(e);
        if (tiles_ev) (void)hipEventDestroy(tiles_ev);
        if (tiles_ev0) (void)hipEventDestroy(tiles_ev0);
        if (stream2) (void)hipStreamDestroy(stream2);
        if (up) (void)hipStreamSynchronize(up);
        if (down) (void)hipStreamSynchronize(down);
        for (auto e : chunk_ev) (void)hipEventDestroy(e);
        for (auto e : chunk_down_ev) (void)hipEventDestroy(e);
        if (arena8) (void)hipHostFree(arena8);
        for (int k = 0; k < kSlots; k++) {
            if (up_done[k]) (void)hipEventDestroy(up_done[k]);
            if (comp_done[k]) (void)hipEventDestroy(comp_done[k]);
            if (down_done[k]) (void)hipEventDestroy(down_done[k]);
            stage_in[k].release(); stage_off[k].release(); stage_cnt[k].release(); stage_pack[k].release(); stage_c8[k].release(); stage_exc[k].release();
        }
        if (up) (void)hipStreamDestroy(up);
        if (down) (void)hipStreamDestroy(down);
        arena_release();
        for (auto& e : ev_pool) { (void)hipEventDestroy(e.a); (void)hipEventDestroy(e.b); }
        if (hostblk) (void)hipHostFree(hostblk);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

void Engine::arena_register() {
    auto& R = occ_registry();
    std::lock_guard<std::mutex> g(R.m);
    R.own[arena] = {this, false};
}
void Engine::arena_checkout() {
    auto& R = occ_registry();
    std::lock_guard<std::mutex> g(R.m);
    R.own[arena] = {this, true};
}
void Engine::arena_checkin() {
    auto& R = occ_registry();
    std::lock_guard<std::mutex> g(R.m);
    auto it = R.own.find(arena);
    if (it != R.own.end()) it->second.second = false;
}
bool Engine::arena_checked_out() {
    if (!arena) return false;
    auto& R = occ_registry();
    std::lock_guard<std::mutex> g(R.m);
    auto it = R.own.find(arena);
    return it != R.own.end() && it->second.second;
}
void Engine::arena_release() {
    if (!arena) return;
    bool out = false;
    {
        auto& R = occ_registry();
        std::lock_guard<std::mutex> g(R.m);
        auto it = R.own.find(arena);
        out = it != R.own.end() && it->second.second;
        if (out) it->second.first = nullptr;  // detached: edsbwt_occ_free frees it
        else if (it != R.own.end()) R.own.erase(it);
    }
    if (!out) (void)hipHostFree(arena);
    arena = nullptr;
    arena_cap = 0;
}
// edsbwt_occ_free: give an engine's buffer back, free a detached one, or free() a malloc'd one
static void occ_free_any(edsbwt_occ* p) {
    if (!p) return;
    {
        auto& R = occ_registry();
        std::lock_guard<std::mutex> g(R.m);
        auto it = R.own.find(p);
        if (it != R.own.end()) {
            if (it->second.first) {
                it->second.second = false;
                return;
            }
            R.own.erase(it);
        } else {
            std::free(p);
            return;
        }
    }
    (void)hipHostFree(p);
}

}  // namespace edsbwt

using edsbwt::Engine;
using edsbwt::Fail;
using edsbwt::Rccl;

struct edsbwt_index {
    std::unique_ptr<Engine> eng;
};

#define ABI_TRY try {
#define ABI_CATCH                                                        \
    }                                                                    \
    catch (const Fail& f) {                                              \
        edsbwt::g_err = f.what();                                        \
        return f.code;                                                   \
    }                                                                    \
    catch (const std::bad_alloc&) {                                      \
        edsbwt::g_err = "host allocation failed";                        \
        return EDSBWT_E_NOMEM;                                           \
    }                                                                    \
    catch (const std::exception& e) {                                    \
        edsbwt::g_err = e.what();                                        \
        return EDSBWT_E_DEVICE;                                          \
    }

namespace edsbwt {
// ------------------------------------------------------------ index writer: GPU suffix sort
// The generalized suffix array eds_transform needs (gsufsort's order over word·'#',
// EDS-BWTransform.sh:26): suffixes compared up to and including their word's '#' ('#' = code 0,
// the smallest), equal ones by text position (= word id).  Prefix doubling over ranks: the
// first key packs each suffix's next cpw codes (zeros after its '#'); round h sorts by
// (rank[t], rank[t+h]) — or (rank[t], 0) when t's '#' lies within its first h codes — stably,
// from the previous order, so equal keys keep position order; it stops once h passes the
// longest word.  O(log(longest word)) radix sorts of N 64-bit keys.
__global__ void k_gsa_dist(const uint64_t* __restrict__ ends, uint64_t W, uint64_t n, uint32_t* __restrict__ dist) {
    GRID_STRIDE(t, n) {
        uint64_t lo = 0, hi = W;  // first '#' at or after t
        while (lo < hi) {
            const uint64_t m = (lo + hi) >> 1;
            if (ends[m] < t) lo = m + 1; else hi = m;
        }
        dist[t] = (uint32_t)(ends[lo] - t);
    }
}
__global__ void k_gsa_key0(const uint8_t* __restrict__ codes, const uint32_t* __restrict__ dist, uint64_t n, uint32_t b, uint32_t cpw,
                           uint64_t* __restrict__ key, uint32_t* __restrict__ pos) {
    GRID_STRIDE(t, n) {
        const uint32_t m = min(dist[t] + 1, cpw);  // codes through the '#', at most cpw
        uint64_t k = 0;
        for (uint32_t j = 0; j < cpw; j++) k = (k << b) | (j < m ? (uint64_t)codes[t + j] : 0ull);
        key[t] = k;
        pos[t] = (uint32_t)t;
    }
}
// group-start index of sorted entry i (heads by key inequality), as rank of its suffix
__global__ void k_gsa_heads(const uint64_t* __restrict__ key, uint64_t n, uint32_t* __restrict__ head) {
    GRID_STRIDE(i, n) head[i] = (i == 0 || key[i] != key[i - 1]) ? (uint32_t)i : 0u;
}
__global__ void k_gsa_rank(const uint32_t* __restrict__ sa, const uint32_t* __restrict__ grp, uint64_t n, uint32_t* __restrict__ rank) {
    GRID_STRIDE(i, n) rank[sa[i]] = grp[i];
}
__global__ void k_gsa_key(const uint32_t* __restrict__ sa, const uint32_t* __restrict__ rank, const uint32_t* __restrict__ dist, uint64_t n,
                          uint64_t h, uint64_t* __restrict__ key) {
    GRID_STRIDE(i, n) {
        const uint32_t t = sa[i];
        key[i] = (uint64_t)rank[t] << 32 | (dist[t] < h ? 0ull : (uint64_t)rank[t + h] + 1ull);
    }
}
struct MaxOp {
    __device__ __forceinline__ uint32_t operator()(uint32_t a, uint32_t b) const { return a > b ? a : b; }
};

static void gsa_sort(const uint8_t* h_codes, uint64_t n, const uint64_t* h_ends, uint64_t W, uint32_t b, int device, uint32_t* h_sa,
                     double* ms_out) {
    if (!n) return;
    if (n > 0x7fffffffull) throw Fail(EDSBWT_E_UNSUPPORTED, "text longer than 2^31-1 symbols (the suffix sort's hipcub passes count items in int)");
    if (b < 1 || b > 8) throw Fail(EDSBWT_E_ARG, "bits per code must be 1..8");
    if (!W || h_ends[W - 1] != n - 1) throw Fail(EDSBWT_E_ARG, "the text must end with a word's '#'");
    HIPCHK(hipSetDevice(device));
    hipStream_t s;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    struct StreamGuard { hipStream_t s; ~StreamGuard() { (void)hipStreamSynchronize(s); (void)hipStreamDestroy(s); } } sg{s};
    const auto t0 = std::chrono::steady_clock::now();
    const uint32_t cpw = 64 / b;
    DBuf<uint8_t> codes;
    DBuf<uint64_t> ends, k1, k2;
    DBuf<uint32_t> dist, sa1, sa2, grp, rank;
    DBuf<uint8_t> tmp;
    codes.ensure(n + cpw);
    ends.ensure(W);
    HIPCHK(hipMemcpyAsync(codes.p, h_codes, n, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemsetAsync(codes.p + n, 0, cpw, s));
    HIPCHK(hipMemcpyAsync(ends.p, h_ends, W * 8, hipMemcpyHostToDevice, s));
    dist.ensure(n); k1.ensure(n); k2.ensure(n); sa1.ensure(n); sa2.ensure(n); grp.ensure(n); rank.ensure(n);
    const unsigned G = (unsigned)std::min<uint64_t>(65535, (n + 255) / 256);
    hipLaunchKernelGGL(k_gsa_dist, dim3(G), dim3(256), 0, s, (const uint64_t*)ends.p, W, n, dist.p);
    hipLaunchKernelGGL(k_gsa_key0, dim3(G), dim3(256), 0, s, (const uint8_t*)codes.p, (const uint32_t*)dist.p, n, b, cpw, k1.p, sa1.p);
    HIPCHK(hipGetLastError());
    const int nbits = (int)std::max<uint32_t>(1, 64 - __builtin_clzll((unsigned long long)n));  // ranks < n
    auto sort = [&](int end_bit) {
        size_t tb = 0;
        HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k1.p, k2.p, sa1.p, sa2.p, cub_n(n), 0, end_bit, s));
        tmp.ensure(tb);
        HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, k1.p, k2.p, sa1.p, sa2.p, cub_n(n), 0, end_bit, s));
        std::swap(k1.p, k2.p); std::swap(k1.cap, k2.cap);
        std::swap(sa1.p, sa2.p); std::swap(sa1.cap, sa2.cap);
    };
    auto ranks = [&]() {
        hipLaunchKernelGGL(k_gsa_heads, dim3(G), dim3(256), 0, s, (const uint64_t*)k1.p, n, sa2.p);
        size_t tb = 0;
        HIPCHK(hipcub::DeviceScan::InclusiveScan(nullptr, tb, sa2.p, grp.p, MaxOp{}, cub_n(n), s));
        tmp.ensure(tb);
        HIPCHK(hipcub::DeviceScan::InclusiveScan(tmp.p, tb, sa2.p, grp.p, MaxOp{}, cub_n(n), s));
        hipLaunchKernelGGL(k_gsa_rank, dim3(G), dim3(256), 0, s, (const uint32_t*)sa1.p, (const uint32_t*)grp.p, n, rank.p);
        HIPCHK(hipGetLastError());
    };
    sort((int)(b * cpw));
    // longest word (with its '#'): the rounds stop once h passes it
    uint64_t maxw = 0, prev = 0;
    for (uint64_t w = 0; w < W; w++) { maxw = std::max<uint64_t>(maxw, h_ends[w] + 1 - prev); prev = h_ends[w] + 1; }
    for (uint64_t h = cpw; h < maxw; h *= 2) {
        ranks();
        hipLaunchKernelGGL(k_gsa_key, dim3(G), dim3(256), 0, s, (const uint32_t*)sa1.p, (const uint32_t*)rank.p, (const uint32_t*)dist.p, n, h, k1.p);
        HIPCHK(hipGetLastError());
        sort(std::min(64, 32 + nbits + 1));
    }
    HIPCHK(hipMemcpyAsync(h_sa, sa1.p, n * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (ms_out) *ms_out = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
}  // namespace edsbwt

extern "C" {

int edsbwt_abi_version(void) { return EDSBWT_ABI_VERSION; }
const char* edsbwt_last_error(void) { return edsbwt::g_err.c_str(); }

int edsbwt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}
const char* edsbwt_kernel_name(int k) { return (k >= 0 && k < edsbwt::KC_COUNT) ? edsbwt::kKNames[k] : ""; }

int edsbwt_index_open(const char* base, int device, uint32_t a_balance, edsbwt_index** out) {
    (void)a_balance;
    if (!base || !out) { edsbwt::g_err = "null argument"; return EDSBWT_E_ARG; }
    *out = nullptr;
    ABI_TRY
    auto h = std::make_unique<edsbwt_index>();
    h->eng = std::make_unique<Engine>();
    h->eng->open(base, device);
    *out = h.release();
    return 0;
    ABI_CATCH
}

void edsbwt_index_close(edsbwt_index* idx) {
    if (!idx) return;
    try { delete idx; } catch (...) {}
}

int edsbwt_index_get_info(const edsbwt_index* idx, edsbwt_index_info* info) {
    if (!idx || !info) { edsbwt::g_err = "null argument"; return EDSBWT_E_ARG; }
    const Engine& E = *idx->eng;
    std::memset(info, 0, sizeof *info);
    info->n_rows = E.N;
    info->n_words = E.W;
    info->n_segments = E.S;
    info->sigma = E.sigma;
    std::memcpy(info->alphabet, E.alpha, sizeof info->alphabet);
    info->device_bytes = E.device_bytes;
    info->ktab_depth = E.ktab_depth;
    info->ktab_items = E.ktab_items;
    info->ltab_depth = E.lt_depth;
    info->ltab_groups = E.lt_G;
    info->ltab_items = E.lt_items;
    info->open_peak_bytes = E.open_peak_bytes;
    info->open_seconds = E.open_seconds;
    info->pair_blocks = E.rent2.p != nullptr;
    return 0;
}

static int search_device_impl(edsbwt_index* idx, const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t npat,
                              uint32_t first_pattern_id, const uint32_t* d_ids, uint32_t flags, uint32_t* d_counts, edsbwt_occ** d_occ,
                              uint64_t* nocc, void* stream) {
    if (!idx || (!d_counts && npat) || (npat && (!d_bytes || !d_offsets))) { edsbwt::g_err = "null argument"; return EDSBWT_E_ARG; }
    ABI_TRY
    Engine& E = *idx->eng;
    HIPCHK(hipSetDevice(E.device));
    // order after the caller's stream — the null (legacy default) stream when stream is NULL,
    // which the engine's non-blocking stream would not wait for by itself
    hipEvent_t ev;
    HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(ev, (hipStream_t)stream));
    HIPCHK(hipStreamWaitEvent(E.stream, ev, 0));
    (void)hipEventDestroy(ev);
    E.wait_gathers_on(d_counts);  // (a gather of the previous use of this buffer must end first)
    struct TagReset { bool& t; ~TagReset() { t = false; } } tr{E.tag_now};
    if (E.tag_paths) {
        E.ptag.ensure(npat + 1);
        HIPCHK(hipMemsetAsync(E.ptag.p, 0, npat + 1, E.stream));
        E.ptag_n = npat;
        E.tag_now = true;
    }
    struct IdsReset { const uint32_t*& p; ~IdsReset() { p = nullptr; } } ir{E.pat_ids};
    E.pat_ids = d_ids;
    uint64_t n = E.search(d_bytes, d_offsets, npat, first_pattern_id, flags, d_counts);
    if (d_occ) *d_occ = n ? E.rec.p : nullptr;
    if (nocc) *nocc = n;
    return 0;
    ABI_CATCH
}

int edsbwt_search_device(edsbwt_index* idx, const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t npat,
                         uint32_t first_pattern_id, uint32_t flags, uint32_t* d_counts, edsbwt_occ** d_occ, uint64_t* nocc,
                         void* stream) {
    return search_device_impl(idx, d_bytes, d_offsets, npat, first_pattern_id, nullptr, flags, d_counts, d_occ, nocc, stream);
}

int edsbwt_search_device_ids(edsbwt_index* idx, const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t npat,
                             const uint32_t* d_ids, uint32_t flags, uint32_t* d_counts, edsbwt_occ** d_occ, uint64_t* nocc,
                             void* stream) {
    if (npat && !d_ids) { edsbwt::g_err = "null argument"; return EDSBWT_E_ARG; }
    // the legacy engine order sorts records by #Pat = first_pattern_id + i (no id map)
    if (flags & EDSBWT_LEGACY_ORDER) { edsbwt::g_err = "EDSBWT_LEGACY_ORDER with an id map"; return EDSBWT_E_ARG; }
    return search_device_impl(idx, d_bytes, d_offsets, npat, 0, d_ids, flags, d_counts, d_occ, nocc, stream);
}

int edsbwt_search(edsbwt_index* idx, const char* pat_bytes, const uint64_t* pat_offsets, uint64_t npat, uint32_t first_pattern_id,
                  uint32_t flags, uint32_t* counts, edsbwt_occ** occ, uint64_t* nocc) {
    if (!idx || (npat && (!pat_offsets || !counts))) { edsbwt::g_err = "null argument"; return EDSBWT_E_ARG; }
    if (occ) *occ = nullptr;
    if (nocc) *nocc = 0;
    ABI_TRY
    Engine& E = *idx->eng;
    HIPCHK(hipSetDevice(E.device));
    if (npat && !pat_bytes && pat_offsets[npat]) throw Fail(EDSBWT_E_ARG, "null pattern bytes");
    E.wait_gathers_on(E.counts_mirror);
    uint64_t n = E.search_host((const uint8_t*)pat_bytes, npat ? pat_offsets[npat] : 0, pat_offsets, npat, false, first_pattern_id, flags,
                               counts, npat, occ, nullptr);
    if (nocc) *nocc = n;
    return 0;
    ABI_CATCH
}

int edsbwt_search_lines(edsbwt_index* idx, const char* text, uint64_t len, uint32_t first_pattern_id, uint32_t flags, uint32_t* counts,
                        uint64_t counts_cap, uint64_t* npat, edsbwt_occ** occ, uint64_t* nocc) {
    if (!idx || (len && (!text || !counts))) { edsbwt::g_err = "null argument"; return EDSBWT_E_ARG; }
    if (occ) *occ = nullptr;
    if (nocc) *nocc = 0;
    if (npat) *npat = 0;
    ABI_TRY
    Engine& E = *idx->eng;
    HIPCHK(hipSetDevice(E.device));
    E.wait_gathers_on(E.counts_mirror);
    uint64_t n = E.search_host((const uint8_t*)text, len, nullptr, 0, true, first_pattern_id, flags, counts, counts_cap, occ, npat);
    if (nocc) *nocc = n;
    return 0;
    ABI_CATCH
}

int edsbwt_prepare(edsbwt_index* idx, uint64_t text_bytes, uint64_t npat, uint64_t records_hint, uint32_t flags) {
    if (!idx) { edsbwt::g_err = "null argument"; return EDSBWT_E_ARG; }
    ABI_TRY
    Engine& E = *idx->eng;
    HIPCHK(hipSetDevice(E.device));
    E.prepare_lines(text_bytes, npat, records_hint, flags);
    return 0;
    ABI_CATCH
}

int edsbwt_host_alloc(uint64_t bytes, void** out) {
    if (!out) { edsbwt::g_err = "null argument"; return EDSBWT_E_ARG; }
    *out = nullptr;
    if (hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
        *out = nullptr;
        edsbwt::g_err = "hipHostMalloc of " + std::to_string(bytes) + " bytes failed";
        return EDSBWT_E_NOMEM;
    }
    return 0;
}

void edsbwt_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

const char* edsbwt_build_id(void) { return EDSBWT_BUILD_ID; }

void edsbwt_occ_free(edsbwt_occ* occ) { edsbwt::occ_free_any(occ); }

#ifdef EDSBWT_KDEEP_DUMP
// diagnostic builds only (not in the header): k_deep's dumped list starts of the last launch
extern "C" int edsbwt_debug_kdeep_dump(uint32_t* out, uint32_t n) {
    if (!out) return EDSBWT_E_ARG;
    n = std::min<uint32_t>(n, edsbwt::kDumpMax * 16);
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(edsbwt::g_kdeep_dump), n * 4, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : EDSBWT_E_DEVICE;
}
#endif

int edsbwt_comm_unique_id(void* id_out, uint64_t cap) {
    if (!id_out || cap < sizeof(ncclUniqueId)) { edsbwt::g_err = "id buffer smaller than 128 bytes"; return EDSBWT_E_ARG; }
    ABI_TRY
    Rccl& R = Rccl::get();
    if (!R.ok) throw Fail(EDSBWT_E_UNSUPPORTED, "librccl.so not found");
    ncclUniqueId id;
    NCCLCHK(R.get_id(&id));
    std::memcpy(id_out, &id, sizeof id);
    return 0;
    ABI_CATCH
}

int edsbwt_comm_init(edsbwt_index* idx, const void* id, uint64_t id_bytes, int nranks, int rank) {
    if (!idx || !id || id_bytes != sizeof(ncclUniqueId) || nranks < 1 || rank < 0 || rank >= nranks) {
        edsbwt::g_err = "bad argument";
        return EDSBWT_E_ARG;
    }
    ABI_TRY
    Engine& E = *idx->eng;
    Rccl& R = Rccl::get();
    if (!R.ok) throw Fail(EDSBWT_E_UNSUPPORTED, "librccl.so not found");
    if (E.comm) throw Fail(EDSBWT_E_ARG, "the index already has a communicator");
    HIPCHK(hipSetDevice(E.device));
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    NCCLCHK(R.init(&E.comm, nranks, uid, rank));
    E.comm_rank = rank;
    E.comm_size = nranks;
    if (!E.xs) HIPCHK(hipStreamCreateWithFlags(&E.xs, hipStreamNonBlocking));
    if (!E.xs_after) HIPCHK(hipEventCreateWithFlags(&E.xs_after, hipEventDisableTiming));
    for (auto& g : E.gathers)
        if (!g.ev) HIPCHK(hipEventCreateWithFlags(&g.ev, hipEventDisableTiming));
    return 0;
    ABI_CATCH
}

int edsbwt_gather_counts(edsbwt_index* idx, const uint32_t* d_counts, uint64_t n, uint32_t* d_out, const uint64_t* sizes, int dst) {
    if (!idx || !sizes || (n && !d_counts)) { edsbwt::g_err = "null argument"; return EDSBWT_E_ARG; }
    ABI_TRY
    Engine& E = *idx->eng;
    Rccl& R = Rccl::get();
    if (!E.comm) throw Fail(EDSBWT_E_ARG, "no communicator: edsbwt_comm_init first");
    if (dst < 0 || dst >= E.comm_size) throw Fail(EDSBWT_E_ARG, "dst outside the communicator");
    if (sizes[E.comm_rank] != n) throw Fail(EDSBWT_E_ARG, "n differs from sizes[rank]");
    if (E.comm_rank == dst && !d_out) throw Fail(EDSBWT_E_ARG, "null d_out on the receiving rank");
    HIPCHK(hipSetDevice(E.device));
    // after everything queued on the search stream (the search that wrote d_counts)
    HIPCHK(hipEventRecord(E.xs_after, E.stream));
    HIPCHK(hipStreamWaitEvent(E.xs, E.xs_after, 0));
    NCCLCHK(R.group_start());
    if (E.comm_rank == dst) {
        uint64_t at = 0;
        for (int r = 0; r < E.comm_size; r++) {
            if (r == dst) {
                if (n) HIPCHK(hipMemcpyAsync(d_out + at, d_counts, n * 4, hipMemcpyDeviceToDevice, E.xs));
            } else if (sizes[r]) {
                NCCLCHK(R.recv(d_out + at, sizes[r], ncclUint32, r, E.comm, E.xs));
            }
            at += sizes[r];
        }
    } else if (n) {
        NCCLCHK(R.send(d_counts, n, ncclUint32, dst, E.comm, E.xs));
    }
    NCCLCHK(R.group_end());
    // the gather's end, for the next search that writes d_counts (wait_gathers_on)
    Engine::PendingGather* g = nullptr;
    for (auto& x : E.gathers)
        if (x.p == d_counts) g = &x;
    if (!g) g = &E.gathers[E.gather_next++ % 4];
    g->p = d_counts;
    HIPCHK(hipEventRecord(g->ev, E.xs));
    return 0;
    ABI_CATCH
}

int edsbwt_comm_sync(edsbwt_index* idx) {
    if (!idx) { edsbwt::g_err = "null argument"; return EDSBWT_E_ARG; }
    ABI_TRY
    Engine& E = *idx->eng;
    if (E.xs) HIPCHK(hipStreamSynchronize(E.xs));
    return 0;
    ABI_CATCH
}

int edsbwt_set_counts_mirror(edsbwt_index* idx, uint32_t* d_counts, uint64_t cap) {
    if (!idx) { edsbwt::g_err = "null argument"; return EDSBWT_E_ARG; }
    idx->eng->counts_mirror = cap ? d_counts : nullptr;
    idx->eng->counts_mirror_cap = d_counts ? cap : 0;
    return 0;
}

int edsbwt_last_paths(const edsbwt_index* idx, uint8_t* out, uint64_t n) {
    if (!idx || (n && !out)) { edsbwt::g_err = "null argument"; return EDSBWT_E_ARG; }
    const Engine& E = *idx->eng;
    if (!E.tag_paths || n > E.ptag_n) { edsbwt::g_err = "no path tags (EDSBWT_PATH_TAGS=1 and edsbwt_search_device first)"; return EDSBWT_E_ARG; }
    ABI_TRY
    HIPCHK(hipSetDevice(E.device));
    HIPCHK(hipStreamSynchronize(E.stream));
    if (n) HIPCHK(hipMemcpy(out, E.ptag.p, n, hipMemcpyDeviceToHost));
    return 0;
    ABI_CATCH
}

int edsbwt_last_stats(const edsbwt_index* idx, edsbwt_stats* st) {
    if (!idx || !st) { edsbwt::g_err = "null argument"; return EDSBWT_E_ARG; }
    *st = idx->eng->st;
    return 0;
}

int edsbwt_gsa(const uint8_t* codes, uint64_t n, const uint64_t* word_ends, uint64_t n_words, uint32_t bits, int device,
               uint32_t* sa, double* ms) {
    if ((n && (!codes || !word_ends || !sa))) { edsbwt::g_err = "null argument"; return EDSBWT_E_ARG; }
    ABI_TRY
    edsbwt::gsa_sort(codes, n, word_ends, n_words, bits, device, sa, ms);
    return 0;
    ABI_CATCH
}

}  // extern "C"
