/*
 * include/edsbwt.h — C ABI of the MI355X-native EDS-BWT backward-search engine.
 *
 * Drop-in boundary for riccardo-nozza/EDS-BWT's MOVE_EDSBWTSearch path.  The
 * reference has no FFI: its boundary is the process `MOVE_EDSBWTSearch <base>
 * <patterns>` (mainMove_EDSBWT.cpp:17-62) and, inside it, the class
 * MOVE_EDSBWT (MOVE_EDSBWTSearch.hpp:54-136).  Each entry point below names the
 * reference interface it replaces.  Plain pointers and sizes only.
 *
 * Conventions: 0 on success, a negative EDSBWT_E_* code on failure (never exit());
 * the message is in edsbwt_last_error() (thread-local).  One index per device;
 * calls on distinct handles are thread-safe, calls on one handle are serialized
 * by the caller.
 */
#ifndef EDSBWT_H
#define EDSBWT_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EDSBWT_ABI_VERSION 7

enum {
    EDSBWT_OK = 0,
    EDSBWT_E_IO = -1,          /* cannot open / short read of an index file */
    EDSBWT_E_FORMAT = -2,      /* index file contents inconsistent */
    EDSBWT_E_UNSUPPORTED = -3, /* e.g. alphabet larger than the device layout supports */
    EDSBWT_E_DEVICE = -4,      /* HIP runtime error */
    EDSBWT_E_ARG = -5,         /* bad argument */
    EDSBWT_E_NOMEM = -6        /* host or device allocation failed */
};

/* search flags */
#define EDSBWT_COUNT_ONLY   0x1u /* counts only; RECOVERBW=0 of the legacy engine (README.md:42-45) */
#define EDSBWT_LOCATE       0x2u /* counts + occurrence records (MOVE engine default, MOVE_EDSBWTSearch.cpp:328-369) */
#define EDSBWT_LOCATE_TABLE 0x4u /* with LOCATE: read (word, offset) from the per-row table
                                    instead of walking LF to '#'; identical records */
#define EDSBWT_PROFILE      0x8u /* record per-kernel HIP-event times into edsbwt_stats */
#define EDSBWT_NO_DEEP      0x10u/* level-synchronous trie walk for every depth (no per-pattern
                                    finishing kernel); same results, used by tests */
#define EDSBWT_PROFILE_LIGHT 0x40u/* events only around the few large launches (fused step, deep,
                                    locate, link sort): what bench.py uses inside its timed region */
#define EDSBWT_NO_WIDE      0x80u/* tests: skip the wide-list retry of k_deep overflows */
#define EDSBWT_LEGACY_ORDER 0x200u/* with LOCATE: records in the legacy EDSBWTsearch engine's order
                                    (findMultipleDollarsBackward, EDSBWTsearch.cpp:300-610): per
                                    pattern by offset, then by the word's '#' row — the order of
                                    <patterns>output.csv and of the README example */
#define EDSBWT_LOCATE_WALK  0x100u/* with LOCATE: walk LF all the way to the '#' row as the
                                    reference does (:348-353), ignoring the row samples;
                                    identical records (default: stop at the first sampled row) */
#define EDSBWT_ORDERED      0x20u/* keep every interval list in the reference's order at every
                                    depth (the path patterns holding '#' take); same results */
#define EDSBWT_NO_KTAB      0x400u/* start the trie walk at depth 0 instead of at the k-mer start
                                    table's depth (tests: same results either way) */
#define EDSBWT_NO_DIRECT    0x800u/* build the reversed-pattern trie even when every pattern could
                                    start straight from its k-mer table list (tests: same results) */
#define EDSBWT_NO_PAIRS     0x1000u/* deep walk one character per rank line instead of two from the
                                    pair blocks (sigma <= 5; tests: same results) */
#define EDSBWT_NO_TEXT      0x2000u/* step single-row intervals through the rank entries instead of
                                    comparing the pattern with the words' text (tests: same results) */
#define EDSBWT_NO_COUNTERS  0x4000u/* the direct start's deep kernels without their per-lane work
                                    counters (steps, lines, text rows): the same results, those
                                    statistics read 0 for them, and the kernels run with fewer
                                    registers (C3: k_deep_direct 0.816 against 0.850 ms).  Only the
                                    default builds have counter-free instantiations — k_deep_direct
                                    at 8 waves per SIMD and k_deep<4 intervals> at 5 or 6 waves;
                                    the builds chosen by EDSBWT_DIRECT_WAVES < 8, EDSBWT_DEEPQ_WAVES=1,
                                    EDSBWT_EOF_ROWS=1 or EDSBWT_DEEP_K != 4 keep their counters */

typedef struct edsbwt_index edsbwt_index;

/* One output row of <patterns>output_M_LF.csv (MOVE_EDSBWTSearch.cpp:365):
 * #Pat, $_i (word id), D[i] (1-based segment), S_j (word in segment), S_j[r] (offset). */
typedef struct {
    uint32_t pat, word, seg, word_in_seg, offset;
} edsbwt_occ;

/* Loaded-index facts (recoverInfo, MOVE_EDSBWTSearch.cpp:628-770). */
typedef struct {
    uint64_t n_rows;      /* lengthTot_plus_eof */
    uint64_t n_words;     /* nText */
    uint64_t n_segments;  /* ones in <base>.bitvector */
    uint32_t sigma;       /* sizeAlpha */
    uint8_t alphabet[16]; /* alphaInverse[0..sigma) */
    uint64_t device_bytes;/* HBM held by the index */
    uint32_t ktab_depth;  /* k-mer start table: depth D (0 = none) — the interval lists of
                             every D-mer over the non-'#' symbols, built at open */
    uint32_t pair_blocks; /* 1 when the two-step rank blocks are built (sigma <= 5) */
    uint64_t ktab_items;  /* intervals held by that table */
    uint32_t ltab_depth;  /* deep level start table (C5-like indexes): its depth L, 0 = none */
    uint32_t ltab_groups; /* ... kept in groups by the L-mer's last characters */
    uint64_t ltab_items;  /* intervals held by it */
    uint64_t open_peak_bytes; /* most device memory the engine held at once while opening (tables +
                                 their builds' transient workspace): the per-rank HBM a deployment
                                 that opens several indexes on one GPU must leave for each open */
    double open_seconds;      /* wall time of edsbwt_index_open */
} edsbwt_index_info;

/* Per-call counters and timings (filled by every edsbwt_search*). */
typedef struct {
    uint64_t patterns, found, not_found, occurrences;
    uint64_t depths;          /* trie depths processed */
    uint64_t trie_nodes;      /* Σ nodes over depths */
    uint64_t intervals_stepped;/* backward_search_step work items (each = 2 rank queries) */
    uint64_t link_hash_rows;  /* '#' rows read by link (dollars_in_interval) */
    uint64_t link_ranges;     /* merged previous-segment ranges produced by link */
    uint64_t locate_lf_steps; /* LF steps of the locate walk (0 with LOCATE_TABLE) */
    uint64_t deep_from_depth; /* depth at which patterns were finished one per thread (0: never) */
    uint64_t deep_overflow;   /* patterns whose lists outgrew k_deep's registers (retried with wide lists) */
    uint64_t deep_level_rerun;/* of those, patterns re-run by the level path (lists beyond the wide limit) */
    double ms_total;          /* device time of the call (hipEvent) */
    double ms_kernel[16];     /* EDSBWT_PROFILE: per kernel class, see edsbwt_kernel_name */
    uint64_t launches_kernel[16];
    uint64_t bytes_kernel[16];/* algorithmic bytes per kernel class */
    uint64_t lines_kernel[16];/* occ-block lines the kernels actually read (a narrow interval's two
                                 ends share one line; the locate table reads none) */
    uint64_t locate_offsets;  /* sum of the records' offsets = the LF moves of the reference's
                                 locate walk (:348-353), whatever walk the device did */
    uint64_t search_groups;   /* 0, or the number of trie-subtree groups the batch was split into
                                 because a depth outgrew 32-bit counts */
    uint64_t start_depth;     /* depth the trie walk started from (the k-mer start table's
                                 depth when it served the batch, else 0) */
    /* host-memory calls (edsbwt_search, edsbwt_search_lines): the pipeline */
    double ms_wall;           /* host wall time of the call: first H2D of the patterns to the last
                                 D2H of counts and records (SURVEY.md §8(d)'s patterns/s clock) */
    uint64_t chunks;          /* chunks the batch was cut into (uploads overlap searches) */
    uint64_t bytes_h2d, bytes_d2h;
    uint64_t text_chars;      /* pattern characters decided by the single-row text compare */
    uint64_t text_rows;       /* single-row intervals the text compare met */
    uint64_t redo_searches;   /* searches (chunks) run again on the checked path because a
                                 deferred check failed ('#' in a pattern, long overflow lists,
                                 more records than the pre-sized buffers) */
} edsbwt_stats;

/* Replaces recoverInfo + retrieve_MLF + bitvector load (MOVE_EDSBWTSearch.cpp:23-95,
 * 178-218, 628-770) and build_MLF (build_MLF.cpp:53-164): reads <base>_info.aux,
 * <base>.ebwt (or the _bwt_<j>.aux piles) and <base>.bitvector, builds the device
 * rank/LF table and segment tables on `device`.  a_balance is the build_MLF `a`
 * parameter (kept for CLI compatibility; the device LF table does not need it). */
int edsbwt_index_open(const char* base, int device, uint32_t a_balance, edsbwt_index** out);
void edsbwt_index_close(edsbwt_index* idx);

/* GPUs this process sees (0 when none).  The reference's pattern loop (MOVE_EDSBWTSearch.cpp:
 * 111-136) is a sequence of independent searches over one read-only index, so N devices take
 * contiguous line ranges of the pattern file, one index each (EDSBWTsearch --gpus N; SURVEY.md
 * §5 / §8(e)); this is how a host program sizes N. */
int edsbwt_device_count(void);
int edsbwt_index_get_info(const edsbwt_index* idx, edsbwt_index_info* info);

/* Replaces the pattern loop + backwardSearch (MOVE_EDSBWTSearch.cpp:97-155, 228-374).
 * Patterns are pat_bytes[pat_offsets[i] .. pat_offsets[i+1]) (host memory, no
 * terminator), i < npat; pattern i is reported as #Pat = first_pattern_id + i.
 * counts[npat] (caller-owned) receives backwardSearch's return value per pattern.
 * With EDSBWT_LOCATE, *occ (library-owned, page-locked; give it back with
 * edsbwt_occ_free) receives *nocc records in reference order: pattern-major, then
 * interval order, rows ascending — the order of <patterns>output_M_LF.csv.
 * A batch of more than EDSBWT_CHUNK_SINGLE_MB (default 24 MB) of pattern bytes is cut into
 * chunks (EDSBWT_CHUNK_MB, default 40 MB): uploads, searches and downloads of consecutive
 * chunks overlap (two SDMA engines and the index's stream).
 * Host buffers from edsbwt_host_alloc (page-locked) are transferred directly;
 * pageable ones are staged through page-locked buffers. */
int edsbwt_search(edsbwt_index* idx, const char* pat_bytes, const uint64_t* pat_offsets,
                  uint64_t npat, uint32_t first_pattern_id, uint32_t flags,
                  uint32_t* counts, edsbwt_occ** occ, uint64_t* nocc);

/* The same over a pattern file as it lies in memory (the reference's input,
 * MOVE_EDSBWTSearch.cpp:100-111): text[0..len) is split into lines with std::getline
 * semantics (at '\n'; '\r' is kept; a last line without '\n' counts).  The lines go
 * to the device as they are and are split there.  counts[counts_cap] receives one count
 * per line (E_ARG if the file has more lines); *npat = lines. */
int edsbwt_search_lines(edsbwt_index* idx, const char* text, uint64_t len, uint32_t first_pattern_id,
                        uint32_t flags, uint32_t* counts, uint64_t counts_cap, uint64_t* npat,
                        edsbwt_occ** occ, uint64_t* nocc);
void edsbwt_occ_free(edsbwt_occ* occ);

/* Page-locked host memory for pattern buffers and counts (transferred at full PCIe rate). */
int edsbwt_host_alloc(uint64_t bytes, void** out);
void edsbwt_host_free(void* p);

/* Hash of the sources the library was built from (eds-bwt_amd/Makefile): callers compare it
 * with the sources in their tree to refuse a stale binary. */
const char* edsbwt_build_id(void);

/* Device-resident variant (benchmarks, multi-GPU shards): d_bytes / d_offsets /
 * d_counts are device pointers on the index's device; occurrence records stay in
 * a library-owned device buffer returned through *d_occ (valid until the next
 * call on this index).  `stream` is a hipStream_t (NULL = the index's stream). */
int edsbwt_search_device(edsbwt_index* idx, const uint8_t* d_bytes, const uint64_t* d_offsets,
                         uint64_t npat, uint32_t first_pattern_id, uint32_t flags,
                         uint32_t* d_counts, edsbwt_occ** d_occ, uint64_t* nocc, void* stream);

/* The same over a batch that is a subset of the pattern file in another order: pattern i is
 * reported as #Pat = d_ids[i] (device array of npat ids) instead of first_pattern_id + i; counts
 * and records follow the batch's order.  The reference's loop searches and locates each line on
 * its own (MOVE_EDSBWTSearch.cpp:111-136, 328-369), so the lines can be batched in any order: a
 * located search too large for HBM is cut into batches of patterns sharing their last characters
 * (one subtree of the reversed-pattern trie each, so no two batches walk the same trie nodes)
 * instead of contiguous line ranges.  E_ARG with EDSBWT_LEGACY_ORDER. */
int edsbwt_search_device_ids(edsbwt_index* idx, const uint8_t* d_bytes, const uint64_t* d_offsets,
                             uint64_t npat, const uint32_t* d_ids, uint32_t flags,
                             uint32_t* d_counts, edsbwt_occ** d_occ, uint64_t* nocc, void* stream);

/* Tests: the kernels each pattern of the last edsbwt_search_device call went through, when the
 * process runs with EDSBWT_PATH_TAGS=1 (else E_ARG): out[i] for pattern i, i < n (n <= that
 * call's npat), bits EDSBWT_PATH_*.  Lets parity tests add every pattern of a rare path
 * (register-list walk, wide lists, level re-run, a searched-again batch) to their oracle sample. */
#define EDSBWT_PATH_DEEP   0x1u /* queued for k_deep (a list or a link, MOVE_EDSBWTSearch.cpp:258,512-563) */
#define EDSBWT_PATH_WIDE   0x2u /* list outgrew k_deep's registers: k_deep_wide */
#define EDSBWT_PATH_LEVELS 0x4u /* ... and the wide lists: re-run on the level-synchronous path */
#define EDSBWT_PATH_REDO   0x8u /* the batch failed a deferred check and was searched again */
int edsbwt_last_paths(const edsbwt_index* idx, uint8_t* out, uint64_t n);

/* Multi-GPU exchange: later edsbwt_search / edsbwt_search_lines calls on this
 * index also write every pattern's count (u32, pattern i at d_counts[i]) into d_counts, a device
 * array of cap entries on the index's device, complete when the call returns — the counts RCCL
 * gathers to rank 0 without a second upload; every host-pipeline path fills it.  cap = 0 or
 * d_counts = NULL turns it off.  A batch larger than cap fails with E_ARG: an edsbwt_search batch
 * before any chunk is searched (the mirror is untouched); an edsbwt_search_lines batch, whose
 * line count is known chunk by chunk, before the first chunk that would overflow it (the
 * mirror then holds the earlier chunks' counts). */
int edsbwt_set_counts_mirror(edsbwt_index* idx, uint32_t* d_counts, uint64_t cap);

/* Native RCCL exchange (ABI 7): the per-step gather of every rank's per-pattern
 * counts to one rank over RCCL/xGMI, issued by the library on its own exchange stream — no Python
 * and no host wait on the search's thread.  One process per GPU, one index per process:
 *   rank 0: edsbwt_comm_unique_id(id, 128); broadcast the 128 bytes to the other ranks (any channel);
 *   every rank: edsbwt_comm_init(idx, id, 128, nranks, rank) — an RCCL communicator on the index's
 *   device (librccl.so is loaded on first use; E_UNSUPPORTED without it).
 * edsbwt_gather_counts(idx, d_counts, n, d_out, sizes, dst): after the work already queued on the
 * index's stream (the search that wrote d_counts), rank `dst` receives every rank's counts into
 * d_out in rank order (rank r's n_r = sizes[r] counts at offset sizes[0] + .. + sizes[r-1]; d_out is
 * ignored elsewhere); this rank's n must equal sizes[rank].  Returns once the gather is queued; the
 * library orders any later search that writes d_counts (or a counts mirror at d_counts) after the
 * gather that reads it, so callers alternate two count buffers and the gather of step i overlaps
 * step i + 1.  edsbwt_comm_sync waits (host) until every queued gather is done.  The
 * communicator is destroyed with the index.  (Replaces the reference's single-process output
 * loop, MOVE_EDSBWTSearch.cpp:111-136, gathered in file order.) */
int edsbwt_comm_unique_id(void* id_out, uint64_t cap);
int edsbwt_comm_init(edsbwt_index* idx, const void* id, uint64_t id_bytes, int nranks, int rank);
int edsbwt_gather_counts(edsbwt_index* idx, const uint32_t* d_counts, uint64_t n, uint32_t* d_out, const uint64_t* sizes, int dst);
int edsbwt_comm_sync(edsbwt_index* idx);

/* Setup for a following edsbwt_search_lines of ~text_bytes bytes in npat lines (flags as that
 * call's): the host pipeline's threads, streams and copy engines, every slot's page-locked and
 * device buffers at the batch's chunk sizes, a chunk's search workspace, and (EDSBWT_LOCATE) the
 * page-locked record arena for records_hint records (0: 1.25 per line) — by one pass of the pipeline
 * over synthetic lines of the batch's mean length (nothing of the caller's batch is read).  The
 * work the reference does before its clock (index load, MOVE_EDSBWTSearch.cpp:23-95; clock at
 * :109), so the EDSBWTsearch CLI's "bs took:" times the steady-state pattern loop.  Optional. */
int edsbwt_prepare(edsbwt_index* idx, uint64_t text_bytes, uint64_t npat, uint64_t records_hint, uint32_t flags);

/* Counters/timings of the last search on this index. */
int edsbwt_last_stats(const edsbwt_index* idx, edsbwt_stats* st);
const char* edsbwt_kernel_name(int k);

/* Format records as the reference CSV body (no header), one row per record:
 * "%u\t%u\t%u\t%u\t%u\n" (MOVE_EDSBWTSearch.cpp:365).  Returns bytes written, or
 * the size needed when buf is NULL.  Multi-threaded. */
uint64_t edsbwt_format_csv(const edsbwt_occ* occ, uint64_t nocc, char* buf, uint64_t cap, int threads);

/* The same rows written to file descriptor fd at byte offset `at` (pwrite, several threads, no
 * buffer of the whole CSV): the EDSBWTsearch CLI's <patterns>output_M_LF.csv body after its
 * header (MOVE_EDSBWTSearch.cpp:55-64,365).  Returns the bytes written, or -1 with errno set. */
int64_t edsbwt_write_csv(const edsbwt_occ* occ, uint64_t nocc, int fd, uint64_t at, int threads);

const char* edsbwt_last_error(void);

/* Index writer support (eds_transform --gpu; replaces gsufsort's suffix sort, EDS-BWTransform.sh:26
 * and gsufsort --da over eds_to_fasta's output): the generalized suffix array of the words'
 * texts, each word followed by its terminator.  codes[n]: symbol codes, the terminator '#' = 0
 * and the other symbols 1..2^bits-1 in byte order; word_ends[n_words]: positions of the
 * terminators, ascending, the last one n-1.  sa[n] receives the text positions in suffix
 * order: suffixes compared up to and including their word's terminator, equal ones by
 * position.  *ms (optional): device time including the transfers. */
int edsbwt_gsa(const uint8_t* codes, uint64_t n, const uint64_t* word_ends, uint64_t n_words, uint32_t bits, int device,
               uint32_t* sa, double* ms);
int edsbwt_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
