/*
 * oracle/edsbwt_oracle.h — TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of riccardo-nozza/EDS-BWT's MOVE_EDSBWTSearch hot path and of
 * the index-construction chain that feeds it.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library.  The product
 * (eds-bwt_amd/, libedsbwt.so) never links or calls it.
 *
 * Parity pins (see DESIGN.md "Oracle"):
 *   - README.md:144-167 known-answer test (7 rows, multiset; legacy order) —
 *     reproduced by tests/test_oracle.py.
 *   - an independent brute-force EDS matcher (tests/brute.py) over random EDSs.
 *   - Move-r (un-vendored submodule, .gitmodules:1-3, commit not recorded) is
 *     restated from its published move-structure definition; no reference test
 *     pins its outputs, so the M_LF *layout* is unpinned.  The search result is
 *     provably independent of the M_LF interval split.
 *   - The prebuilt legacy binary inside the reference is never run.
 */
#ifndef EDSBWT_ORACLE_H
#define EDSBWT_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_engine orc_engine;

typedef struct {
    uint32_t pat, word, seg, word_in_seg, offset;
} orc_occ;

typedef struct {
    uint64_t interval_steps;  /* updateSingleInterval calls (number_updates, MOVE_EDSBWTSearch.cpp:392) */
    uint64_t step_moves;      /* M_LF.move calls inside updateSingleInterval (:460,:476,:492,:494) */
    uint64_t locate_moves;    /* M_LF.move calls inside the locate walk (:349) */
    uint64_t pdf_calls;       /* preceding_dollars_finder calls (:544) */
    uint64_t eof_reads;       /* EOF_ID_Copy reads inside dollars_in_interval (:617) */
    uint64_t occurrences;     /* rows emitted by locate (:336) */
    uint64_t found, not_found;/* count_found / count_not_found (:123,:128) */
} orc_counters;

const char* orc_last_error(void);

/* EDS-BWTransform.sh chain (eds_to_fasta + gsufsort + da_to_everything):
 * writes <base>.bitvector, .ebwt, _info.aux, _bwt_<j>.aux, _runs.aux, _runs.txt.
 * Naive suffix sort: small inputs only (tests). */
int orc_transform(const char* eds_path, const char* base);

/* recoverInfo + retrieve_MLF (rebuilt from _runs.txt/_runs.aux as build_MLF.cpp does
 * when from_runs_files != 0, else from .ebwt — identical M_LF) + bitvector load. */
orc_engine* orc_open(const char* base, uint32_t a_balance, int from_runs_files);
void orc_close(orc_engine*);

/* engine facts for tests */
uint32_t orc_n(const orc_engine*);
uint32_t orc_words(const orc_engine*);
uint32_t orc_r_prime(const orc_engine*);
uint32_t orc_runs(const orc_engine*);
int orc_last_run_split(const orc_engine*);
/* copy the M_LF arrays out (p: r'+1, q, idx: r', L: r') */
void orc_mlf_arrays(const orc_engine*, uint32_t* p, uint32_t* q, uint32_t* idx, uint8_t* L);

/* The pattern loop of MOVE_EDSBWT::MOVE_EDSBWT (MOVE_EDSBWTSearch.cpp:97-155) over an
 * in-memory batch: counts[i] = backwardSearch(...) result, occurrences in reference
 * row order (pattern-major).  threads>1 shards contiguous pattern ranges. */
int orc_search_batch(orc_engine*, const char* bytes, const uint64_t* offsets, uint64_t npat,
                     uint32_t first_pattern_id, int threads, uint32_t* counts,
                     orc_occ** occ, uint64_t* nocc, orc_counters* ctr);
/* The same batch searched with the reversed-suffix trie shared (sorted by reversed
 * pattern, each thread a contiguous range of that order): identical counts and records
 * (pattern-major, pattern order); counters count each distinct suffix once. */
int orc_search_batch_trie(orc_engine*, const char* bytes, const uint64_t* offsets, uint64_t npat,
                          uint32_t first_pattern_id, int threads, uint32_t* counts,
                          orc_occ** occ, uint64_t* nocc, orc_counters* ctr);
void orc_free(void* p);
/* The literal loop (orc_search_batch, one thread per contiguous range) also reporting, per
 * pattern, whether backwardSearch returned before its locate loop (early[i] = 1: the
 * `return 0` of MOVE_EDSBWTSearch.cpp:250-253 / :295-297, so no "num occ" line, :371): the
 * per-pattern console stream of the reference is a function of (pattern, count, early). */
int orc_search_batch_console(orc_engine*, const char* bytes, const uint64_t* offsets, uint64_t npat,
                             uint32_t first_pattern_id, int threads, uint32_t* counts, uint8_t* early);

/* Same loop over a pattern file (getline semantics), writing <out_csv>
 * byte-for-byte as MOVE_EDSBWTSearch.cpp:55-64,365 does. limit=0 → all lines. */
int orc_search_file(orc_engine*, const char* patterns_path, const char* out_csv,
                    uint64_t limit, int threads, orc_counters* ctr, double* seconds);

/* Record checker, independent of any BWT: counts records whose (word, seg, word_in_seg,
 * offset) disagree with the .eds segmentation or from which the pattern cannot be spelled
 * (continuing into any word of the next segment; segments holding the empty word may be
 * skipped).  *first_bad = index of the first bad record (~0 if none). */
int orc_check_records(const char* eds_path, const char* bytes, const uint64_t* offsets, uint64_t npat,
                      uint32_t first_pattern_id, const orc_occ* rec, uint64_t nocc, int threads,
                      uint64_t* bad, uint64_t* first_bad);

#ifdef __cplusplus
}
#endif
#endif
