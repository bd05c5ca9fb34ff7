/*
 * oracle/edsbwt_oracle.c — TEST INFRASTRUCTURE ONLY (checker + CPU baseline).
 *
 * A plain-C restatement of the reference's MOVE_EDSBWTSearch path
 * (riccardo-nozza/EDS-BWT) and of the index chain that feeds it.  Every function
 * names the reference file:line it follows.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product never does.
 *
 *   parse            eds_to_fasta.cpp:55-153
 *   gsa / ebwt       gsufsort --da --bwt (EDS-BWTransform.sh:26, external, absent):
 *                    suffixes of word·'#' sorted, ties by word id; then
 *                    remove_empty_symbols da_to_everything.cpp:371-486
 *   freq / alphabet  da_to_everything.cpp:301-366
 *   info / piles     da_to_everything.cpp:113-290
 *   runs LF pairs    da_to_everything.cpp:62-109 (build_ilf)
 *   M_LF             build_MLF.cpp:53-164 + Move-r move_data_structure_l_
 *                    (a-balanced move structure; restated, version unpinned)
 *   recoverInfo      MOVE_EDSBWTSearch.cpp:628-770
 *   retrieve_MLF     MOVE_EDSBWTSearch.cpp:178-218
 *   backwardSearch   MOVE_EDSBWTSearch.cpp:228-374
 *   step / update    MOVE_EDSBWTSearch.cpp:376-510
 *   link & helpers   MOVE_EDSBWTSearch.cpp:512-625
 *   pattern loop/CSV MOVE_EDSBWTSearch.cpp:55-64,97-155,365
 *
 * The `.bitvector` is read as an sdsl int_vector<1> (u64 bit count + u64 words).
 * numEOF[j] is taken from tableOcc[j][alpha['#']] rather than from the sdsl
 * rrr_vector files _bv_<j>.aux (equal by construction, da_to_everything.cpp:219,225).
 */
#define _GNU_SOURCE
#include "edsbwt_oracle.h"

#include <errno.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define TERM '#'      /* TERMINATE_CHAR, Parameters.h:30 */
#define EMPTYC 'Z'    /* EMPTY_CHAR, Parameters.h:34 */
#define EMPTY_EDS 'E' /* EMPTY_CHAR_EDS, Parameters.h:33 */

static __thread char g_err[512];
const char* orc_last_error(void) { return g_err; }
static int fail(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return -1;
}
void orc_free(void* p) { free(p); }

/* ------------------------------------------------------------------ vectors */
typedef struct { uint32_t b, e, bi, ei; } rng_t; /* rangeElement, Sorting.h:38-47 */
typedef struct { rng_t* v; size_t n, cap; } rvec;
typedef struct { uint32_t* v; size_t n, cap; } uvec;
typedef struct { uint8_t* v; size_t n, cap; } bvec;
typedef struct { orc_occ* v; size_t n, cap; } ovec;

#define VEC_PUSH(V, X)                                                        \
    do {                                                                      \
        if ((V)->n == (V)->cap) {                                             \
            (V)->cap = (V)->cap ? (V)->cap * 2 : 16;                          \
            (V)->v = realloc((V)->v, (V)->cap * sizeof(*(V)->v));             \
            if (!(V)->v) { fprintf(stderr, "oracle: out of memory\n"); abort(); } \
        }                                                                     \
        (V)->v[(V)->n++] = (X);                                               \
    } while (0)

static void* xmalloc(size_t n) {
    void* p = malloc(n ? n : 1);
    if (!p) { fprintf(stderr, "oracle: out of memory (%zu)\n", n); abort(); }
    return p;
}
static void* xcalloc(size_t n, size_t s) {
    void* p = calloc(n ? n : 1, s ? s : 1);
    if (!p) { fprintf(stderr, "oracle: out of memory\n"); abort(); }
    return p;
}

static int read_file(const char* path, uint8_t** buf, size_t* len) {
    FILE* f = fopen(path, "rb");
    if (!f) return fail("cannot open %s: %s", path, strerror(errno));
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    *buf = xmalloc((size_t)sz + 1);
    if (sz > 0 && fread(*buf, 1, (size_t)sz, f) != (size_t)sz) {
        fclose(f);
        free(*buf);
        return fail("short read %s", path);
    }
    (*buf)[sz] = 0;
    *len = (size_t)sz;
    fclose(f);
    return 0;
}

/* ------------------------------------------------------------ EDS parsing */
/* eds_to_fasta.cpp:55-153.  Words are concatenated into `text`, each followed by
 * '#'; the empty word is the single char 'Z' (eds_to_fasta.cpp:558-560,607-610,613-616).
 * Inputs the reference chain cannot represent consistently are rejected:
 * "{}" (zero-length record), 'E' inside a non-empty word, bytes outside ('#','Z'). */
typedef struct {
    bvec text;      /* words, '#'-terminated */
    uvec wstart;    /* text offset of each word */
    bvec bits;      /* bit per word: 1 = first word of a segment */
    uint32_t empty; /* empty_counter */
    uint32_t chars; /* chars (incl. 'Z') */
} eds_t;

static void eds_free(eds_t* E) {
    free(E->text.v);
    free(E->wstart.v);
    free(E->bits.v);
}

static int eds_parse(const uint8_t* s, size_t n, eds_t* E) {
    memset(E, 0, sizeof *E);
    if (n == 0) return fail("empty EDS");
    if (s[n - 1] != '}') return fail("ERROR: file .eds must end with }"); /* EDS-BWTransform.sh:11-14 */
    if (s[0] == EMPTYC) return fail("input contains %c", EMPTYC);     /* :544-550 */
    if (s[0] != '{') return fail("the string does not start with {"); /* :564-567 */
    int in_word = 0;
    size_t wlen = 0;
#define START_WORD(BIT)                             \
    do {                                            \
        if (in_word) {                              \
            if (wlen == 0) return fail("zero-length word ({} or ,,-less record)"); \
            VEC_PUSH(&E->text, (uint8_t)TERM);      \
        }                                           \
        VEC_PUSH(&E->wstart, (uint32_t)E->text.n);  \
        VEC_PUSH(&E->bits, (uint8_t)(BIT));         \
        in_word = 1;                                \
        wlen = 0;                                   \
    } while (0)
#define PUT(C)                                      \
    do {                                            \
        VEC_PUSH(&E->text, (uint8_t)(C));           \
        wlen++;                                     \
        E->chars++;                                 \
    } while (0)
    START_WORD(1); /* :553-557 */
    if (n > 1 && s[1] == ',') { PUT(EMPTYC); E->empty++; }
    for (size_t i = 1; i < n; i++) {
        uint8_t c = s[i];
        int next = (i + 1 < n) ? s[i + 1] : -1;
        if (c == EMPTYC) return fail("input contains %c", EMPTYC); /* :572-578 */
        if (c == '{') {                                           /* :580-594 */
            START_WORD(1);
            if (next == ',') { PUT(EMPTYC); E->empty++; }
        } else if (c == '}') {                                    /* :595-601 */
        } else if (c == ',') {                                    /* :602-612 */
            START_WORD(0);
            if (next == ',' || next == '}') { PUT(EMPTYC); E->empty++; }
        } else if (c == EMPTY_EDS) {                              /* :613-617 */
            if (wlen != 0 || !(next == ',' || next == '}'))
                return fail("'E' inside a non-empty word at byte %zu", i);
            PUT(EMPTYC);
            E->empty++;
        } else {                                                  /* :618-622 */
            if (c <= TERM || c >= EMPTYC)
                return fail("byte 0x%02x at %zu is outside the supported range ('#','Z')", c, i);
            PUT(c);
        }
    }
    if (in_word) {
        if (wlen == 0) return fail("zero-length word");
        VEC_PUSH(&E->text, (uint8_t)TERM);
    }
#undef START_WORD
#undef PUT
    return 0;
}

/* ------------------------------------------------------ suffix sorting (GSA) */
typedef struct { const uint8_t* T; const uint32_t* wid; } gsa_ctx;
/* gsufsort order: suffixes of w·'#' compared up to and including '#', '#' smallest,
 * equal suffixes ordered by word id. */
static int gsa_cmp(const void* pa, const void* pb, void* arg) {
    const gsa_ctx* G = arg;
    uint32_t a = *(const uint32_t*)pa, b = *(const uint32_t*)pb;
    const uint8_t* T = G->T;
    for (;;) {
        uint8_t ca = T[a], cb = T[b];
        if (ca == TERM && cb == TERM) return (G->wid[a] > G->wid[b]) - (G->wid[a] < G->wid[b]);
        if (ca == TERM) return -1;
        if (cb == TERM) return 1;
        if (ca != cb) return ca < cb ? -1 : 1;
        a++;
        b++;
    }
}

static int write_all(const char* path, const void* p, size_t n) {
    FILE* f = fopen(path, "wb");
    if (!f) return fail("cannot write %s", path);
    if (n && fwrite(p, 1, n, f) != n) { fclose(f); return fail("short write %s", path); }
    fclose(f);
    return 0;
}

int orc_transform(const char* eds_path, const char* base) {
    uint8_t* raw;
    size_t rawn;
    if (read_file(eds_path, &raw, &rawn)) return -1;
    eds_t E;
    int rc = eds_parse(raw, rawn, &E);
    free(raw);
    if (rc) { eds_free(&E); return -1; }
    const uint8_t* T = E.text.v;
    uint32_t tot = (uint32_t)E.text.n, W = (uint32_t)E.wstart.n;
    uint32_t* wid = xmalloc((size_t)tot * 4);
    for (uint32_t w = 0; w < W; w++) {
        uint32_t end = (w + 1 < W) ? E.wstart.v[w + 1] : tot;
        for (uint32_t t = E.wstart.v[w]; t < end; t++) wid[t] = w;
    }
    uint32_t* sa = xmalloc((size_t)tot * 4);
    for (uint32_t i = 0; i < tot; i++) sa[i] = i;
    gsa_ctx G = {T, wid};
    if (tot > 1) qsort_r(sa, tot, 4, gsa_cmp, &G);

    /* .bwt + .4.da → remove_empty_symbols (da_to_everything.cpp:371-486) */
    uint32_t N = tot - E.empty; /* toKeep */
    for (uint32_t i = N; i < tot; i++)
        if (T[sa[i]] != EMPTYC) { free(wid); free(sa); eds_free(&E); return fail("Z suffixes are not last"); }
    uint8_t* rawL = xmalloc(N ? N : 1);
    uint32_t* da = xmalloc((size_t)(N ? N : 1) * 4);
    for (uint32_t i = 0; i < N; i++) {
        uint32_t t = sa[i];
        int word_start = (t == E.wstart.v[wid[t]]);
        rawL[i] = word_start ? TERM : T[t - 1];
        da[i] = wid[t];
    }
    char path[4096];
    /* _runs.aux (da_to_everything.cpp:414-443) and .ebwt (:447-456) */
    snprintf(path, sizeof path, "%s_runs.aux", base);
    FILE* fr = fopen(path, "wb");
    uint8_t* L = xmalloc(N ? N : 1);
    uint8_t prev = TERM;
    uint32_t freq[256] = {0};
    for (uint32_t i = 0; i < N; i++) {
        uint8_t c = rawL[i];
        if (prev != c || c == EMPTYC || c == TERM) fprintf(fr, "%d,%c\n", (int)i, c);
        prev = c;
        L[i] = (c == EMPTYC) ? TERM : c;
        freq[L[i]]++;
    }
    fclose(fr);
    snprintf(path, sizeof path, "%s.ebwt", base);
    if (write_all(path, L, N)) goto err;
    /* buildFreq (da_to_everything.cpp:301-366) */
    if (freq[TERM] != W) { fail("ERROR: The end-marker must be #"); goto err; }
    int alpha[256];
    uint8_t ainv[256];
    uint32_t sigma = 0;
    memset(alpha, 0, sizeof alpha); /* global zero-init in the reference: alpha['Z'] == 0 */
    for (int c = 0; c < 256; c++)
        if (freq[c]) { alpha[c] = (int)sigma; ainv[sigma++] = (uint8_t)c; }
    /* da_to_everything (da_to_everything.cpp:113-290) */
    uint32_t* tocc = xcalloc((size_t)sigma * sigma, 4);
    snprintf(path, sizeof path, "%s_info.aux", base);
    FILE* fi = fopen(path, "wb");
    fwrite(&N, 4, 1, fi);
    fwrite(&freq[ainv[0]], 4, 1, fi);
    uint8_t s8 = (uint8_t)sigma;
    fwrite(&s8, 1, 1, fi);
    fwrite(ainv, 1, sigma, fi);
    uint32_t row = 0;
    for (uint32_t j = 0; j < sigma; j++) {
        uint32_t pile = freq[ainv[j]];
        snprintf(path, sizeof path, "%s_bwt_%u.aux", base, j);
        if (write_all(path, L + row, pile)) { fclose(fi); free(tocc); goto err; }
        for (uint32_t k = 0; k < pile; k++, row++) {
            if (L[row] == TERM) fwrite(&da[row], 4, 1, fi);
            tocc[j * sigma + alpha[L[row]]]++;
        }
    }
    fwrite(tocc, 4, (size_t)sigma * sigma, fi);
    fclose(fi);
    /* build_ilf → _runs.txt (da_to_everything.cpp:62-109) */
    {
        uint32_t* sp = xcalloc(sigma, 4);
        for (uint32_t j = 0; j + 1 < sigma; j++) {
            sp[j + 1] = sp[j];
            for (uint32_t h = 0; h < sigma; h++) sp[j + 1] += tocc[j * sigma + h];
        }
        snprintf(path, sizeof path, "%s_runs.txt", base);
        FILE* ft = fopen(path, "wb");
        int have = 0;
        uint32_t ip = 0;
        uint8_t let = 0;
        prev = TERM;
        for (uint32_t i = 0; i < N; i++) {
            uint8_t c = rawL[i];
            int head = (prev != c || c == EMPTYC || c == TERM);
            prev = c;
            if (!head) continue;
            if (have) {
                sp[alpha[let]] += i - ip;
            }
            ip = i;
            let = c;
            have = 1;
            fprintf(ft, "%d,%d\n", (int)ip, (int)sp[alpha[let]]);
        }
        fclose(ft);
        free(sp);
    }
    /* .bitvector (eds_to_fasta.cpp:151-153): sdsl int_vector<1> */
    {
        uint64_t nb = W, nwords = (nb + 63) / 64;
        uint64_t* words = xcalloc(nwords ? nwords : 1, 8);
        for (uint32_t w = 0; w < W; w++)
            if (E.bits.v[w]) words[w >> 6] |= 1ull << (w & 63);
        snprintf(path, sizeof path, "%s.bitvector", base);
        FILE* fb = fopen(path, "wb");
        fwrite(&nb, 8, 1, fb);
        fwrite(words, 8, nwords, fb);
        fclose(fb);
        free(words);
    }
    free(tocc);
    free(L); free(rawL); free(da); free(wid); free(sa); eds_free(&E);
    return 0;
err:
    free(L); free(rawL); free(da); free(wid); free(sa); eds_free(&E);
    return -1;
}

/* ------------------------------------------------- rank/select supports */
/* Move-r rank_select_support<char,u32> over L' (MOVE_EDSBWTSearch.hpp:47) and over
 * the segment bitvector (MOVE_EDSBWTSearch.cpp:81-86): rank(c,i) = #c in [0,i),
 * select(c,k) = index of the k-th c (1-based), frequency(c), contains(c). */
typedef struct {
    uint32_t n, K;         /* length, number of distinct symbols */
    int code[256];         /* byte → code or -1 */
    uint32_t* cnt;         /* per 64-block × K cumulative counts */
    uint64_t* mask;        /* per 64-block × K membership masks */
    uint32_t** pos;        /* per code: sorted positions */
    uint32_t* freq;        /* per code */
} rsl_t;

static void rsl_build(rsl_t* R, const uint8_t* s, uint32_t n) {
    memset(R, 0, sizeof *R);
    R->n = n;
    for (int c = 0; c < 256; c++) R->code[c] = -1;
    for (uint32_t i = 0; i < n; i++)
        if (R->code[s[i]] < 0) R->code[s[i]] = (int)R->K++;
    uint32_t K = R->K ? R->K : 1, nb = n / 64 + 1;
    R->cnt = xcalloc((size_t)nb * K, 4);
    R->mask = xcalloc((size_t)nb * K, 8);
    R->freq = xcalloc(K, 4);
    uint32_t* run = xcalloc(K, 4);
    for (uint32_t i = 0; i < n; i++) {
        if ((i & 63) == 0) memcpy(R->cnt + (size_t)(i >> 6) * K, run, K * 4);
        int c = R->code[s[i]];
        R->mask[(size_t)(i >> 6) * K + c] |= 1ull << (i & 63);
        run[c]++;
    }
    if ((n & 63) == 0) memcpy(R->cnt + (size_t)(n >> 6) * K, run, K * 4);
    R->pos = xcalloc(K, sizeof(uint32_t*));
    for (uint32_t c = 0; c < K; c++) { R->freq[c] = run[c]; R->pos[c] = xmalloc((size_t)run[c] * 4 + 4); run[c] = 0; }
    for (uint32_t i = 0; i < n; i++) { int c = R->code[s[i]]; R->pos[c][run[c]++] = i; }
    free(run);
}
static void rsl_free(rsl_t* R) {
    for (uint32_t c = 0; c < R->K; c++) free(R->pos[c]);
    free(R->pos); free(R->cnt); free(R->mask); free(R->freq);
}
static inline int rsl_contains(const rsl_t* R, uint8_t c) { return R->code[c] >= 0; }
static inline uint32_t rsl_freq(const rsl_t* R, uint8_t c) { int k = R->code[c]; return k < 0 ? 0 : R->freq[k]; }
static inline uint32_t rsl_rank(const rsl_t* R, uint8_t c, uint32_t i) {
    int k = R->code[c];
    if (k < 0) return 0;
    size_t blk = (size_t)(i >> 6) * R->K + (uint32_t)k;
    uint32_t off = i & 63;
    uint64_t m = off ? (R->mask[blk] & ((1ull << off) - 1)) : 0;
    return R->cnt[blk] + (uint32_t)__builtin_popcountll(m);
}
/* returns 0 and sets *ok=0 when out of range (Move-r's optional → the
 * bad_optional_access catch of MOVE_EDSBWTSearch.cpp:502-507) */
static inline uint32_t rsl_select(const rsl_t* R, uint8_t c, uint32_t k1, int* ok) {
    int k = R->code[c];
    if (k < 0 || k1 == 0 || k1 > R->freq[k]) { *ok = 0; return 0; }
    return R->pos[k][k1 - 1];
}

/* ------------------------------------------------------------ M_LF */
/* build_MLF.cpp:53-164 with Move-r's a-balanced move_data_structure_l_:
 * input intervals [p_i, p_{i+1}), output intervals [q_i, q_i + d_i).  An output
 * interval holding >= 2a input starts is split at the (a+1)-th start it holds
 * (Nishimoto–Tabei balancing); repeated until none is heavy. */
typedef struct { uint32_t p, q; } pq_t;
/* rank directory over the input-interval starts p_i (bit per row, ones before each
 * 64-row word): number of starts <= x in O(1) instead of a binary search per query */
typedef struct { uint64_t* bits; uint32_t* pre; uint32_t n; } pstart_t;
static void pstart_build(pstart_t* R, const pq_t* v, uint32_t k, uint32_t n) {
    uint32_t nw = n / 64 + 2;
    R->n = n;
    R->bits = xcalloc(nw, 8);
    R->pre = xmalloc((size_t)nw * 4);
    for (uint32_t j = 0; j < k; j++) R->bits[v[j].p >> 6] |= 1ull << (v[j].p & 63);
    uint32_t acc = 0;
    for (uint32_t w = 0; w < nw; w++) { R->pre[w] = acc; acc += (uint32_t)__builtin_popcountll(R->bits[w]); }
}
/* number of starts < x (= lower_bound over the sorted p's) */
static inline uint32_t pstart_lb(const pstart_t* R, uint32_t x) {
    uint32_t w = x >> 6, o = x & 63;
    return R->pre[w] + (o ? (uint32_t)__builtin_popcountll(R->bits[w] & ((1ull << o) - 1)) : 0u);
}
static void pstart_free(pstart_t* R) { free(R->bits); free(R->pre); }

static void mlf_balance(pq_t** pv, uint32_t* pk, uint32_t n, uint32_t a) {
    if (a < 2) a = 2;
    pq_t* v = *pv;
    uint32_t k = *pk;
    for (;;) {
        pq_t* add = NULL;
        size_t nadd = 0, cadd = 0;
        pstart_t R;
        pstart_build(&R, v, k, n);
        for (uint32_t j = 0; j < k; j++) {
            uint32_t len = ((j + 1 < k) ? v[j + 1].p : n) - v[j].p;
            uint32_t lo = pstart_lb(&R, v[j].q);
            uint32_t hi = pstart_lb(&R, v[j].q + len);
            if (hi - lo >= 2 * a) {
                uint32_t s = v[lo + a].p;
                uint32_t d = s - v[j].q;
                if (nadd == cadd) { cadd = cadd ? cadd * 2 : 1024; add = realloc(add, cadd * sizeof(pq_t)); }
                add[nadd].p = v[j].p + d;
                add[nadd].q = s;
                nadd++;
            }
        }
        pstart_free(&R);
        if (!nadd) { free(add); break; }
        /* add[] is ascending in p (one split inside each input interval j, j ascending):
         * merge instead of re-sorting */
        pq_t* m = xmalloc((k + nadd) * sizeof(pq_t));
        size_t a0 = 0, b0 = 0, o = 0;
        while (a0 < k || b0 < nadd)
            m[o++] = (b0 == nadd || (a0 < k && v[a0].p < add[b0].p)) ? v[a0++] : add[b0++];
        free(v);
        v = m;
        k += (uint32_t)nadd;
        free(add);
    }
    *pv = v;
    *pk = k;
}

struct orc_engine {
    /* recoverInfo (MOVE_EDSBWTSearch.cpp:628-770) */
    uint32_t n, nText, sigma;
    uint8_t ainv[256];
    uint32_t* eof_id;   /* EOF_ID_Copy */
    uint32_t* tocc;
    /* M_LF */
    uint32_t r, runs;
    uint32_t *p, *q, *idx;
    uint8_t* L;
    int last_run_split;
    rsl_t rsL;          /* _RS_L_ */
    uint32_t* dollar_ii;/* M_LF_Dollar_Input_interval */
    /* bitvector */
    uint32_t bv_size;
    uint64_t* bv;
    uint32_t* bv_rank;  /* per 64-bit word: ones before */
    uint32_t* bv_sel;   /* positions of ones */
    uint32_t bv_ones;
    uint32_t first_symbol_index;
};

uint32_t orc_n(const orc_engine* E) { return E->n; }
uint32_t orc_words(const orc_engine* E) { return E->nText; }
uint32_t orc_r_prime(const orc_engine* E) { return E->r; }
uint32_t orc_runs(const orc_engine* E) { return E->runs; }
int orc_last_run_split(const orc_engine* E) { return E->last_run_split; }
void orc_mlf_arrays(const orc_engine* E, uint32_t* p, uint32_t* q, uint32_t* idx, uint8_t* L) {
    memcpy(p, E->p, (size_t)(E->r + 1) * 4);
    memcpy(q, E->q, (size_t)E->r * 4);
    memcpy(idx, E->idx, (size_t)E->r * 4);
    memcpy(L, E->L, E->r);
}

static inline uint32_t bv_rank1(const orc_engine* E, uint32_t i) {
    if (i > E->bv_size) i = E->bv_size;
    uint32_t w = i >> 6, o = i & 63;
    uint32_t r = E->bv_rank[w];
    if (o) r += (uint32_t)__builtin_popcountll(E->bv[w] & ((1ull << o) - 1));
    return r;
}
static inline uint32_t bv_select1(const orc_engine* E, uint32_t k) {
    if (k == 0 || k > E->bv_ones) return 0; /* unreachable from the search paths */
    return E->bv_sel[k - 1];
}

/* M_LF.move(x, x') — Move-r move query */
static inline void mlf_move(const orc_engine* E, uint32_t* x, uint32_t* xi) {
    uint32_t i = *xi;
    uint32_t y = E->q[i] + (*x - E->p[i]);
    uint32_t j = E->idx[i];
    while (y >= E->p[j + 1]) j++;
    *x = y;
    *xi = j;
}

static int read_exact(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n ? 0 : -1; }

/* run heads + LF(run head): from _runs.txt/_runs.aux (build_MLF.cpp:66-92,118-151)
 * or recomputed from .ebwt (same runs: every '#' and 'Z' is its own run,
 * da_to_everything.cpp:440; 'Z' and '#' both map to pile 0). */
static int load_runs(orc_engine* E, const char* base, int from_files, const uint8_t* L, uint32_t N,
                     pq_t** out, uint8_t** let_out, uint32_t* nruns) {
    size_t cap = 1024, k = 0;
    pq_t* v = xmalloc(cap * sizeof(pq_t));
    uint8_t* let = xmalloc(cap);
    if (from_files) {
        char path[4096];
        snprintf(path, sizeof path, "%s_runs.txt", base);
        FILE* ft = fopen(path, "rb");
        snprintf(path, sizeof path, "%s_runs.aux", base);
        FILE* fa = fopen(path, "rb");
        if (!ft || !fa) { if (ft) fclose(ft); if (fa) fclose(fa); free(v); free(let); return fail("cannot open runs files for %s", base); }
        unsigned lp, lf, ip;
        char c;
        while (fscanf(ft, "%u,%u\n", &lp, &lf) == 2) {
            if (fscanf(fa, "%u,%c\n", &ip, &c) != 2 || ip != lp) { fclose(ft); fclose(fa); free(v); free(let); return fail("runs files disagree"); }
            if (k == cap) { cap *= 2; v = realloc(v, cap * sizeof(pq_t)); let = realloc(let, cap); }
            v[k].p = lp; v[k].q = lf; let[k] = (uint8_t)c; k++;
        }
        fclose(ft);
        fclose(fa);
    } else {
        uint32_t C[256] = {0}, seen[256] = {0};
        uint32_t acc = 0;
        for (uint32_t j = 0; j < E->sigma; j++) { C[E->ainv[j]] = acc; for (uint32_t h = 0; h < E->sigma; h++) acc += E->tocc[j * E->sigma + h]; }
        for (uint32_t i = 0; i < N; i++) {
            uint8_t c = L[i];
            if (i == 0 || c != L[i - 1] || c == TERM) {
                if (k == cap) { cap *= 2; v = realloc(v, cap * sizeof(pq_t)); let = realloc(let, cap); }
                v[k].p = i; v[k].q = C[c] + seen[c]; let[k] = c; k++;
            }
            seen[c]++;
        }
    }
    *out = v;
    *let_out = let;
    *nruns = (uint32_t)k;
    return 0;
}

orc_engine* orc_open(const char* base, uint32_t a, int from_runs_files) {
    orc_engine* E = xcalloc(1, sizeof *E);
    char path[4096];
    /* recoverInfo (MOVE_EDSBWTSearch.cpp:628-770) */
    snprintf(path, sizeof path, "%s_info.aux", base);
    FILE* f = fopen(path, "rb");
    if (!f) { fail("Error opening %s.", path); free(E); return NULL; }
    uint8_t s8;
    if (read_exact(f, &E->n, 4) || read_exact(f, &E->nText, 4) || read_exact(f, &s8, 1)) { fclose(f); fail("Error reading header of %s", path); free(E); return NULL; }
    E->sigma = s8 ? s8 : 256;
    if (read_exact(f, E->ainv, E->sigma)) { fclose(f); fail("Error reading alphaInverse"); free(E); return NULL; }
    E->eof_id = xmalloc((size_t)E->nText * 4 + 4);
    E->tocc = xmalloc((size_t)E->sigma * E->sigma * 4);
    if (read_exact(f, E->eof_id, (size_t)E->nText * 4) || read_exact(f, E->tocc, (size_t)E->sigma * E->sigma * 4)) {
        fclose(f); fail("Error reading EOF_ID/tableOcc"); orc_close(E); return NULL;
    }
    fclose(f);
    /* .ebwt (build_MLF.cpp:55-64 reads its length; piles _bwt_<j>.aux concatenate to it) */
    uint8_t* L = NULL;
    size_t ln = 0;
    snprintf(path, sizeof path, "%s.ebwt", base);
    if (read_file(path, &L, &ln)) { orc_close(E); return NULL; }
    if (ln != E->n) { free(L); fail(".ebwt length %zu != %u", ln, E->n); orc_close(E); return NULL; }
    /* M_LF construction (build_MLF.cpp:82-149) */
    pq_t* v = NULL;
    uint8_t* let = NULL;
    uint32_t k = 0;
    if (load_runs(E, base, from_runs_files, L, E->n, &v, &let, &k)) { free(L); orc_close(E); return NULL; }
    E->runs = k;
    pq_t* heads = xmalloc((size_t)k * sizeof(pq_t));
    if (k) memcpy(heads, v, (size_t)k * sizeof(pq_t));
    mlf_balance(&v, &k, E->n, a);
    E->r = k;
    E->p = xmalloc((size_t)(k + 1) * 4);
    E->q = xmalloc((size_t)k * 4 + 4);
    E->idx = xmalloc((size_t)k * 4 + 4);
    E->L = xcalloc(k + 1, 1);
    for (uint32_t i = 0; i < k; i++) { E->p[i] = v[i].p; E->q[i] = v[i].q; }
    E->p[k] = E->n;
    {   /* idx: input interval containing q_i = (number of starts <= q_i) - 1 */
        pstart_t R;
        pstart_build(&R, v, k, E->n);
        for (uint32_t i = 0; i < k; i++) E->idx[i] = pstart_lb(&R, E->q[i] + 1) - 1;
        pstart_free(&R);
    }
    /* L' from the run letters (build_MLF.cpp:133-149): split pieces inherit `prev`;
     * pieces after the last run head are never assigned (left 0, recorded). */
    {
        uint32_t i = 0;
        uint8_t prev = 0;
        for (uint32_t h = 0; h < E->runs; h++) {
            while (E->p[i] < heads[h].p) { E->L[i] = prev; i++; }
            E->L[i] = (let[h] == EMPTYC) ? TERM : let[h];
            prev = let[h];
            i++;
        }
        E->last_run_split = (i < k);
    }
    free(heads); free(v); free(let); free(L);
    rsl_build(&E->rsL, E->L, E->r); /* _RS_L_ = rsl_t(read,0,r_) (:51-53) */
    /* M_LF_Dollar_Input_interval (:201-206 → findInputInterval :212-218) */
    E->dollar_ii = xmalloc((size_t)E->nText * 4 + 4);
    if (E->nText) E->dollar_ii[0] = 0;
    for (uint32_t i = 1; i < E->nText; i++) {
        uint32_t x = E->dollar_ii[i - 1];
        while (i >= E->p[x]) x++;
        E->dollar_ii[i] = x - 1;
    }
    /* .bitvector (:67-94) */
    snprintf(path, sizeof path, "%s.bitvector", base);
    f = fopen(path, "rb");
    uint64_t nb;
    if (!f || read_exact(f, &nb, 8)) { if (f) fclose(f); fail("Error opening \"%s\" file", path); orc_close(E); return NULL; }
    E->bv_size = (uint32_t)nb;
    uint32_t nw = (uint32_t)((nb + 63) / 64);
    E->bv = xcalloc(nw + 1, 8);
    if (read_exact(f, E->bv, (size_t)nw * 8)) { fclose(f); fail("short .bitvector"); orc_close(E); return NULL; }
    fclose(f);
    E->bv_rank = xmalloc((size_t)(nw + 1) * 4);
    uint32_t ones = 0;
    for (uint32_t w = 0; w <= nw; w++) { E->bv_rank[w] = ones; if (w < nw) ones += (uint32_t)__builtin_popcountll(E->bv[w]); }
    E->bv_ones = ones;
    E->bv_sel = xmalloc((size_t)ones * 4 + 4);
    for (uint32_t i = 0, o = 0; i < E->bv_size; i++)
        if ((E->bv[i >> 6] >> (i & 63)) & 1) E->bv_sel[o++] = i;
    /* first_symbol_index = bsel_1(2)-1 (:93-94); one segment → no linkable word */
    E->first_symbol_index = (ones >= 2) ? E->bv_sel[1] - 1 : (E->bv_size ? E->bv_size - 1 : 0);
    return E;
}

void orc_close(orc_engine* E) {
    if (!E) return;
    free(E->eof_id); free(E->tocc); free(E->p); free(E->q); free(E->idx); free(E->L);
    if (E->rsL.cnt) rsl_free(&E->rsL);
    free(E->dollar_ii); free(E->bv); free(E->bv_rank); free(E->bv_sel);
    free(E);
}

/* ------------------------------------------------------------ search */
typedef struct {
    rvec other, dollar, valid, merged;
    uvec d;
    ovec out;
    orc_counters c;
    int early; /* the last backward_search returned before locate (:250-253, :295-297) */
} ctx_t;

/* updateSingleInterval (MOVE_EDSBWTSearch.cpp:424-510) */
static int update_single(const orc_engine* E, ctx_t* X, uint8_t sym, rng_t* it) {
    uint32_t b = it->b, e = it->e, b_ = it->bi, e_ = it->ei;
    const rsl_t* R = &E->rsL;
    int ok = 1;
    if (!rsl_contains(R, sym)) return 0;
    if (sym != E->L[b_]) {
        b_ = rsl_rank(R, sym, b_);
        if (b_ == rsl_freq(R, sym)) return 0;
        b_ = rsl_select(R, sym, b_ + 1, &ok);
        if (!ok) return 0;
        if (b_ > e_) return 0;
        b = E->p[b_];
    }
    if (sym != E->L[e_]) {
        e_ = rsl_select(R, sym, rsl_rank(R, sym, e_), &ok);
        if (!ok) return 0;
        e = E->p[e_ + 1] - 1;
    }
    if (b > e) return 0;
    if (b_ == e_) {
        if (b == e) {
            mlf_move(E, &b, &b_);
            X->c.step_moves++;
            e = b;
            e_ = b_;
        } else {
            uint32_t diff = e - b;
            mlf_move(E, &b, &b_);
            X->c.step_moves++;
            e = b + diff;
            e_ = b_;
            while (e >= E->p[e_ + 1]) e_++;
        }
    } else {
        mlf_move(E, &b, &b_);
        mlf_move(E, &e, &e_);
        X->c.step_moves += 2;
    }
    it->b = b; it->e = e; it->bi = b_; it->ei = e_;
    return 1;
}

/* backward_search_step (:376-422): false only when the INPUT list is empty */
static int bs_step(const orc_engine* E, ctx_t* X, uint8_t sym, rvec* V) {
    X->valid.n = 0;
    for (size_t k = 0; k < V->n; k++) {
        int res = update_single(E, X, sym, &V->v[k]);
        X->c.interval_steps++;
        if (res) VEC_PUSH(&X->valid, V->v[k]);
    }
    if (V->n == 0) return 0;
    rvec t = *V; *V = X->valid; X->valid = t;
    return 1;
}

/* dollars_in_interval (:607-625) */
static void dollars_in_interval(const orc_engine* E, ctx_t* X, uint32_t i, uint32_t j) {
    uint32_t l = rsl_rank(&E->rsL, TERM, i);
    uint32_t u = rsl_rank(&E->rsL, TERM, j + 1);
    for (uint32_t k = l; k < u; k++) {
        uint32_t index = E->eof_id[k];
        X->c.eof_reads++;
        if (index > E->first_symbol_index) VEC_PUSH(&X->d, index);
    }
}

/* preceding_dollars_finder (:570-605) */
static rng_t preceding_dollars_finder(const orc_engine* E, uint32_t i) {
    uint32_t a = (i + 1 > E->bv_size) ? bv_rank1(E, E->bv_size) : bv_rank1(E, i + 1);
    uint32_t start = bv_select1(E, a - 1);
    uint32_t end = bv_select1(E, a) - 1;
    rng_t o;
    o.b = start;
    o.bi = E->dollar_ii[start];
    o.e = end;
    o.ei = E->dollar_ii[end];
    return o;
}

static int u32_cmp(const void* a, const void* b) {
    uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    return (x > y) - (x < y);
}

/* link (:512-563) — the deque is only used via push_back/back/pop_back/sort */
static void link_(const orc_engine* E, ctx_t* X) {
    X->d.n = 0;
    for (size_t it = 0; it < X->other.n; it++) {
        uint32_t b_ = X->other.v[it].bi, e_ = X->other.v[it].ei;
        if (b_ <= e_) dollars_in_interval(E, X, b_, e_);
    }
    if (X->d.n > 1) qsort(X->d.v, X->d.n, 4, u32_cmp); /* (n = 0: v may be NULL — qsort's argument must not be) */
    rvec* D = &X->dollar;
    while (X->d.n) {
        uint32_t x = X->d.v[--X->d.n];
        rng_t cur = preceding_dollars_finder(E, x);
        X->c.pdf_calls++;
        if (D->n && (cur.e + 1 >= D->v[D->n - 1].b)) {
            if (cur.b < D->v[D->n - 1].b) {
                D->v[D->n - 1].b = cur.b;
                D->v[D->n - 1].bi = cur.bi;
            }
        } else {
            VEC_PUSH(D, cur);
        }
        dollars_in_interval(E, X, cur.bi, cur.ei);
    }
    for (size_t i = 0, j = D->n ? D->n - 1 : 0; i < j; i++, j--) { rng_t t = D->v[i]; D->v[i] = D->v[j]; D->v[j] = t; }
}

/* LOCATE (:328-369): every row of the final list walks M_LF to its '#' */
static uint32_t locate_list(const orc_engine* E, ctx_t* X, uint32_t n_kmer, const rvec* V) {
    uint32_t num_occ = 0;
    for (size_t i = 0; i < V->n; i++) {
        rng_t iv = V->v[i];
        uint32_t prev_copy = iv.bi, prevII = iv.bi;
        num_occ += iv.e - iv.b + 1;
        for (uint32_t j = iv.b; j <= iv.e; j++) {
            uint32_t position = j, pos_in_string = 0;
            if (!(E->p[prev_copy + 1] - position > 0)) { prev_copy++; prevII = prev_copy; }
            while (E->L[prevII] != TERM) {
                mlf_move(E, &position, &prevII);
                pos_in_string++;
                X->c.locate_moves++;
            }
            uint32_t nd = rsl_rank(&E->rsL, TERM, prevII);
            uint32_t index = E->eof_id[nd];
            uint32_t D = bv_rank1(E, index + 1);
            uint32_t start = bv_select1(E, D);
            orc_occ o = {n_kmer, index, D, index - start, pos_in_string};
            VEC_PUSH(&X->out, o);
            X->c.occurrences++;
            prevII = prev_copy;
            if (j == 0xffffffffu) break;
        }
    }
    return num_occ;
}

/* One iteration of backwardSearch's character loop (:241-325): link the '#' rows of the
 * list, step both lists by sym, concatenate (:300) and merge adjacent intervals (:309-324).
 * Returns 0 when neither step found anything (the search ends with count 0). */
static int bs_level(const orc_engine* E, ctx_t* X, uint8_t sym) {
    int found = 0;
    link_(E, X);
    if (X->dollar.n) {
        if (bs_step(E, X, sym, &X->dollar)) found = 1;
    }
    if (bs_step(E, X, sym, &X->other)) found = 1;
    if (!found) return 0;
    for (size_t i = 0; i < X->other.n; i++) VEC_PUSH(&X->dollar, X->other.v[i]); /* :300 */
    { rvec t = X->other; X->other = X->dollar; X->dollar = t; }
    X->dollar.n = 0;
    if (X->other.n > 1) { /* adjacency merge (:309-324) */
        X->merged.n = 0;
        VEC_PUSH(&X->merged, X->other.v[0]);
        for (size_t i = 1; i < X->other.n; i++) {
            rng_t* last = &X->merged.v[X->merged.n - 1];
            if (X->other.v[i].b == last->e + 1) {
                last->e = X->other.v[i].e;
                last->ei = X->other.v[i].ei;
            } else {
                VEC_PUSH(&X->merged, X->other.v[i]);
            }
        }
        rvec t = X->other; X->other = X->merged; X->merged = t;
    }
    return 1;
}

/* backwardSearch (:228-374); occurrences appended to X->out */
static uint32_t backward_search(const orc_engine* E, ctx_t* X, uint32_t n_kmer, const uint8_t* kmer, uint32_t len) {
    X->early = 1;
    if (len == 0) return 0; /* kmer[len-1] is undefined behaviour in the reference (:239) */
    X->other.n = 0;
    X->dollar.n = 0;
    rng_t first = {0, E->n - 1, 0, E->r - 1}; /* init_backward_search (:220-225) */
    VEC_PUSH(&X->other, first);
    if (!bs_step(E, X, kmer[len - 1], &X->other)) return 0;
    for (uint32_t pos = len - 1; pos > 0; pos--)
        if (!bs_level(E, X, kmer[pos - 1])) return 0;
    X->early = 0;
    return locate_list(E, X, n_kmer, &X->other);
}

typedef struct {
    const orc_engine* E;
    const uint8_t* bytes;
    const uint64_t* off;
    uint64_t lo, hi;
    uint32_t first_id;
    uint32_t* counts;
    uint8_t* early;
    ctx_t X;
} job_t;

static void* job_run(void* arg) {
    job_t* J = arg;
    for (uint64_t i = J->lo; i < J->hi; i++) {
        uint32_t len = (uint32_t)(J->off[i + 1] - J->off[i]);
        uint32_t r = backward_search(J->E, &J->X, J->first_id + (uint32_t)i, J->bytes + J->off[i], len);
        J->counts[i] = r;
        if (J->early) J->early[i] = (uint8_t)J->X.early;
        if (r > 0) J->X.c.found++; else J->X.c.not_found++;
    }
    return NULL;
}

static void ctx_free(ctx_t* X) {
    free(X->other.v); free(X->dollar.v); free(X->valid.v); free(X->merged.v); free(X->d.v); free(X->out.v);
}

static void add_ctr(orc_counters* a, const orc_counters* b) {
    a->interval_steps += b->interval_steps; a->step_moves += b->step_moves; a->locate_moves += b->locate_moves;
    a->pdf_calls += b->pdf_calls; a->eof_reads += b->eof_reads; a->occurrences += b->occurrences;
    a->found += b->found; a->not_found += b->not_found;
}

static int search_batch(orc_engine* E, const char* bytes, const uint64_t* offsets, uint64_t npat,
                        uint32_t first_pattern_id, int threads, uint32_t* counts,
                        orc_occ** occ, uint64_t* nocc, orc_counters* ctr, uint8_t* early) {
    if (threads < 1) threads = 1;
    if ((uint64_t)threads > npat) threads = npat ? (int)npat : 1;
    job_t* J = xcalloc((size_t)threads, sizeof(job_t));
    pthread_t* th = xcalloc((size_t)threads, sizeof(pthread_t));
    for (int t = 0; t < threads; t++) {
        J[t].E = E; J[t].bytes = (const uint8_t*)bytes; J[t].off = offsets;
        J[t].lo = npat * (uint64_t)t / (uint64_t)threads;
        J[t].hi = npat * (uint64_t)(t + 1) / (uint64_t)threads;
        J[t].first_id = first_pattern_id; J[t].counts = counts; J[t].early = early;
    }
    if (threads == 1) job_run(&J[0]);
    else {
        for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, job_run, &J[t]);
        for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    }
    uint64_t tot = 0;
    for (int t = 0; t < threads; t++) tot += J[t].X.out.n;
    if (ctr) memset(ctr, 0, sizeof *ctr);
    if (occ) {
        *occ = xmalloc((size_t)tot * sizeof(orc_occ) + sizeof(orc_occ));
        uint64_t at = 0;
        for (int t = 0; t < threads; t++) {
            if (J[t].X.out.n) memcpy(*occ + at, J[t].X.out.v, J[t].X.out.n * sizeof(orc_occ));
            at += J[t].X.out.n;
        }
    }
    if (nocc) *nocc = tot;
    for (int t = 0; t < threads; t++) { if (ctr) add_ctr(ctr, &J[t].X.c); ctx_free(&J[t].X); }
    free(J); free(th);
    return 0;
}

int orc_search_batch(orc_engine* E, const char* bytes, const uint64_t* offsets, uint64_t npat,
                     uint32_t first_pattern_id, int threads, uint32_t* counts,
                     orc_occ** occ, uint64_t* nocc, orc_counters* ctr) {
    return search_batch(E, bytes, offsets, npat, first_pattern_id, threads, counts, occ, nocc, ctr, NULL);
}

int orc_search_batch_console(orc_engine* E, const char* bytes, const uint64_t* offsets, uint64_t npat,
                             uint32_t first_pattern_id, int threads, uint32_t* counts, uint8_t* early) {
    return search_batch(E, bytes, offsets, npat, first_pattern_id, threads, counts, NULL, NULL, NULL, early);
}

/* ---------------------------------------------------------- trie-sharing variant
 * backwardSearch's list after the last q characters of a pattern depends only on those q
 * characters, so a batch sorted by reversed pattern shares every common suffix: each thread
 * walks its contiguous range of the sorted order keeping the list of every depth of the
 * current path, and a pattern resumes from the deepest list it shares with the previous one.
 * Same counts and records as orc_search_batch; the counters count each distinct suffix once
 * (SURVEY §8(d)'s deduplicated work). */
typedef struct {
    const uint8_t* bytes;
    const uint64_t* off;
} rsort_arg;

static int rev_cmp(const void* pa, const void* pb, void* arg) {
    const rsort_arg* A = arg;
    uint64_t i = *(const uint64_t*)pa, j = *(const uint64_t*)pb;
    const uint8_t *x = A->bytes + A->off[i], *y = A->bytes + A->off[j];
    uint64_t m = A->off[i + 1] - A->off[i], n = A->off[j + 1] - A->off[j];
    for (uint64_t k = 0; k < m && k < n; k++) {
        uint8_t a = x[m - 1 - k], b = y[n - 1 - k];
        if (a != b) return (a > b) - (a < b);
    }
    if (m != n) return (m > n) - (m < n);
    return (i > j) - (i < j);
}

typedef struct {
    const orc_engine* E;
    const uint8_t* bytes;
    const uint64_t* off;
    const uint64_t* order;
    uint64_t lo, hi;
    uint32_t first_id;
    uint32_t* counts;
    uint64_t* rec_at; /* per pattern: its first record in X.out */
    ctx_t X;
} tjob_t;

static void* tjob_run(void* arg) {
    tjob_t* J = arg;
    const orc_engine* E = J->E;
    ctx_t* X = &J->X;
    rvec* st = NULL;   /* st[d]: the list after d characters of the current path */
    size_t nst = 0;
    uint32_t top = 0;  /* depths 1..top of st hold the previous pattern's path */
    uint32_t dead = 0; /* the previous path's search ended at this depth (0: it did not) */
    const uint8_t* prev = NULL;
    uint64_t prev_len = 0;
    for (uint64_t k = J->lo; k < J->hi; k++) {
        uint64_t i = J->order[k];
        const uint8_t* P = J->bytes + J->off[i];
        uint32_t len = (uint32_t)(J->off[i + 1] - J->off[i]);
        uint32_t h = 0; /* shared reversed prefix with the previous pattern */
        while (h < len && h < prev_len && h < top && P[len - 1 - h] == prev[prev_len - 1 - h]) h++;
        prev = P; prev_len = len;
        J->rec_at[i] = X->out.n;
        uint32_t r = 0;
        if (len == 0) { top = 0; dead = 0; goto done; }
        if (dead && dead <= h) { top = dead; goto done; } /* a shared suffix already failed */
        dead = 0;
        if (nst < (size_t)len + 1) {
            st = realloc(st, ((size_t)len + 1) * sizeof(rvec));
            memset(st + nst, 0, ((size_t)len + 1 - nst) * sizeof(rvec));
            nst = (size_t)len + 1;
        }
        X->dollar.n = 0;
        if (h == 0) {
            X->other.n = 0;
            rng_t first = {0, E->n - 1, 0, E->r - 1}; /* init_backward_search (:220-225) */
            VEC_PUSH(&X->other, first);
            bs_step(E, X, P[len - 1], &X->other);
            h = 1;
        } else {
            X->other.n = 0;
            for (size_t t = 0; t < st[h].n; t++) VEC_PUSH(&X->other, st[h].v[t]);
        }
        for (uint32_t d = h;; d++) {
            st[d].n = 0;
            for (size_t t = 0; t < X->other.n; t++) VEC_PUSH(&st[d], X->other.v[t]);
            top = d;
            if (d == len) break;
            if (!bs_level(E, X, P[len - 1 - d])) { dead = d + 1; top = d + 1; goto done; }
        }
        r = locate_list(E, X, J->first_id + (uint32_t)i, &X->other);
    done:
        J->counts[i] = r;
        if (r > 0) X->c.found++; else X->c.not_found++;
    }
    for (size_t d = 0; d < nst; d++) free(st[d].v);
    free(st);
    return NULL;
}

int orc_search_batch_trie(orc_engine* E, const char* bytes, const uint64_t* offsets, uint64_t npat,
                          uint32_t first_pattern_id, int threads, uint32_t* counts,
                          orc_occ** occ, uint64_t* nocc, orc_counters* ctr) {
    if (threads < 1) threads = 1;
    if (threads > 255) threads = 255;
    if ((uint64_t)threads > npat) threads = npat ? (int)npat : 1;
    uint64_t* order = xmalloc((size_t)npat * 8 + 8);
    uint64_t* rec_at = xmalloc((size_t)npat * 8 + 8);
    uint8_t* owner = xmalloc((size_t)npat + 1);
    for (uint64_t i = 0; i < npat; i++) order[i] = i;
    rsort_arg A = {(const uint8_t*)bytes, offsets};
    if (npat > 1) qsort_r(order, npat, 8, rev_cmp, &A);
    tjob_t* J = xcalloc((size_t)threads, sizeof(tjob_t));
    pthread_t* th = xcalloc((size_t)threads, sizeof(pthread_t));
    for (int t = 0; t < threads; t++) {
        J[t].E = E; J[t].bytes = (const uint8_t*)bytes; J[t].off = offsets; J[t].order = order;
        J[t].lo = npat * (uint64_t)t / (uint64_t)threads;
        J[t].hi = npat * (uint64_t)(t + 1) / (uint64_t)threads;
        J[t].first_id = first_pattern_id; J[t].counts = counts; J[t].rec_at = rec_at;
        for (uint64_t k = J[t].lo; k < J[t].hi; k++) owner[order[k]] = (uint8_t)t;
    }
    if (threads == 1) tjob_run(&J[0]);
    else {
        for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, tjob_run, &J[t]);
        for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    }
    uint64_t tot = 0;
    for (int t = 0; t < threads; t++) tot += J[t].X.out.n;
    if (ctr) memset(ctr, 0, sizeof *ctr);
    if (occ) { /* pattern order, as the reference writes them */
        *occ = xmalloc((size_t)tot * sizeof(orc_occ) + sizeof(orc_occ));
        uint64_t at = 0;
        for (uint64_t i = 0; i < npat; i++) {
            if (counts[i]) memcpy(*occ + at, J[owner[i]].X.out.v + rec_at[i], (size_t)counts[i] * sizeof(orc_occ));
            at += counts[i];
        }
    }
    if (nocc) *nocc = tot;
    for (int t = 0; t < threads; t++) { if (ctr) add_ctr(ctr, &J[t].X.c); ctx_free(&J[t].X); }
    free(J); free(th); free(order); free(rec_at); free(owner);
    return 0;
}

int orc_search_file(orc_engine* E, const char* patterns_path, const char* out_csv,
                    uint64_t limit, int threads, orc_counters* ctr, double* seconds) {
    uint8_t* buf;
    size_t n;
    if (read_file(patterns_path, &buf, &n)) return -1;
    /* std::getline semantics: split at '\n'; a final line without '\n' still counts */
    uint64_t* off = NULL;
    size_t np = 0, cap = 0;
    size_t s = 0;
    bvec pb = {0};
    while (s < n && (!limit || np < limit)) {
        size_t e = s;
        while (e < n && buf[e] != '\n') e++;
        if (np + 2 > cap) { cap = cap ? cap * 2 : 1024; off = realloc(off, cap * 8); }
        if (np == 0) off[0] = 0;
        for (size_t i = s; i < e; i++) VEC_PUSH(&pb, buf[i]);
        off[np + 1] = pb.n;
        np++;
        s = e + 1;
    }
    free(buf);
    uint32_t* counts = xcalloc(np + 1, 4);
    orc_occ* occ = NULL;
    uint64_t nocc = 0;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    orc_search_batch(E, (const char*)pb.v, off ? off : (uint64_t[]){0}, np, 1, threads, counts, &occ, &nocc, ctr);
    FILE* f = out_csv ? fopen(out_csv, "wb") : NULL;
    if (out_csv && !f) { free(pb.v); free(off); free(counts); free(occ); return fail("ERROR opening file %s to write output", out_csv); }
    if (f) {
        fputs("#Pat\t$_i\tD[i]\tS_j\tS_j[r] \n", f); /* :59 (trailing space) */
        for (uint64_t i = 0; i < nocc; i++)
            fprintf(f, "%u\t%u\t%u\t%u\t%u\n", occ[i].pat, occ[i].word, occ[i].seg, occ[i].word_in_seg, occ[i].offset);
        fclose(f);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (seconds) *seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    free(pb.v); free(off); free(counts); free(occ);
    return 0;
}

/* ------------------------------------------------ record checker (tests) */
/* Independent of any BWT: a record (pat, word, seg, word_in_seg, offset) is sound when
 * word/seg/word_in_seg agree with the .eds segmentation (rank1/select1 of the segment
 * bitvector, MOVE_EDSBWTSearch.cpp:361-363), word is non-empty, offset < |word|, and the
 * pattern can be spelled from word[offset], continuing at the start of any word of the
 * next segment, where a segment holding the empty word may be skipped (the link()
 * semantics of :512-625 seen forwards; tests/edsgen.py brute_occurrences). */
typedef struct {
    const eds_t* E;
    const uint32_t* seg_of; /* 1-based segment of each word */
    const uint32_t* seg_first; /* first word of segment s (1-based), [S+1] = W */
    uint32_t W, S;
} chk_t;

static inline uint32_t chk_wlen(const chk_t* C, uint32_t w) {
    const uint32_t e = w + 1 < C->W ? C->E->wstart.v[w + 1] - 1 : (uint32_t)C->E->text.n - 1;
    return e - C->E->wstart.v[w];
}
static inline int chk_empty(const chk_t* C, uint32_t w) {
    return chk_wlen(C, w) == 1 && C->E->text.v[C->E->wstart.v[w]] == EMPTYC;
}
static int chk_from_word(const chk_t* C, uint32_t w, uint32_t o, const uint8_t* P, uint32_t m, uint32_t p, uint64_t* budget);
static int chk_from_segment(const chk_t* C, uint32_t s, const uint8_t* P, uint32_t m, uint32_t p, uint64_t* budget) {
    if (p == m) return 1;
    if (s > C->S || !*budget) return 0;
    (*budget)--;
    for (uint32_t w = C->seg_first[s]; w < C->seg_first[s + 1]; w++) {
        if (chk_empty(C, w)) { if (chk_from_segment(C, s + 1, P, m, p, budget)) return 1; }
        else if (chk_from_word(C, w, 0, P, m, p, budget)) return 1;
    }
    return 0;
}
static int chk_from_word(const chk_t* C, uint32_t w, uint32_t o, const uint8_t* P, uint32_t m, uint32_t p, uint64_t* budget) {
    const uint32_t L = chk_wlen(C, w);
    uint32_t n = L - o;
    if (n > m - p) n = m - p;
    if (memcmp(C->E->text.v + C->E->wstart.v[w] + o, P + p, n) != 0) return 0;
    if (p + n == m) return 1;
    return chk_from_segment(C, C->seg_of[w] + 1, P, m, p + n, budget);
}

typedef struct {
    const chk_t* C;
    const uint8_t* bytes;
    const uint64_t* off;
    uint64_t npat;
    uint32_t first_id;
    const orc_occ* rec;
    uint64_t lo, hi, bad, first_bad;
} chk_job;

static void* chk_run(void* arg) {
    chk_job* J = arg;
    const chk_t* C = J->C;
    J->first_bad = ~0ull;
    for (uint64_t i = J->lo; i < J->hi; i++) {
        const orc_occ r = J->rec[i];
        int ok = r.pat >= J->first_id && (uint64_t)(r.pat - J->first_id) < J->npat && r.word < C->W;
        if (ok) ok = C->seg_of[r.word] == r.seg && r.word - C->seg_first[r.seg] == r.word_in_seg && !chk_empty(C, r.word) &&
                     r.offset < chk_wlen(C, r.word);
        if (ok) {
            const uint64_t k = r.pat - J->first_id;
            uint64_t budget = 1u << 20;
            ok = chk_from_word(C, r.word, r.offset, J->bytes + J->off[k], (uint32_t)(J->off[k + 1] - J->off[k]), 0, &budget);
        }
        if (!ok) { J->bad++; if (J->first_bad == ~0ull) J->first_bad = i; }
    }
    return NULL;
}

int orc_check_records(const char* eds_path, const char* bytes, const uint64_t* offsets, uint64_t npat, uint32_t first_pattern_id,
                      const orc_occ* rec, uint64_t nocc, int threads, uint64_t* bad, uint64_t* first_bad) {
    uint8_t* s;
    size_t n;
    if (read_file(eds_path, &s, &n)) return -1;
    eds_t E;
    int rc = eds_parse(s, n, &E);
    free(s);
    if (rc) return -1;
    chk_t C = {&E, NULL, NULL, (uint32_t)E.wstart.n, 0};
    uint32_t* so = xmalloc((size_t)C.W * 4);
    uint32_t* sf = xmalloc(((size_t)C.W + 2) * 4);
    for (uint32_t w = 0; w < C.W; w++) {
        if (E.bits.v[w]) sf[++C.S] = w;
        so[w] = C.S;
    }
    sf[C.S + 1] = C.W;
    C.seg_of = so;
    C.seg_first = sf;
    if (threads < 1) threads = 1;
    chk_job* J = xcalloc((size_t)threads, sizeof(chk_job));
    pthread_t* th = xcalloc((size_t)threads, sizeof(pthread_t));
    for (int t = 0; t < threads; t++) {
        J[t] = (chk_job){&C, (const uint8_t*)bytes, offsets, npat, first_pattern_id, rec,
                         nocc * (uint64_t)t / (uint64_t)threads, nocc * (uint64_t)(t + 1) / (uint64_t)threads, 0, 0};
        pthread_create(&th[t], NULL, chk_run, &J[t]);
    }
    *bad = 0;
    *first_bad = ~0ull;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        *bad += J[t].bad;
        if (J[t].first_bad < *first_bad) *first_bad = J[t].first_bad;
    }
    free(J); free(th); free(so); free(sf);
    eds_free(&E);
    return 0;
}
