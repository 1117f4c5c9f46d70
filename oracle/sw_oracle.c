/*
 * sw_oracle.c -- CPU restatement of the reference's scoring path (checker).
 *
 * TEST INFRASTRUCTURE ONLY: see sw_oracle.h.  Plain scalar C, deliberately
 * written as the textbook recurrence (row-major scan, strict '>' for the best
 * cell) so that it is easy to audit against the reference lines it follows:
 *   constants            smith_waterman.cl:5-7   (MATCH 2, MISMATCH -1, GAP -2)
 *   linear recurrence    smith_waterman.cl:112-126 (intended; the reference's
 *                        dead kernel also has races and a last-row-only max,
 *                        which we do not reproduce -- SURVEY.md 8a-3)
 *   byte equality        smith_waterman.cl:43,114 (case-sensitive, 'N'=='N')
 *   compat kernel        smith_waterman.cl:11-71, geometry aligner.rs:413-424
 */
#include "sw_oracle.h"

#include <limits.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define NEG_INF (INT_MIN / 4)

static inline int imax(int a, int b) { return a > b ? a : b; }

oracle_hit_t oracle_sw_linear(const uint8_t* read, int m, const uint8_t* win, int n,
                              int match, int mismatch, int gap) {
    oracle_hit_t hit = {0, -1, -1};
    if (m <= 0 || n <= 0) return hit;
    /* prev[j+1] = H[i-1][j], cur[j+1] = H[i][j]; index 0 is the zero column. */
    int* prev = (int*)calloc((size_t)n + 1, sizeof(int));
    int* cur = (int*)calloc((size_t)n + 1, sizeof(int));
    for (int i = 0; i < m; ++i) {
        cur[0] = 0;
        for (int j = 0; j < n; ++j) {
            int s = (read[i] == win[j]) ? match : mismatch;
            int h = prev[j] + s;                 /* diagonal */
            h = imax(h, prev[j + 1] - gap);      /* up: gap in the window */
            h = imax(h, cur[j] - gap);           /* left: gap in the read */
            h = imax(h, 0);
            cur[j + 1] = h;
            if (h > hit.score) { hit.score = h; hit.end_i = i; hit.end_j = j; }
        }
        int* t = prev; prev = cur; cur = t;
    }
    free(prev);
    free(cur);
    return hit;
}

oracle_hit_t oracle_sw_affine(const uint8_t* read, int m, const uint8_t* win, int n,
                              int match, int mismatch, int gap_open, int gap_extend) {
    oracle_hit_t hit = {0, -1, -1};
    if (m <= 0 || n <= 0) return hit;
    const int goe = gap_open + gap_extend;
    int* Hp = (int*)calloc((size_t)n + 1, sizeof(int));   /* H[i-1][*] */
    int* Hc = (int*)calloc((size_t)n + 1, sizeof(int));   /* H[i][*]   */
    int* F = (int*)malloc(((size_t)n + 1) * sizeof(int)); /* F[i-1][*] -> F[i][*] */
    for (int j = 0; j <= n; ++j) F[j] = NEG_INF;
    for (int i = 0; i < m; ++i) {
        int E = NEG_INF;                                   /* E[i][-1] */
        Hc[0] = 0;
        for (int j = 0; j < n; ++j) {
            /* E: gap in the read (horizontal), from H[i][j-1] / E[i][j-1]. */
            E = imax(E - gap_extend, Hc[j] - goe);
            /* F: gap in the window (vertical), from H[i-1][j] / F[i-1][j]. */
            int f = imax(F[j + 1] - gap_extend, Hp[j + 1] - goe);
            F[j + 1] = f;
            int s = (read[i] == win[j]) ? match : mismatch;
            int h = Hp[j] + s;
            h = imax(h, E);
            h = imax(h, f);
            h = imax(h, 0);
            Hc[j + 1] = h;
            if (h > hit.score) { hit.score = h; hit.end_i = i; hit.end_j = j; }
        }
        int* t = Hp; Hp = Hc; Hc = t;
    }
    free(Hp);
    free(Hc);
    free(F);
    return hit;
}

typedef struct {
    const uint8_t* reads; const uint8_t* wins;
    const uint16_t* read_len; const uint16_t* win_len;
    uint32_t read_stride, win_stride;
    uint64_t begin, end;
    int match, mismatch, gap_open, gap_extend, affine;
    int32_t* score; int16_t* end_i; int16_t* end_j;
} batch_job_t;

static void* batch_worker(void* arg) {
    batch_job_t* jb = (batch_job_t*)arg;
    for (uint64_t p = jb->begin; p < jb->end; ++p) {
        const uint8_t* r = jb->reads + p * jb->read_stride;
        const uint8_t* w = jb->wins + p * jb->win_stride;
        oracle_hit_t h = jb->affine
            ? oracle_sw_affine(r, jb->read_len[p], w, jb->win_len[p], jb->match, jb->mismatch,
                               jb->gap_open, jb->gap_extend)
            : oracle_sw_linear(r, jb->read_len[p], w, jb->win_len[p], jb->match, jb->mismatch,
                               jb->gap_extend);
        jb->score[p] = h.score;
        if (jb->end_i) jb->end_i[p] = (int16_t)h.end_i;
        if (jb->end_j) jb->end_j[p] = (int16_t)h.end_j;
    }
    return NULL;
}

void oracle_sw_batch(const uint8_t* reads, const uint8_t* wins,
                     const uint16_t* read_len, const uint16_t* win_len,
                     uint32_t read_stride, uint32_t win_stride, uint64_t n_pairs,
                     int match, int mismatch, int gap_open, int gap_extend, int affine,
                     int32_t* score, int16_t* end_i, int16_t* end_j, int threads) {
    if (threads < 1) threads = 1;
    if ((uint64_t)threads > n_pairs) threads = n_pairs ? (int)n_pairs : 1;
    batch_job_t* jobs = (batch_job_t*)calloc((size_t)threads, sizeof(batch_job_t));
    pthread_t* tids = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    for (int t = 0; t < threads; ++t) {
        batch_job_t* jb = &jobs[t];
        jb->reads = reads; jb->wins = wins; jb->read_len = read_len; jb->win_len = win_len;
        jb->read_stride = read_stride; jb->win_stride = win_stride;
        jb->begin = n_pairs * (uint64_t)t / (uint64_t)threads;
        jb->end = n_pairs * (uint64_t)(t + 1) / (uint64_t)threads;
        jb->match = match; jb->mismatch = mismatch;
        jb->gap_open = gap_open; jb->gap_extend = gap_extend; jb->affine = affine;
        jb->score = score; jb->end_i = end_i; jb->end_j = end_j;
    }
    if (threads == 1) {
        batch_worker(&jobs[0]);
    } else {
        for (int t = 0; t < threads; ++t) pthread_create(&tids[t], NULL, batch_worker, &jobs[t]);
        for (int t = 0; t < threads; ++t) pthread_join(tids[t], NULL);
    }
    free(jobs);
    free(tids);
}

int32_t oracle_compat_align(const uint8_t* s1, size_t n1, const uint8_t* s2, size_t n2,
                            uint32_t wg, uint32_t max_groups) {
    /* aligner.rs:411-416 */
    size_t L = n1 < n2 ? n1 : n2;
    if (L == 0 || wg == 0) return 0;
    /* aligner.rs:422-424: W = min(max_wg, 1024); G = min(ceil(L/W), 1e6) */
    size_t W = wg;
    size_t G = (L + W - 1) / W;
    const size_t cap = max_groups ? max_groups : 1000000;
    if (G > cap) G = cap;
    /* smith_waterman.cl:26-28 */
    size_t C = (L + G - 1) / G;
    int32_t result = 0; /* uninitialised result buffer (aligner.rs:494-499) taken as 0 */
    for (size_t g = 0; g < G; ++g) {
        size_t start = g * C;
        if (start >= L) continue;                       /* smith_waterman.cl:30-32 */
        size_t end = start + C < L ? start + C : L;
        for (size_t t = 0; t < W; ++t) {
            int32_t best = 0, cur = 0;                   /* smith_waterman.cl:35-36 */
            for (size_t p = start + t; p < end; p += W) { /* :39 */
                int32_t s = (s1[p] == s2[p]) ? 2 : -1;   /* :43-47 */
                cur = cur + s > 0 ? cur + s : 0;         /* :50 */
                if (cur > best) best = cur;              /* :51 */
            }
            if (best > result) result = best;            /* work-group max + atomic_max :60-69 */
        }
    }
    return result;
}

/* ---- inter-sequence SIMD baseline (sw_simd.c, compiled per ISA) ---- */
typedef void (*simd_range_fn)(const uint8_t*, const uint8_t*, const uint16_t*, const uint16_t*, uint32_t, uint32_t,
                              uint64_t, uint64_t, uint64_t, int, int, int, int, int, int32_t*, int16_t*, int16_t*);
void oracle_simd_range_avx512(const uint8_t*, const uint8_t*, const uint16_t*, const uint16_t*, uint32_t, uint32_t,
                              uint64_t, uint64_t, uint64_t, int, int, int, int, int, int32_t*, int16_t*, int16_t*);
void oracle_simd_range_avx2(const uint8_t*, const uint8_t*, const uint16_t*, const uint16_t*, uint32_t, uint32_t,
                            uint64_t, uint64_t, uint64_t, int, int, int, int, int, int32_t*, int16_t*, int16_t*);

typedef struct {
    simd_range_fn fn;
    batch_job_t jb;
    uint64_t n_pairs;
} simd_job_t;

static void* simd_worker(void* arg) {
    simd_job_t* s = (simd_job_t*)arg;
    batch_job_t* jb = &s->jb;
    if (jb->begin < jb->end)
        s->fn(jb->reads, jb->wins, jb->read_len, jb->win_len, jb->read_stride, jb->win_stride, jb->begin, jb->end,
              s->n_pairs, jb->match, jb->mismatch, jb->gap_open, jb->gap_extend, jb->affine, jb->score, jb->end_i,
              jb->end_j);
    return NULL;
}

int oracle_simd_isa(void) {
    __builtin_cpu_init();
    if (__builtin_cpu_supports("avx512bw")) return 512;
    if (__builtin_cpu_supports("avx2")) return 256;
    return 0;
}

int oracle_sw_batch_simd(const uint8_t* reads, const uint8_t* wins, const uint16_t* read_len,
                         const uint16_t* win_len, uint32_t read_stride, uint32_t win_stride, uint64_t n_pairs,
                         int match, int mismatch, int gap_open, int gap_extend, int affine, int32_t* score,
                         int16_t* end_i, int16_t* end_j, int threads) {
    const int isa = oracle_simd_isa();
    if (isa == 0) {
        oracle_sw_batch(reads, wins, read_len, win_len, read_stride, win_stride, n_pairs, match, mismatch, gap_open,
                        gap_extend, affine, score, end_i, end_j, threads);
        return 0;
    }
    const uint64_t vw = isa == 512 ? 32 : 16;
    const uint64_t groups = (n_pairs + vw - 1) / vw;
    if (threads < 1) threads = 1;
    if ((uint64_t)threads > groups) threads = groups ? (int)groups : 1;
    simd_job_t* jobs = (simd_job_t*)calloc((size_t)threads, sizeof(simd_job_t));
    pthread_t* tids = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    for (int t = 0; t < threads; ++t) {
        simd_job_t* s = &jobs[t];
        s->fn = isa == 512 ? oracle_simd_range_avx512 : oracle_simd_range_avx2;
        s->n_pairs = n_pairs;
        batch_job_t* jb = &s->jb;
        jb->reads = reads; jb->wins = wins; jb->read_len = read_len; jb->win_len = win_len;
        jb->read_stride = read_stride; jb->win_stride = win_stride;
        jb->begin = groups * (uint64_t)t / (uint64_t)threads * vw;
        jb->end = groups * (uint64_t)(t + 1) / (uint64_t)threads * vw;
        jb->match = match; jb->mismatch = mismatch;
        jb->gap_open = gap_open; jb->gap_extend = gap_extend; jb->affine = affine;
        jb->score = score; jb->end_i = end_i; jb->end_j = end_j;
    }
    if (threads == 1) {
        simd_worker(&jobs[0]);
    } else {
        for (int t = 0; t < threads; ++t) pthread_create(&tids[t], NULL, simd_worker, &jobs[t]);
        for (int t = 0; t < threads; ++t) pthread_join(tids[t], NULL);
    }
    free(jobs);
    free(tids);
    return isa;
}
