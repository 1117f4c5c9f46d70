/*
 * sw_simd.c -- inter-sequence SIMD restatement of the oracle (TEST
 * INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg times it, tests check it
 * bit-exact against the scalar oracle; nothing in the product links it).
 *
 * The reference's CPU/SIMD path does not exist (the crate has
 * no CPU aligner and Rust is absent here), so the CPU baseline is this
 * restatement of oracle/sw_oracle.c, vectorised the classic way for short
 * reads: VW pairs side by side, one int16 lane each (AVX-512BW: 32 lanes,
 * AVX2: 16), row-major over (i, j) of the longest pair of the group with
 * per-lane validity masks, so every lane computes exactly the scalar
 * recurrence (linear or Gotoh) and the row-major strict '>' best cell.
 * Compiled twice by oracle/Makefile (-mavx512bw -DSW_AVX512 / -mavx2); int16
 * without saturation is exact for every scheme msw.h accepts: |H| <= 64 * 256
 * and E/F stay >= -(30000 + 1024) - 1024.
 */
#include <immintrin.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef SW_AVX512
#define VW 32
typedef __m512i V;
typedef __mmask32 M;
#define SET1(x) _mm512_set1_epi16((short)(x))
#define ADD _mm512_add_epi16
#define SUB _mm512_sub_epi16
#define MAX _mm512_max_epi16
#define LOAD(p) _mm512_load_si512((const void*)(p))
#define STORE(p, v) _mm512_store_si512((void*)(p), v)
#define EQ_SEL(a, b, x, y) _mm512_mask_blend_epi16(_mm512_cmpeq_epi16_mask(a, b), y, x)
#define GT_MASK(a, b) _mm512_cmpgt_epi16_mask(a, b)
#define MASK_AND(a, b) ((M)((a) & (b)))
#define MASK_SEL(m, x, y) _mm512_mask_blend_epi16(m, y, x) /* m ? x : y */
#define MASK_MAX(acc, m, h) _mm512_mask_max_epi16(acc, m, acc, h)
#define FN(name) name##_avx512
#else
#define VW 16
typedef __m256i V;
typedef __m256i M;
#define SET1(x) _mm256_set1_epi16((short)(x))
#define ADD _mm256_add_epi16
#define SUB _mm256_sub_epi16
#define MAX _mm256_max_epi16
#define LOAD(p) _mm256_load_si256((const __m256i*)(p))
#define STORE(p, v) _mm256_store_si256((__m256i*)(p), v)
#define EQ_SEL(a, b, x, y) _mm256_blendv_epi8(y, x, _mm256_cmpeq_epi16(a, b))
#define GT_MASK(a, b) _mm256_cmpgt_epi16(a, b)
#define MASK_AND(a, b) _mm256_and_si256(a, b)
#define MASK_SEL(m, x, y) _mm256_blendv_epi8(y, x, m)
#define MASK_MAX(acc, m, h) _mm256_blendv_epi8(acc, _mm256_max_epi16(acc, h), m)
#define FN(name) name##_avx2
#endif

typedef struct {
    int16_t v[VW];
} __attribute__((aligned(64))) row_t;

/* lanes whose length exceeds idx: i < m_lane / j < n_lane */
static inline M valid_mask(V len, int idx) { return GT_MASK(len, SET1(idx)); }

/* Score (and best cell) of pairs [p0, p0 + VW) of the batch (lanes past
 * n_pairs are empty).  Scratch: (max_n + 1) rows each of H and F. */
static void group(const uint8_t* reads, const uint8_t* wins, const uint16_t* read_len, const uint16_t* win_len,
                  uint32_t read_stride, uint32_t win_stride, uint64_t p0, uint64_t n_pairs, int match, int mismatch,
                  int gap_open, int gap_extend, int affine, int32_t* score, int16_t* end_i, int16_t* end_j,
                  row_t* rt, row_t* wt, row_t* H, row_t* F) {
    int mm = 0, nn = 0;
    int16_t ml[VW], nl[VW];
    for (int l = 0; l < VW; ++l) {
        const uint64_t p = p0 + l;
        ml[l] = p < n_pairs ? (int16_t)read_len[p] : 0;
        nl[l] = p < n_pairs ? (int16_t)win_len[p] : 0;
        if (ml[l] > mm) mm = ml[l];
        if (nl[l] > nn) nn = nl[l];
    }
    /* transposed bytes: rt[i].v[l] = read l byte i, wt[j].v[l] = window l byte j */
    for (int i = 0; i < mm; ++i)
        for (int l = 0; l < VW; ++l) rt[i].v[l] = i < ml[l] ? reads[(p0 + l) * read_stride + i] : 0;
    for (int j = 0; j < nn; ++j)
        for (int l = 0; l < VW; ++l) wt[j].v[l] = j < nl[l] ? wins[(p0 + l) * win_stride + j] : 0;
    V mlen, nlen;
    memcpy(&mlen, ml, sizeof(V));
    memcpy(&nlen, nl, sizeof(V));
    const V vmatch = SET1(match), vmis = SET1(mismatch), zero = SET1(0);
    const V vge = SET1(gap_extend), vgoe = SET1(gap_open + gap_extend), vgap = SET1(gap_extend);
    const V neg = SET1(-(30000 + 1024));
    for (int j = 0; j <= nn; ++j) {
        STORE(&H[j], zero);
        STORE(&F[j], neg);
    }
    V best = zero, bi = SET1(-1), bj = SET1(-1);
    const int coords = end_i != NULL;
    for (int i = 0; i < mm; ++i) {
        const V ri = LOAD(&rt[i]);
        const M vrow = valid_mask(mlen, i);
        const V iv = SET1(i);
        V diag = zero; /* H[i-1][j-1], column -1 is zero */
        V left = zero; /* H[i][j-1] */
        V E = neg;
        for (int j = 0; j < nn; ++j) {
            const V up = LOAD(&H[j + 1]);
            const V s = EQ_SEL(ri, LOAD(&wt[j]), vmatch, vmis);
            V h = ADD(diag, s);
            if (affine) {
                E = MAX(SUB(E, vge), SUB(left, vgoe));
                const V f = MAX(SUB(LOAD(&F[j + 1]), vge), SUB(up, vgoe));
                STORE(&F[j + 1], f);
                h = MAX(MAX(h, E), MAX(f, zero));
            } else {
                h = MAX(MAX(h, SUB(up, vgap)), MAX(SUB(left, vgap), zero));
            }
            STORE(&H[j + 1], h);
            diag = up;
            left = h;
            const M valid = MASK_AND(vrow, valid_mask(nlen, j));
            if (coords) {
                const M better = MASK_AND(valid, GT_MASK(h, best));
                best = MASK_SEL(better, h, best);
                bi = MASK_SEL(better, iv, bi);
                bj = MASK_SEL(better, SET1(j), bj);
            } else {
                best = MASK_MAX(best, valid, h);
            }
        }
    }
    int16_t b[VW], ei[VW], ej[VW];
    memcpy(b, &best, sizeof(V));
    memcpy(ei, &bi, sizeof(V));
    memcpy(ej, &bj, sizeof(V));
    for (int l = 0; l < VW && p0 + l < n_pairs; ++l) {
        score[p0 + l] = b[l];
        if (coords) {
            end_i[p0 + l] = b[l] ? ei[l] : -1;
            end_j[p0 + l] = b[l] ? ej[l] : -1;
        }
    }
}

/* Pairs [begin, end) in groups of VW (begin a multiple of VW). */
void FN(oracle_simd_range)(const uint8_t* reads, const uint8_t* wins, const uint16_t* read_len,
                           const uint16_t* win_len, uint32_t read_stride, uint32_t win_stride, uint64_t begin,
                           uint64_t end, uint64_t n_pairs, int match, int mismatch, int gap_open, int gap_extend,
                           int affine, int32_t* score, int16_t* end_i, int16_t* end_j) {
    int mm = 1, nn = 1;
    for (uint64_t p = begin; p < end && p < n_pairs; ++p) {
        if (read_len[p] > mm) mm = read_len[p];
        if (win_len[p] > nn) nn = win_len[p];
    }
    row_t* rt = (row_t*)aligned_alloc(64, sizeof(row_t) * (size_t)mm);
    row_t* wt = (row_t*)aligned_alloc(64, sizeof(row_t) * (size_t)nn);
    row_t* H = (row_t*)aligned_alloc(64, sizeof(row_t) * (size_t)(nn + 1));
    row_t* F = (row_t*)aligned_alloc(64, sizeof(row_t) * (size_t)(nn + 1));
    for (uint64_t p0 = begin; p0 < end; p0 += VW)
        group(reads, wins, read_len, win_len, read_stride, win_stride, p0, end < n_pairs ? end : n_pairs, match,
              mismatch, gap_open, gap_extend, affine, score, end_i, end_j, rt, wt, H, F);
    free(rt);
    free(wt);
    free(H);
    free(F);
}
