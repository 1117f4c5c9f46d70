/*
 * sw_oracle.h -- CPU restatement of the reference's scoring path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (mini_parallel_amd/,
 * include/msw.h, the rustseq_mini CLI) links, loads or calls this code.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it,
 * and only as the checker / the timed CPU baseline.
 *
 * Parity status: the reference (bmwoolf/mini_parallel, Rust + OpenCL) has no
 * tests, no golden vectors and no runnable implementation of the SW recurrence
 * (smith_waterman_detailed, smith_waterman.cl:74-152, is never launched and has
 * data races).  The SW functions below are therefore "parity unpinned" against
 * the reference itself; they are pinned by the known-answer table of
 * SURVEY.md 8(c) and cross-checked against an independent numpy restatement
 * (oracle/sw_oracle_np.py).  The compat function restates the kernel the
 * reference actually launches (smith_waterman.cl:11-71 + aligner.rs:410-532).
 */
#ifndef MSW_SW_ORACLE_H
#define MSW_SW_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One alignment result.  score >= 0; (end_i, end_j) are the 0-based read /
 * window coordinates of the best cell, smallest i then smallest j on ties,
 * (-1,-1) when score == 0. */
typedef struct {
    int32_t score;
    int32_t end_i;
    int32_t end_j;
} oracle_hit_t;

/* Linear gap SW: H = max(0, H[i-1][j-1]+s, H[i-1][j]-gap, H[i][j-1]-gap),
 * s = match if read[i]==win[j] (byte equality) else mismatch.
 * Follows the intended recurrence of smith_waterman.cl:112-126 with
 * the constants of smith_waterman.cl:5-7, but takes the global max. */
oracle_hit_t oracle_sw_linear(const uint8_t* read, int m, const uint8_t* win, int n,
                              int match, int mismatch, int gap);

/* Affine (Gotoh) SW: a gap of length k costs gap_open + k*gap_extend.
 * E (gap in read, horizontal) / F (gap in window, vertical).
 * gap_open == 0 reproduces oracle_sw_linear with gap == gap_extend. */
oracle_hit_t oracle_sw_affine(const uint8_t* read, int m, const uint8_t* win, int n,
                              int match, int mismatch, int gap_open, int gap_extend);

/* Batched driver over a padded SoA batch (same layout as msw_batch_t):
 * pair p: read = reads + p*read_stride (read_len[p] bytes), window likewise.
 * affine == 0 -> linear with gap = gap_extend (gap_open ignored).
 * threads <= 1 -> single-threaded.  Writes score[p] and, when non-NULL,
 * end_i[p] / end_j[p]. */
void oracle_sw_batch(const uint8_t* reads, const uint8_t* wins,
                     const uint16_t* read_len, const uint16_t* win_len,
                     uint32_t read_stride, uint32_t win_stride, uint64_t n_pairs,
                     int match, int mismatch, int gap_open, int gap_extend, int affine,
                     int32_t* score, int16_t* end_i, int16_t* end_j, int threads);

/* Same results as oracle_sw_batch (bit-exact), computed by the inter-sequence
 * SIMD restatement (sw_simd.c: AVX-512BW 32 x int16 lanes, else AVX2 16, else
 * the scalar code).  Returns the vector width used in bits (512 / 256 / 0).
 * bench.py times it as the CPU baseline. */
int oracle_sw_batch_simd(const uint8_t* reads, const uint8_t* wins, const uint16_t* read_len,
                         const uint16_t* win_len, uint32_t read_stride, uint32_t win_stride, uint64_t n_pairs,
                         int match, int mismatch, int gap_open, int gap_extend, int affine, int32_t* score,
                         int16_t* end_i, int16_t* end_j, int threads);
int oracle_simd_isa(void);

/* Restatement of the kernel the reference launches, smith_waterman_align
 * (smith_waterman.cl:11-71), with the host geometry of gpu_align
 * (aligner.rs:413-424): L = min(n1,n2); W = work-group size; G = min(ceil(L/W), 1e6);
 * chunk C = ceil(L/G) (max_groups replaces the 1e6 cap, gpu.rs:10, when non-zero); work-item (g,t) runs Kadane over positions
 * g*C + t + k*W < min((g+1)*C, L) with s = +2/-1 on seq1[p]==seq2[p];
 * result = max(0, max over work-items).  L == 0 -> 0 (aligner.rs:414-416). */
int32_t oracle_compat_align(const uint8_t* s1, size_t n1, const uint8_t* s2, size_t n2,
                            uint32_t wg, uint32_t max_groups);

#ifdef __cplusplus
}
#endif
#endif
