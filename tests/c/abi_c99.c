/* A plain C99 consumer of the C ABI (include/msw.h, include/msw_fastq.h):
 * compiled with -std=c99 -pedantic -Werror by tests/test_abi.py and run.  It
 * references every entry point (so the link proves they exist) and checks the
 * no-GPU / bad-argument contract: status codes plus msw_last_error text.
 * With a GPU (argv[1] == "gpu") it also scores one pair. */
#include <stdio.h>
#include <string.h>

#include "msw.h"
#include "msw_fastq.h"

typedef void (*fn_t)(void);
static int fails = 0;
#define CHECK(cond)                                                       \
    do {                                                                  \
        if (!(cond)) {                                                    \
            fprintf(stderr, "FAIL %s:%d: %s (%s)\n", __FILE__, __LINE__, #cond, \
                    msw_last_error());                                    \
            ++fails;                                                      \
        }                                                                 \
    } while (0)

int main(int argc, char** argv) {
    fn_t fns[] = {(fn_t)msw_device_count, (fn_t)msw_device_info, (fn_t)msw_ctx_create, (fn_t)msw_ctx_create_ex,
                   (fn_t)msw_ctx_destroy, (fn_t)msw_align_batch, (fn_t)msw_align_batch_async,
                   (fn_t)msw_wait, (fn_t)msw_align_batch_device, (fn_t)msw_plan_create,
                   (fn_t)msw_align_batch_planned, (fn_t)msw_plan_destroy, (fn_t)msw_align_compat,
                   (fn_t)msw_host_alloc, (fn_t)msw_host_free, (fn_t)msw_genome_create,
                   (fn_t)msw_genome_destroy, (fn_t)msw_genome_length, (fn_t)msw_align_reads,
                   (fn_t)msw_align_reads_async, (fn_t)msw_genome_cut_device, (fn_t)msw_dev_alloc, (fn_t)msw_dev_free,
                   (fn_t)msw_memcpy_h2d, (fn_t)msw_memcpy_d2h, (fn_t)msw_synchronize,
                   (fn_t)msw_last_error, (fn_t)msw_version, (fn_t)msw_fastq_open,
                   (fn_t)msw_fastq_close, (fn_t)msw_fastq_next, (fn_t)msw_fastq_stats,
                   (fn_t)msw_fastq_count_bases, (fn_t)msw_stream_create, (fn_t)msw_stream_destroy};
    size_t k;
    const int gpu = argc > 1 && strcmp(argv[1], "gpu") == 0;
    int n = -1;
    msw_ctx* ctx = NULL;
    for (k = 0; k < sizeof(fns) / sizeof(fns[0]); ++k) CHECK(fns[k] != (fn_t)0);
    CHECK(strstr(msw_version(), "gfx950") != NULL);
    /* NULL arguments are MSW_E_INVALID, never a crash */
    CHECK(msw_device_count(NULL) == MSW_E_INVALID);
    CHECK(msw_ctx_create(0, NULL) == MSW_E_INVALID);
    CHECK(msw_ctx_create_ex(0, MSW_CTX_LEAN, NULL) == MSW_E_INVALID);
    CHECK(msw_stream_create(NULL, NULL) == MSW_E_INVALID);
    CHECK(msw_stream_destroy(NULL, NULL) == MSW_E_INVALID);
    CHECK(msw_align_batch(NULL, NULL, NULL, NULL, 0) == MSW_E_INVALID);
    CHECK(strlen(msw_last_error()) > 0);
    CHECK(msw_fastq_open("/nonexistent.fastq.gz", NULL) == MSW_E_INVALID);
    if (!gpu) {
        /* no GPU: the reference refuses to run without one (main.rs:160-163) */
        CHECK(msw_device_count(&n) == MSW_E_NODEVICE && n == 0);
        CHECK(msw_ctx_create(0, &ctx) == MSW_E_NODEVICE && ctx == NULL);
    } else {
        const msw_scoring_t sc = {2, -1, 0, 2, 0, 1};
        const uint8_t read[16] = "ACGTACGT", win[16] = "ACGACGT";
        const uint16_t rl = 8, wl = 7;
        int32_t score = 0;
        int16_t ei = 0, ej = 0;
        msw_batch_t b;
        msw_out_t o;
        b.reads = read; b.wins = win; b.read_len = &rl; b.win_len = &wl;
        b.read_stride = 16; b.win_stride = 16; b.n_pairs = 1;
        o.score = &score; o.end_i = &ei; o.end_j = &ej;
        CHECK(msw_device_count(&n) == MSW_OK && n >= 1);
        CHECK(msw_ctx_create(0, &ctx) == MSW_OK);
        CHECK(msw_align_batch(ctx, &sc, &b, &o, 0) == MSW_OK);
        CHECK(score == 12 && ei == 7 && ej == 6); /* SURVEY.md 8c known answer */
        msw_ctx_destroy(ctx);
        /* a lean context: its extra streams made by the first async call */
        ctx = NULL;
        score = 0;
        CHECK(msw_ctx_create_ex(0, 7u, &ctx) == MSW_E_INVALID && ctx == NULL);
        CHECK(msw_ctx_create_ex(0, MSW_CTX_LEAN, &ctx) == MSW_OK);
        CHECK(msw_align_batch(ctx, &sc, &b, &o, 0) == MSW_OK && score == 12);
        {
            uint64_t t = 0;
            score = 0;
            CHECK(msw_align_batch_async(ctx, &sc, &b, &o, 0, &t) == MSW_OK && msw_wait(ctx, t) == MSW_OK);
            CHECK(score == 12 && ei == 7 && ej == 6);
        }
        {
            /* a stream of the caller's: a copy and a fence on it */
            void* st = NULL;
            uint64_t f = 0;
            uint8_t back[16] = {0};
            void* d = msw_dev_alloc(ctx, 16);
            CHECK(d != NULL);
            CHECK(msw_stream_create(ctx, &st) == MSW_OK && st != NULL);
            CHECK(msw_memcpy_h2d(ctx, d, read, 16) == MSW_OK);
            CHECK(msw_memcpy_d2h_async(ctx, back, d, 16, st) == MSW_OK);
            CHECK(msw_fence_record(ctx, st, &f) == MSW_OK && msw_fence_wait(ctx, f) == MSW_OK);
            CHECK(memcmp(back, read, 16) == 0);
            CHECK(msw_synchronize(ctx) == MSW_OK);
            CHECK(msw_stream_destroy(ctx, st) == MSW_OK);
            CHECK(msw_stream_destroy(ctx, st) == MSW_E_INVALID); /* no longer this context's */
            msw_dev_free(ctx, d);
        }
        msw_ctx_destroy(ctx);
    }
    if (fails) return 1;
    printf("abi_c99 ok (%s)\n", gpu ? "gpu" : "no gpu");
    return 0;
}
