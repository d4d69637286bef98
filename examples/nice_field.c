/*
 * nice_field.c -- a plain C (C99) host of the drop-in boundary: one field
 * through include/nice_hip.h and libnice_hip.so, nothing else (no Python, no
 * HIP headers).  It is what the reference client's field step does
 * (client/src/main.rs:120-207: process one claimed field, detailed or
 * niceonly, on the GPU with --gpu or on the CPU path without it) reduced to
 * one call per mode, and what a cgo / Rust FFI binding would do first.
 *
 *   nice_field [--gpu] [--device D] [--repeat R] [--no-timing] detailed|niceonly BASE START END
 *   nice_field [--gpu] [--device D] [--repeat R] [--no-timing] detailed|niceonly BASE range [SIZE]
 *
 * START / END are decimal u128; "range" takes the base's valid range
 * (get_base_range_u128, base_range.rs:14-54), truncated to SIZE numbers.
 * Prints "dist U COUNT" lines (detailed: bins 1..=base, zeros included, as
 * FieldResults.distribution), "nice N U" lines (ascending) and a "numbers
 * checked/sec" line (client/src/main.rs:363-370).  Without --gpu the
 * reference's CPU API is used (nice_cpu_process_range_*); with --gpu a
 * missing device is an error, never a silent CPU run.  --repeat R then calls
 * the same field R more times and prints the wall time per call (median and
 * minimum over the R calls, clock_gettime around the library call: what a
 * native caller waits) and, with --gpu detailed, the kernel time of each
 * (nice_last_kernel_stats, HIP events); --no-timing turns the context's kernel
 * timing off (nice_ctx_set_kernel_timing: no events per field).  Exit code: 0,
 * or the library's error code with nice_last_error() on stderr.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "nice_hip.h"

__extension__ typedef unsigned __int128 u128;  /* gcc: u128 as in the reference */

static int parse_u128(const char *s, u128 *out) {
    u128 v = 0;
    if (!*s) return 0;
    for (; *s; s++) {
        if (*s < '0' || *s > '9') return 0;
        const u128 d = (u128)(*s - '0');
        if (v > (~(u128)0 - d) / 10) return 0;
        v = v * 10 + d;
    }
    *out = v;
    return 1;
}

static void print_u128(FILE *f, u128 v) {
    char buf[48];
    int i = (int)sizeof buf - 1;
    buf[i] = 0;
    do {
        buf[--i] = (char)('0' + (int)(v % 10));
        v /= 10;
    } while (v);
    fputs(buf + i, f);
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int fail(int rc, const char *what) {
    fprintf(stderr, "nice_field: %s failed (%d): %s\n", what, rc, nice_last_error());
    return rc;
}

static int usage(void) {
    fprintf(stderr, "usage: nice_field [--gpu] [--device D] [--repeat R] [--no-timing] detailed|niceonly BASE "
                    "START END\n"
                    "       nice_field [--gpu] [--device D] [--repeat R] [--no-timing] detailed|niceonly BASE "
                    "range [SIZE]\n");
    return NICE_ERR_INVALID;
}

static int cmp_double(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

int main(int argc, char **argv) {
    int gpu = 0, device = 0, a = 1, repeat = 0, timing = 1;
    for (; a < argc && strncmp(argv[a], "--", 2) == 0; a++) {
        if (strcmp(argv[a], "--gpu") == 0) gpu = 1;
        else if (strcmp(argv[a], "--device") == 0 && a + 1 < argc) device = atoi(argv[++a]);
        else if (strcmp(argv[a], "--repeat") == 0 && a + 1 < argc) repeat = atoi(argv[++a]);
        else if (strcmp(argv[a], "--no-timing") == 0) timing = 0;
        else return usage();
    }
    if (argc - a < 3) return usage();
    const char *mode = argv[a];
    const int detailed = strcmp(mode, "detailed") == 0;
    if (!detailed && strcmp(mode, "niceonly") != 0) return usage();
    const uint32_t base = (uint32_t)strtoul(argv[a + 1], NULL, 10);
    u128 start, end;
    if (strcmp(argv[a + 2], "range") == 0) {
        uint64_t s_lo, s_hi, e_lo, e_hi;
        /* 1: a range, 0: none, -1: beyond u128 (get_base_range_u128's None) */
        if (nice_base_range(base, &s_lo, &s_hi, &e_lo, &e_hi) != 1) {
            fprintf(stderr, "nice_field: base %u has no u128 range\n", base);
            return NICE_ERR_INVALID;
        }
        start = ((u128)s_hi << 64) | s_lo;
        end = ((u128)e_hi << 64) | e_lo;
        u128 size;
        if (argc - a > 3) {
            if (!parse_u128(argv[a + 3], &size)) return usage();
            if (end - start > size) end = start + size;
        }
    } else {
        if (argc - a < 4 || !parse_u128(argv[a + 2], &start) || !parse_u128(argv[a + 3], &end)) return usage();
    }
    const uint64_t s_lo = (uint64_t)start, s_hi = (uint64_t)(start >> 64);
    const uint64_t e_lo = (uint64_t)end, e_hi = (uint64_t)(end >> 64);

    nice_ctx *ctx = NULL;
    if (gpu) {
        const int rc = nice_ctx_create(&device, 1, &ctx);
        if (rc != NICE_OK) return fail(rc, "nice_ctx_create");
        const int rt = timing ? NICE_OK : nice_ctx_set_kernel_timing(ctx, 0);
        if (rt != NICE_OK) {
            nice_ctx_destroy(ctx);
            return fail(rt, "nice_ctx_set_kernel_timing");
        }
    }
    uint64_t hist[129];
    memset(hist, 0, sizeof hist);
    size_t cap = 1024, n = 0;
    nice_number *list = NULL;
    int rc;
    double t0 = 0.0, t1 = 0.0;
    for (;;) {  /* NICE_ERR_CAPACITY: *n_out is the length needed */
        nice_number *grown = (nice_number *)realloc(list, cap * sizeof *list);
        if (!grown) {
            free(list);
            if (ctx) nice_ctx_destroy(ctx);
            fprintf(stderr, "nice_field: out of memory for %zu entries\n", cap);
            return NICE_ERR_CAPACITY;
        }
        list = grown;
        t0 = now_s();
        if (detailed && gpu)
            rc = nice_process_range_detailed(ctx, s_lo, s_hi, e_lo, e_hi, base, hist, list, cap, &n);
        else if (detailed)
            rc = nice_cpu_process_range_detailed(s_lo, s_hi, e_lo, e_hi, base, 0, hist, list, cap, &n);
        else if (gpu)
            rc = nice_process_range_niceonly(ctx, s_lo, s_hi, e_lo, e_hi, base, list, cap, &n);
        else
            rc = nice_cpu_process_range_niceonly(s_lo, s_hi, e_lo, e_hi, base, 0, 0, list, cap, &n);
        t1 = now_s();
        if (rc != NICE_ERR_CAPACITY || n <= cap) break;
        cap = n;
    }
    if (rc != NICE_OK) {
        free(list);
        if (ctx) nice_ctx_destroy(ctx);
        return fail(rc, detailed ? "detailed" : "niceonly");
    }
    printf("base %u range ", base);
    print_u128(stdout, start);
    printf(" ");
    print_u128(stdout, end);
    printf(" mode %s path %s\n", mode, gpu ? "gpu" : "cpu");
    if (detailed)
        for (uint32_t u = 1; u <= base; u++) printf("dist %u %llu\n", u, (unsigned long long)hist[u]);
    for (size_t i = 0; i < n; i++) {
        printf("nice ");
        print_u128(stdout, ((u128)list[i].number_hi << 64) | list[i].number_lo);
        printf(" %u\n", list[i].num_uniques);
    }
    const double secs = t1 - t0;
    printf("numbers checked/sec %.6g (%.6f s)\n", secs > 0 ? (double)(end - start) / secs : 0.0, secs);
    if (repeat > 0) {
        double *wall = (double *)malloc((size_t)repeat * sizeof *wall);
        double *kern = (double *)malloc((size_t)repeat * sizeof *kern);
        int nk = 0;
        for (int r = 0; r < repeat && rc == NICE_OK; r++) {
            size_t m = 0;
            t0 = now_s();
            if (detailed && gpu)
                rc = nice_process_range_detailed(ctx, s_lo, s_hi, e_lo, e_hi, base, hist, list, cap, &m);
            else if (detailed)
                rc = nice_cpu_process_range_detailed(s_lo, s_hi, e_lo, e_hi, base, 0, hist, list, cap, &m);
            else if (gpu)
                rc = nice_process_range_niceonly(ctx, s_lo, s_hi, e_lo, e_hi, base, list, cap, &m);
            else
                rc = nice_cpu_process_range_niceonly(s_lo, s_hi, e_lo, e_hi, base, 0, 0, list, cap, &m);
            wall[r] = now_s() - t0;
            if (rc == NICE_OK && m != n) rc = NICE_ERR_INVALID;  /* the same field, the same list */
            nice_kernel_stats ks;
            if (rc == NICE_OK && detailed && gpu && timing && nice_last_kernel_stats(ctx, 0, &ks) == NICE_OK)
                kern[nk++] = ks.kernel_ms * 1e-3;
        }
        if (rc != NICE_OK) {
            free(wall);
            free(kern);
            free(list);
            if (ctx) nice_ctx_destroy(ctx);
            return fail(rc, "repeat");
        }
        qsort(wall, (size_t)repeat, sizeof *wall, cmp_double);
        printf("repeat %d: wall per call median %.2f us, min %.2f us", repeat, wall[repeat / 2] * 1e6,
               wall[0] * 1e6);
        if (nk) {
            qsort(kern, (size_t)nk, sizeof *kern, cmp_double);
            printf("; kernel median %.2f us", kern[nk / 2] * 1e6);
        }
        printf("\n");
        free(wall);
        free(kern);
    }
    free(list);
    if (ctx) nice_ctx_destroy(ctx);
    return 0;
}
