/*
 * fmx_locate.c — a C host of the engine over include/fmx.h alone (no Python,
 * no torch): the reference bench's `locate` step.  A blob file is loaded
 * (bench/src/locate/sview_mmap.rs:17-45 + FmIndex::load, load_from_blob.rs:28-85:
 * here fmx_load_file), every line of a pattern file is located
 * (sview_memory.rs:30-34: FmIndex::locate per line; here one
 * fmx_locate_batch), and each pattern's locations are written comma-joined,
 * one line per pattern, in the order FmIndex::locate returns them
 * (write_locations_to_file, bench/src/locate/mod.rs:115-124).  Timings are
 * printed the way the reference bench prints them.
 *
 *   fmx_locate <blob> <pattern.txt> <results.txt> [--block2] [--direct] [--device N]
 *   fmx_locate --abi
 *
 * Layout: u32 positions, Block3<u64> (symbols ACGTN) or, with --block2,
 * Block2<u64> (ACGT, T as the wildcard) — the bench's two blobs
 * (bench/src/build/mod.rs:29-30), EncodingTable.
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "fmx.h"

static uint64_t now_ns(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

static int fail(const char *what, fmx_status st) {
    fprintf(stderr, "%s: %s (%d)\n", what, fmx_status_str(st), (int)st);
    return 1;
}

/* pattern.txt as BufRead::lines: '\n'-separated, a trailing '\r' dropped, no
 * empty last line after a final '\n'.  Returns the line count; bytes/offsets
 * are the packed batch (offsets[n] = total bytes). */
static uint64_t read_patterns(const char *path, uint8_t **bytes, uint64_t **offsets) {
    FILE *f = fopen(path, "rb");
    if (!f) return UINT64_MAX;
    fseek(f, 0, SEEK_END);
    const long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *raw = malloc((size_t)sz + 1);
    if (!raw || fread(raw, 1, (size_t)sz, f) != (size_t)sz) { fclose(f); free(raw); return UINT64_MAX; }
    fclose(f);
    uint64_t lines = 0;
    for (long i = 0; i < sz; ++i) lines += raw[i] == '\n';
    if (sz > 0 && raw[sz - 1] != '\n') ++lines;
    uint64_t *off = malloc((lines + 1) * sizeof(uint64_t));
    uint8_t *out = malloc((size_t)sz + 16);
    uint64_t n = 0, w = 0;
    long start = 0;
    off[0] = 0;
    for (long i = 0; i <= sz; ++i) {
        if (i == sz && start == sz) break;  /* no empty last line */
        if (i == sz || raw[i] == '\n') {
            long end = i;
            if (end > start && raw[end - 1] == '\r') --end;
            memcpy(out + w, raw + start, (size_t)(end - start));
            w += (uint64_t)(end - start);
            off[++n] = w;
            start = i + 1;
        }
    }
    free(raw);
    *bytes = out;
    *offsets = off;
    return n;
}

int main(int argc, char **argv) {
    if (argc == 2 && strcmp(argv[1], "--abi") == 0) {
        printf("fmx ABI %u\n", fmx_abi_version());
        return fmx_abi_version() == FMX_ABI_VERSION ? 0 : 1;
    }
    if (argc < 4) {
        fprintf(stderr, "usage: %s <blob> <pattern.txt> <results.txt> [--block2] [--direct] [--device N]\n", argv[0]);
        return 2;
    }
    int block2 = 0, direct = 0, device = 0;
    for (int i = 4; i < argc; ++i) {
        if (strcmp(argv[i], "--block2") == 0) block2 = 1;
        else if (strcmp(argv[i], "--direct") == 0) direct = 1;
        else if (strcmp(argv[i], "--device") == 0 && i + 1 < argc) device = atoi(argv[++i]);
        else { fprintf(stderr, "unknown argument %s\n", argv[i]); return 2; }
    }
    const fmx_layout layout = {4u, block2 ? 2u : 3u, 64u, FMX_ENC_TABLE};
    const uint64_t t_total = now_ns();
    uint64_t t0 = now_ns();
    fmx_index *ix = NULL;
    uint64_t expected = 0, actual = 0;
    fmx_status st = fmx_load_file(argv[1], layout, device, FMX_OPT_DEFAULT | (direct ? FMX_LOAD_DIRECT : 0u), 0,
                                  &ix, &expected, &actual);
    if (st == FMX_E_SIZE) {
        fprintf(stderr, "mismatched blob size: expected %" PRIu64 ", actual %" PRIu64 "\n", expected, actual);
        return 1;
    }
    if (st) return fail("fmx_load_file", st);
    const uint64_t load_ns = now_ns() - t0;

    t0 = now_ns();
    uint8_t *bytes = NULL;
    uint64_t *offsets = NULL;
    const uint64_t n = read_patterns(argv[2], &bytes, &offsets);
    if (n == UINT64_MAX) { fprintf(stderr, "cannot read %s\n", argv[2]); fmx_free(ix); return 1; }
    uint64_t *loc_off = malloc((n + 1) * sizeof(uint64_t));
    uint64_t cap = n + n / 8 + 4096, needed = 0;
    uint32_t *locs = malloc(cap * sizeof(uint32_t));
    st = fmx_locate_batch(ix, bytes, offsets, n, 0, loc_off, locs, cap, &needed);
    if (st == FMX_E_CAPACITY) {  /* two-phase: room for every location, then again */
        cap = needed;
        locs = realloc(locs, (cap ? cap : 1) * sizeof(uint32_t));
        st = fmx_locate_batch(ix, bytes, offsets, n, 0, loc_off, locs, cap, &needed);
    }
    if (st) { fmx_free(ix); return fail("fmx_locate_batch", st); }
    FILE *out = fopen(argv[3], "wb");
    if (!out) { fprintf(stderr, "cannot write %s\n", argv[3]); fmx_free(ix); return 1; }
    for (uint64_t i = 0; i < n; ++i) {
        for (uint64_t j = loc_off[i]; j < loc_off[i + 1]; ++j)
            fprintf(out, j + 1 < loc_off[i + 1] ? "%" PRIu32 "," : "%" PRIu32, locs[j]);
        fputc('\n', out);
    }
    fclose(out);
    const uint64_t locate_ns = now_ns() - t0;
    printf("Blob loading time: %" PRIu64 " ns\nLocate processing time: %" PRIu64 " ns\n", load_ns, locate_ns);
    printf("Results saved to: %s\nTotal time: %" PRIu64 " ns\n", argv[3], now_ns() - t_total);
    fmx_free(ix);
    free(bytes);
    free(offsets);
    free(loc_off);
    free(locs);
    return 0;
}
