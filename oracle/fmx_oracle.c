/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see fmx_oracle.h for the rules and the
 * parity pins).  A plain-C restatement of baku4/sview-fmindex; every function
 * cites the reference file:line it follows (paths relative to
 * /root/reference/sview-fmindex/).
 */
#include "fmx_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ---------------------------------------------------------------- helpers */

/* Aligned::aligned_size — src/components/mod.rs:1-9 */
static uint64_t align_up(uint64_t raw, uint64_t a) {
    uint64_t r = raw % a;
    return r == 0 ? raw : raw + (a - r);
}

static uint64_t rd_u64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static uint32_t rd_u32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static void wr_u64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }
static void wr_u32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }

/* Position P read/write (text_length.rs:10-129): P is u32 or u64. */
static uint64_t rd_p(const uint8_t *base, uint64_t i, uint32_t pb) {
    return pb == 4 ? (uint64_t)rd_u32(base + 4 * i) : rd_u64(base + 8 * i);
}
static void wr_p(uint8_t *base, uint64_t i, uint32_t pb, uint64_t v) {
    if (pb == 4) wr_u32(base + 4 * i, (uint32_t)v); else wr_u64(base + 8 * i, v);
}
/* P arithmetic wraps at the type's width (release-mode Rust). */
static uint64_t pmask(uint32_t pb) { return pb == 4 ? 0xFFFFFFFFull : ~0ull; }

static int layout_ok(orc_layout L) {
    if (L.pos_bytes != 4 && L.pos_bytes != 8) return 0;
    if (L.planes < 2 || L.planes > 6) return 0;
    if (L.vec_bits != 32 && L.vec_bits != 64 && L.vec_bits != 128) return 0;
    if (L.encoder > 1) return 0;
    return 1;
}
/* Vector::ALIGN_SIZE — blocks/vector.rs:16-17,31-32,46-47 (u32 aligns to 8) */
static uint32_t align_of(orc_layout L) { return L.vec_bits == 128 ? 16 : 8; }

/* One plane V_j of a block, little-endian #[repr(C)] [V; N] (blocks/block3.rs:4-7) */
static u128 rd_vec(const uint8_t *p, uint32_t vec_bytes) {
    u128 v = 0;
    memcpy(&v, p, vec_bytes);
    return v;
}
static u128 vec_all(uint32_t bl) { return bl == 128 ? ~(u128)0 : (((u128)1 << bl) - 1); }
static uint32_t popc128(u128 x) {
    return (uint32_t)__builtin_popcountll((uint64_t)x) + (uint32_t)__builtin_popcountll((uint64_t)(x >> 64));
}

/* ------------------------------------------------------------------- load */

/* FmIndex::load — src/load_from_blob.rs:28-85, with the header readers of
 * components/mod.rs:11-22, magic_number.rs:38-47, count_array.rs:151-191,
 * suffix_array/mod.rs:78-91, bwm/mod.rs:145-190.  The reference panics where a
 * header read runs off the blob or a slice is misaligned; this returns codes. */
int orc_load(const uint8_t *blob, uint64_t len, orc_layout L, orc_index *ix,
             uint64_t *expected_total, uint64_t *actual_total) {
    memset(ix, 0, sizeof(*ix));
    if (!layout_ok(L)) return ORC_E_LAYOUT;
    const uint64_t A = align_of(L);
    const uint32_t pb = L.pos_bytes;
    ix->L = L; ix->blob = blob; ix->blob_len = len;
    ix->bl = L.vec_bits; ix->align = (uint32_t)A;
    ix->block_bytes = L.planes * (L.vec_bits / 8);
    if (((uintptr_t)blob) % A != 0) return ORC_E_ALIGN;

    uint64_t off = 0;
    /* MagicNumber "FI00" + 4 pad bytes (magic_number.rs:3-25, 38-47) */
    if (len < 8) return ORC_E_FORMAT;
    if (!(blob[0] == 'F' && blob[1] == 'I' && blob[2] == '0' && blob[3] == '0')) return ORC_E_FORMAT;
    off = align_up(8, A);
    /* TextEncoder header: EncodingTable([u8;256]) or PassThrough (ZST) */
    if (L.encoder == 0) {
        if (off + 256 > len) return ORC_E_FORMAT;
        memcpy(ix->enc, blob + off, 256);
        off += align_up(256, A);
    } else {
        for (int i = 0; i < 256; ++i) ix->enc[i] = (uint8_t)i;
    }
    /* CountArrayHeader (count_array.rs:6-18): u32 x4 + u64 = 24 B */
    if (off + 24 > len) return ORC_E_FORMAT;
    uint32_t ca_sigma = rd_u32(blob + off), ca_k = rd_u32(blob + off + 4);
    uint32_t ca_len = rd_u32(blob + off + 8), mult_len = rd_u32(blob + off + 12);
    uint64_t kt_len = rd_u64(blob + off + 16);
    off += align_up(24, A);
    /* SuffixArrayHeader (suffix_array/mod.rs:9-18): u32, pad u32, u64 = 16 B */
    if (off + 16 > len) return ORC_E_FORMAT;
    uint32_t sr = rd_u32(blob + off);
    uint64_t sa_len = rd_u64(blob + off + 8);
    off += align_up(16, A);
    /* BwmHeader (bwm/mod.rs:9-16): u32, pad u32, u64, u64 = 24 B */
    if (off + 24 > len) return ORC_E_FORMAT;
    uint32_t bw_sigma = rd_u32(blob + off);
    uint64_t ckpt_len = rd_u64(blob + off + 8), blocks_len = rd_u64(blob + off + 16);
    off += align_up(24, A);
    const uint64_t header_size = off;

    /* body size check (load_from_blob.rs:40-58) — guard the products first */
    if (ca_len > (1u << 20) || mult_len > 64 || kt_len > (1ull << 40) || sa_len > (1ull << 40) ||
        ckpt_len > (1ull << 46) || blocks_len > (1ull << 40))
        return ORC_E_LAYOUT;
    uint64_t body_ca = align_up((uint64_t)ca_len * pb, A) + align_up((uint64_t)mult_len * 8, A) +
                       align_up(kt_len * pb, A);
    uint64_t body_sa = align_up(sa_len * pb, A);
    uint64_t body_bwm = align_up(pb, A) + align_up(ckpt_len * pb, A) + align_up(blocks_len * ix->block_bytes, A);
    uint64_t expected_body = body_ca + body_sa + body_bwm;
    uint64_t actual_body = len - header_size;
    if (expected_total) *expected_total = header_size + expected_body;
    if (actual_total) *actual_total = len;
    if (actual_body != expected_body) return ORC_E_SIZE;

    /* slices */
    ix->off_count_array = header_size;
    ix->off_mult = ix->off_count_array + align_up((uint64_t)ca_len * pb, A);
    ix->off_kmer = ix->off_mult + align_up((uint64_t)mult_len * 8, A);
    ix->off_sa = ix->off_kmer + align_up(kt_len * pb, A);
    ix->off_sentinel = ix->off_sa + body_sa;
    ix->off_ckpt = ix->off_sentinel + align_up(pb, A);
    ix->off_blocks = ix->off_ckpt + align_up(ckpt_len * pb, A);

    /* Consistency checks the reference leaves implicit (its type parameters are
     * not stored in the blob): the layout tag must agree with the header sizes. */
    ix->sigma = ca_sigma; ix->k = ca_k; ix->sr = sr;
    if (ca_sigma == 0 || ca_sigma > 64 || ca_sigma > (1u << L.planes)) return ORC_E_LAYOUT;
    if (ca_sigma != bw_sigma || ca_len != ca_sigma + 1 || mult_len != ca_k || ca_k == 0 || sr == 0)
        return ORC_E_LAYOUT;
    for (uint32_t c = 0; c <= ca_sigma; ++c) ix->count_array[c] = rd_p(blob + ix->off_count_array, c, pb);
    ix->n = ix->count_array[ca_sigma];
    uint64_t W = ca_sigma + 1, wk = 1;
    for (uint32_t i = 0; i < ca_k; ++i) {
        if (wk > (1ull << 40) / W) return ORC_E_LAYOUT;
        wk *= W;
    }
    if (kt_len != wk) return ORC_E_LAYOUT;
    uint64_t p = 1;
    for (uint32_t i = 0; i < ca_k; ++i) { /* mult = [W^(k-1) .. W^0] (count_array.rs:89-93) */
        ix->mult[ca_k - 1 - i] = p;
        if (rd_u64(blob + ix->off_mult + 8 * (ca_k - 1 - i)) != p) return ORC_E_LAYOUT;
        p *= W;
    }
    if (blocks_len != ix->n / ix->bl + 1 || ckpt_len != blocks_len * ca_sigma) return ORC_E_LAYOUT;
    if (sa_len != (ix->n + sr - 1) / sr) return ORC_E_LAYOUT;
    ix->kmer_table = blob + ix->off_kmer; ix->kmer_len = kt_len;
    ix->sa = blob + ix->off_sa; ix->sa_len = sa_len;
    ix->sentinel = rd_p(blob + ix->off_sentinel, 0, pb);
    if (ix->n > 0 && (ix->sentinel == 0 || ix->sentinel > ix->n)) return ORC_E_LAYOUT;
    ix->ckpt = blob + ix->off_ckpt; ix->ckpt_len = ckpt_len;
    ix->blocks = blob + ix->off_blocks; ix->blocks_len = blocks_len;
    return ORC_OK;
}

/* ------------------------------------------------------------ block codec */

/* Block::get_remain_count_of — blocks/block2.rs:38-47, block3.rs:42-55,
 * block4.rs:46-67, block5.rs:50-87, block6.rs:54-123: AND of the planes (or
 * their complements, by the bits of the symbol index), shifted right by
 * BLOCK_LEN - rem, popcount.  rem is in [1, BLOCK_LEN). */
static uint32_t remain_count(const orc_index *ix, uint64_t q, uint32_t rem, uint32_t c) {
    const uint32_t vb = ix->bl / 8;
    const uint8_t *b = ix->blocks + q * ix->block_bytes;
    const u128 all = vec_all(ix->bl);
    u128 m = all;
    for (uint32_t j = 0; j < ix->L.planes; ++j) {
        u128 v = rd_vec(b + j * vb, vb);
        m &= ((c >> j) & 1) ? v : (~v & all);
    }
    m >>= (ix->bl - rem);
    return popc128(m);
}

/* Block::get_symidx_of — block3.rs:57-63 (and siblings): bit BLOCK_LEN-1-rem of
 * plane j is bit j of the symbol index (MSB-first within a block). */
static uint32_t symidx_of(const orc_index *ix, uint64_t q, uint32_t rem) {
    const uint32_t vb = ix->bl / 8;
    const uint8_t *b = ix->blocks + q * ix->block_bytes;
    const uint32_t mov = ix->bl - rem - 1;
    uint32_t s = 0;
    for (uint32_t j = 0; j < ix->L.planes; ++j) {
        u128 v = rd_vec(b + j * vb, vb);
        s |= (uint32_t)((v >> mov) & 1) << j;
    }
    return s;
}

/* BwmView::get_next_rank — components/bwm/mod.rs:197-215 */
static uint64_t next_rank(const orc_index *ix, uint64_t pos, uint32_t c) {
    if (pos < ix->sentinel) pos += 1;
    uint64_t q = pos / ix->bl;
    uint32_t rem = (uint32_t)(pos % ix->bl);
    uint64_t r = rd_p(ix->ckpt, q * ix->sigma + c, ix->L.pos_bytes);
    if (rem != 0) r += remain_count(ix, q, rem, c);
    return r & pmask(ix->L.pos_bytes);
}

/* BwmView::get_pre_rank_and_symidx — components/bwm/mod.rs:217-236.
 * Returns 0 for the text-start row (None), 1 otherwise. */
static int pre_rank_and_symidx(const orc_index *ix, uint64_t pos, uint64_t *rank, uint32_t *sym) {
    const uint64_t pm = pmask(ix->L.pos_bytes);
    if (pos == ((ix->sentinel - 1) & pm)) return 0;
    if (pos < ix->sentinel) pos += 1;
    uint64_t q = pos / ix->bl;
    uint32_t rem = (uint32_t)(pos % ix->bl);
    uint32_t c = symidx_of(ix, q, rem);
    uint64_t r = rd_p(ix->ckpt, q * ix->sigma + c, ix->L.pos_bytes);
    if (rem != 0) r += remain_count(ix, q, rem, c);
    *rank = r & pm;
    *sym = c;
    return 1;
}

/* -------------------------------------------------------------- query path */

static int check_sym(const orc_index *ix, uint8_t byte) {
    /* PassThrough::idx_of is the identity (pass_through.rs:6-12); a byte >=
     * symbol_count indexes past the C-array in the reference (panic / UB). */
    return ix->enc[byte] < ix->sigma;
}

/* CountArrayView::get_initial_pos_range_and_idx_of_pattern — count_array.rs:203-233 */
static int initial_range(const orc_index *ix, const uint8_t *pat, uint64_t m,
                         uint64_t *lo, uint64_t *hi, uint64_t *idx) {
    const uint32_t pb = ix->L.pos_bytes;
    if (m == 0) return ORC_E_EMPTY_PATTERN; /* pattern_len - 1 underflows (count_array.rs:211) */
    const uint64_t k = ix->k;
    if (m < k) {
        uint64_t s = 0;
        for (uint64_t i = 0; i < m; ++i) {
            if (!check_sym(ix, pat[i])) return ORC_E_SYMBOL;
            s += (uint64_t)(ix->enc[pat[i]] + 1) * ix->mult[i];
        }
        uint64_t e = s + ix->mult[m - 1] - 1;
        *lo = rd_p(ix->kmer_table, s - 1, pb);
        *hi = rd_p(ix->kmer_table, e, pb);
        *idx = 0;
    } else {
        const uint8_t *sl = pat + (m - k);
        uint64_t s = 0;
        for (uint64_t i = 0; i < k; ++i) {
            if (!check_sym(ix, sl[i])) return ORC_E_SYMBOL;
            s += (uint64_t)(ix->enc[sl[i]] + 1) * ix->mult[i];
        }
        *lo = rd_p(ix->kmer_table, s - 1, pb);
        *hi = rd_p(ix->kmer_table, s, pb);
        *idx = m - k;
    }
    return ORC_OK;
}

/* FmIndex::get_pos_range — locate/with_slice.rs:21-33, with next_pos_range
 * (locate/mod.rs:38-45). */
static int pos_range(const orc_index *ix, const uint8_t *pat, uint64_t m, uint64_t *plo, uint64_t *phi) {
    uint64_t lo, hi, idx;
    int st = initial_range(ix, pat, m, &lo, &hi, &idx);
    if (st) return st;
    const uint64_t pm = pmask(ix->L.pos_bytes);
    while (lo < hi && idx > 0) {
        idx -= 1;
        uint8_t sym = pat[idx];
        if (!check_sym(ix, sym)) return ORC_E_SYMBOL;
        uint32_t c = ix->enc[sym];
        uint64_t pre = ix->count_array[c];
        uint64_t a = next_rank(ix, lo, c), b = next_rank(ix, hi, c);
        lo = (pre + a) & pm;
        hi = (pre + b) & pm;
    }
    *plo = lo; *phi = hi;
    return ORC_OK;
}

/* get_initial_pos_range_and_idx_of_pattern_rev_iter — count_array.rs:235-274,
 * and get_pos_range_from_rev_iter — locate/with_rev_iter.rs:66-84. */
static int pos_range_rev(const orc_index *ix, const uint8_t *rev, uint64_t m, uint64_t *plo, uint64_t *phi) {
    const uint32_t pb = ix->L.pos_bytes;
    const uint64_t k = ix->k, W = ix->sigma + 1, pm = pmask(pb);
    uint64_t it = 0, sz = 0, s = 0, lo, hi;
    while (sz < k) {
        if (it < m) {
            uint8_t sym = rev[it++];
            if (!check_sym(ix, sym)) return ORC_E_SYMBOL;
            sz += 1;
            s += (uint64_t)(ix->enc[sym] + 1) * ix->mult[k - sz];
        } else {
            if (sz == 0) return ORC_E_EMPTY_PATTERN; /* kmer_multiplier[-1] panics */
            for (uint64_t i = 0; i < k - sz; ++i) s *= W;
            uint64_t e = s + ix->mult[sz - 1] - 1;
            *plo = rd_p(ix->kmer_table, s - 1, pb);
            *phi = rd_p(ix->kmer_table, e, pb);
            return ORC_OK;
        }
    }
    lo = rd_p(ix->kmer_table, s - 1, pb);
    hi = rd_p(ix->kmer_table, s, pb);
    while (lo < hi) {
        if (it >= m) break;
        uint8_t sym = rev[it++];
        if (!check_sym(ix, sym)) return ORC_E_SYMBOL;
        uint32_t c = ix->enc[sym];
        uint64_t pre = ix->count_array[c];
        uint64_t a = next_rank(ix, lo, c), b = next_rank(ix, hi, c);
        lo = (pre + a) & pm;
        hi = (pre + b) & pm;
    }
    *plo = lo; *phi = hi;
    return ORC_OK;
}

/* FmIndex::count — locate/with_slice.rs:5-8 */
int orc_count(const orc_index *ix, const uint8_t *pat, uint64_t m, uint64_t *out_count) {
    uint64_t lo, hi;
    int st = pos_range(ix, pat, m, &lo, &hi);
    if (st) return st;
    *out_count = (hi - lo) & pmask(ix->L.pos_bytes);
    return ORC_OK;
}

/* FmIndex::count_rev_iter — locate/with_rev_iter.rs:5-9 */
int orc_count_rev(const orc_index *ix, const uint8_t *rev, uint64_t m, uint64_t *out_count) {
    uint64_t lo, hi;
    int st = pos_range_rev(ix, rev, m, &lo, &hi);
    if (st) return st;
    *out_count = (hi - lo) & pmask(ix->L.pos_bytes);
    return ORC_OK;
}

/* FmIndex::write_locations_to_buffer — locate/mod.rs:14-37: rows lo..hi in
 * ascending order, each walked by LF to a sampled row (pos % sr == 0) or to the
 * text-start row (pos == sentinel_index - 1, location = offset). */
static void walk_rows(const orc_index *ix, uint64_t lo, uint64_t hi, uint64_t *out, uint64_t cap) {
    const uint32_t pb = ix->L.pos_bytes;
    const uint64_t pm = pmask(pb), sr = ix->sr;
    uint64_t j = 0;
    for (uint64_t row = lo; row < hi; ++row, ++j) {
        uint64_t pos = row, off = 0, loc;
        int done = 0;
        while (pos % sr != 0) {
            uint64_t rank; uint32_t c;
            if (!pre_rank_and_symidx(ix, pos, &rank, &c)) { loc = off; done = 1; break; }
            pos = (ix->count_array[c] + rank) & pm;
            off += 1;
        }
        if (!done) loc = (rd_p(ix->sa, pos / sr, pb) + off) & pm; /* suffix_array/mod.rs:100-105 */
        if (j < cap) out[j] = loc;
    }
}

/* FmIndex::locate — locate/with_slice.rs:10-13 */
int orc_locate(const orc_index *ix, const uint8_t *pat, uint64_t m,
               uint64_t *out_locs, uint64_t cap, uint64_t *out_count) {
    uint64_t lo, hi;
    int st = pos_range(ix, pat, m, &lo, &hi);
    if (st) return st;
    *out_count = hi - lo;
    walk_rows(ix, lo, hi, out_locs, cap);
    return (hi - lo) > cap ? ORC_E_CAPACITY : ORC_OK;
}

/* ------------------------------------------------------ threaded batches */

typedef struct {
    const orc_index *ix;
    const uint8_t *bytes;
    const uint64_t *offsets;
    uint64_t begin, end;
    void *out_counts;        /* count phase */
    const uint64_t *loc_off; /* locate phase */
    void *out_locs;
    int mode; /* 0 = count (also records lo), 1 = locate rows */
    uint64_t *lo_buf;
    int status;
} orc_job;

static void *job_run(void *arg) {
    orc_job *J = (orc_job *)arg;
    const orc_index *ix = J->ix;
    const uint32_t pb = ix->L.pos_bytes;
    uint64_t tmp[64];
    for (uint64_t i = J->begin; i < J->end; ++i) {
        const uint8_t *p = J->bytes + J->offsets[i];
        uint64_t m = J->offsets[i + 1] - J->offsets[i];
        if (J->mode == 0) {
            uint64_t lo, hi;
            int st = pos_range(ix, p, m, &lo, &hi);
            if (st) { J->status = st; return NULL; }
            wr_p((uint8_t *)J->out_counts, i, pb, (hi - lo) & pmask(pb));
            if (J->lo_buf) J->lo_buf[i] = lo;
        } else {
            uint64_t lo = J->lo_buf[i], cnt = J->loc_off[i + 1] - J->loc_off[i];
            uint64_t base = J->loc_off[i];
            /* walk in chunks through a small stack buffer, then widen to P */
            for (uint64_t s = 0; s < cnt; s += 64) {
                uint64_t e = cnt - s < 64 ? cnt - s : 64;
                walk_rows(ix, lo + s, lo + s + e, tmp, 64);
                for (uint64_t t = 0; t < e; ++t) wr_p((uint8_t *)J->out_locs, base + s + t, pb, tmp[t]);
            }
        }
    }
    return NULL;
}

static int run_jobs(orc_job *tmpl, uint64_t n, int threads) {
    if (threads < 1) threads = 1;
    if ((uint64_t)threads > n && n > 0) threads = (int)n;
    if (n == 0) return ORC_OK;
    orc_job *jobs = (orc_job *)calloc((size_t)threads, sizeof(orc_job));
    pthread_t *tids = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    uint64_t per = (n + threads - 1) / threads;
    for (int t = 0; t < threads; ++t) {
        jobs[t] = *tmpl;
        jobs[t].begin = per * t < n ? per * t : n;
        jobs[t].end = per * (t + 1) < n ? per * (t + 1) : n;
        jobs[t].status = ORC_OK;
        if (threads == 1) job_run(&jobs[t]);
        else pthread_create(&tids[t], NULL, job_run, &jobs[t]);
    }
    int st = ORC_OK;
    for (int t = 0; t < threads; ++t) {
        if (threads > 1) pthread_join(tids[t], NULL);
        if (jobs[t].status && !st) st = jobs[t].status;
    }
    free(jobs);
    free(tids);
    return st;
}

int orc_count_batch(const orc_index *ix, const uint8_t *bytes, const uint64_t *offsets,
                    uint64_t n, void *out_counts, int threads) {
    orc_job J;
    memset(&J, 0, sizeof(J));
    J.ix = ix; J.bytes = bytes; J.offsets = offsets; J.out_counts = out_counts; J.mode = 0;
    return run_jobs(&J, n, threads);
}

int orc_locate_batch(const orc_index *ix, const uint8_t *bytes, const uint64_t *offsets,
                     uint64_t n, uint64_t *out_loc_offsets, void *out_locs,
                     uint64_t cap, uint64_t *needed, int threads) {
    const uint32_t pb = ix->L.pos_bytes;
    uint8_t *counts = (uint8_t *)malloc((size_t)(n ? n : 1) * pb);
    uint64_t *lo = (uint64_t *)malloc((size_t)(n ? n : 1) * 8);
    orc_job J;
    memset(&J, 0, sizeof(J));
    J.ix = ix; J.bytes = bytes; J.offsets = offsets; J.out_counts = counts; J.mode = 0; J.lo_buf = lo;
    int st = run_jobs(&J, n, threads);
    if (st) { free(counts); free(lo); return st; }
    uint64_t acc = 0;
    for (uint64_t i = 0; i < n; ++i) {
        out_loc_offsets[i] = acc;
        acc += rd_p(counts, i, pb);
    }
    out_loc_offsets[n] = acc;
    if (needed) *needed = acc;
    if (acc > cap) { free(counts); free(lo); return ORC_E_CAPACITY; }
    J.mode = 1; J.loc_off = out_loc_offsets; J.out_locs = out_locs;
    st = run_jobs(&J, n, threads);
    free(counts);
    free(lo);
    return st;
}

/* ---------------------------------------------------------------- builder */

typedef struct {
    uint64_t magic, enc, cah, sah, bwh, header;
    uint64_t ca_raw, ca, mult_raw, mult, kt_raw, kt, sa_len, sa_raw, sa, sent, ckpt_len, ckpt_raw, ckpt,
        blocks_len, blocks_raw, blocks, total;
} orc_sizes;

/* FmIndexBuilder::generate_headers + blob_size — builder/mod.rs:100-181,
 * CountArrayHeader::new (count_array.rs:57-77), SuffixArrayHeader::new
 * (suffix_array/mod.rs:43-56), BwmHeader::new (bwm/mod.rs:69-90). */
static int sizes_of(uint64_t n, uint32_t sigma, orc_layout L, uint32_t k, uint32_t sr, orc_sizes *S) {
    if (!layout_ok(L)) return ORC_E_LAYOUT;
    if (sigma == 0 || sigma > (1u << L.planes)) return ORC_E_SYMBOL; /* BuildError::SymbolCountOver */
    if (k == 0 || sr == 0) return ORC_E_CONFIG;                     /* InvalidConfig */
    const uint64_t A = align_of(L), pb = L.pos_bytes, W = sigma + 1;
    uint64_t wk = 1;
    for (uint32_t i = 0; i < k; ++i) {
        wk *= W;
        if (wk > 0xFFFFFFFFull) return ORC_E_CONFIG; /* u32::pow overflow in count_array.rs:68 */
    }
    memset(S, 0, sizeof(*S));
    S->magic = align_up(8, A);
    S->enc = L.encoder == 0 ? align_up(256, A) : 0;
    S->cah = align_up(24, A);
    S->sah = align_up(16, A);
    S->bwh = align_up(24, A);
    S->header = S->magic + S->enc + S->cah + S->sah + S->bwh;
    S->ca_raw = W * pb; S->ca = align_up(S->ca_raw, A);
    S->mult_raw = (uint64_t)k * 8; S->mult = align_up(S->mult_raw, A);
    S->kt_raw = wk * pb; S->kt = align_up(S->kt_raw, A);
    S->sa_len = (n + sr - 1) / sr; S->sa_raw = S->sa_len * pb; S->sa = align_up(S->sa_raw, A);
    S->sent = align_up(pb, A);
    S->blocks_len = n / L.vec_bits + 1;
    S->ckpt_len = S->blocks_len * sigma; S->ckpt_raw = S->ckpt_len * pb; S->ckpt = align_up(S->ckpt_raw, A);
    S->blocks_raw = S->blocks_len * L.planes * (L.vec_bits / 8); S->blocks = align_up(S->blocks_raw, A);
    S->total = S->header + S->ca + S->mult + S->kt + S->sa + S->sent + S->ckpt + S->blocks;
    return ORC_OK;
}

int orc_blob_size(uint64_t text_len, uint32_t sigma, orc_layout L, uint32_t k, uint32_t sr, uint64_t *out_size) {
    orc_sizes S;
    int st = sizes_of(text_len, sigma, L, k, sr, &S);
    if (st) return st;
    *out_size = S.total;
    return ORC_OK;
}

/* Suffix array by prefix doubling with two counting sorts per round.  The
 * reference builds it with SA-IS (crate_bio_manual/suffix_array.rs:39-60) or
 * libdivsufsort; the suffix array of a string ending in a unique smallest
 * sentinel is unique, so any correct construction gives the same array. */
int orc_suffix_array(const uint8_t *t, uint64_t len, uint32_t alphabet, uint64_t *sa) {
    if (len == 0) return ORC_OK;
    uint64_t *rank = (uint64_t *)malloc(len * 8), *tmp = (uint64_t *)malloc(len * 8);
    uint64_t cn = len > alphabet ? len : alphabet;
    uint64_t *cnt = (uint64_t *)malloc((cn + 1) * 8);
    if (!rank || !tmp || !cnt) { free(rank); free(tmp); free(cnt); return ORC_E_CONFIG; }
    memset(cnt, 0, (alphabet + 1) * 8);
    for (uint64_t i = 0; i < len; ++i) cnt[t[i] + 1]++;
    for (uint32_t c = 0; c < alphabet; ++c) cnt[c + 1] += cnt[c];
    for (uint64_t i = 0; i < len; ++i) sa[cnt[t[i]]++] = i;
    /* rank = index of the first suffix of the group */
    rank[sa[0]] = 0;
    for (uint64_t r = 1; r < len; ++r)
        rank[sa[r]] = t[sa[r]] == t[sa[r - 1]] ? rank[sa[r - 1]] : r;
    for (uint64_t h = 1;; h <<= 1) {
        /* sorted by second key (rank[i+h], absent = smallest) */
        uint64_t j = 0;
        for (uint64_t i = len - (h < len ? h : len); i < len; ++i) tmp[j++] = i;
        for (uint64_t r = 0; r < len; ++r)
            if (sa[r] >= h) tmp[j++] = sa[r] - h;
        /* stable counting sort by first key rank[] (ranks are group starts in [0,len)) */
        memset(cnt, 0, (len + 1) * 8);
        for (uint64_t i = 0; i < len; ++i) cnt[rank[i]]++;
        uint64_t acc = 0;
        for (uint64_t r = 0; r < len; ++r) { uint64_t c = cnt[r]; cnt[r] = acc; acc += c; }
        for (uint64_t i = 0; i < len; ++i) { uint64_t s = tmp[i]; sa[cnt[rank[s]]++] = s; }
        /* new ranks */
        tmp[sa[0]] = 0;
        int all_unique = 1;
        for (uint64_t r = 1; r < len; ++r) {
            uint64_t a = sa[r - 1], b = sa[r];
            uint64_t ra2 = a + h < len ? rank[a + h] + 1 : 0, rb2 = b + h < len ? rank[b + h] + 1 : 0;
            if (rank[a] == rank[b] && ra2 == rb2) { tmp[b] = tmp[a]; all_unique = 0; }
            else tmp[b] = r;
        }
        memcpy(rank, tmp, len * 8);
        if (all_unique) break;
    }
    free(rank); free(tmp); free(cnt);
    return ORC_OK;
}

/* FmIndexBuilder::build — builder/mod.rs:187-264. */
int orc_build(const uint8_t *text, uint64_t n, const uint8_t *table, uint32_t sigma,
              orc_layout L, uint32_t k, uint32_t sr, uint8_t *blob, uint64_t blob_len) {
    orc_sizes S;
    L.encoder = table ? 0 : 1;
    int st = sizes_of(n, sigma, L, k, sr, &S);
    if (st) return st;
    const uint64_t A = align_of(L), pb = L.pos_bytes, W = sigma + 1, BL = L.vec_bits;
    if (((uintptr_t)blob) % A != 0) return ORC_E_ALIGN;   /* NotAlignedBlob */
    if (blob_len != S.total) return ORC_E_CONFIG;        /* InvalidBlobSize */
    /* padding bytes are zero (the reference's callers hand it vec![0; size]) */
    memset(blob, 0, blob_len);

    /* 1) headers (builder/mod.rs:211-231) */
    uint8_t *h = blob;
    h[0] = 'F'; h[1] = 'I'; h[2] = '0'; h[3] = '0';
    h += S.magic;
    if (table) { memcpy(h, table, 256); h += S.enc; }
    wr_u32(h, sigma); wr_u32(h + 4, k); wr_u32(h + 8, (uint32_t)W); wr_u32(h + 12, k);
    uint64_t wk = 1;
    for (uint32_t i = 0; i < k; ++i) wk *= W;
    wr_u64(h + 16, wk);
    h += S.cah;
    wr_u32(h, sr); wr_u64(h + 8, S.sa_len);
    h += S.sah;
    wr_u32(h, sigma); wr_u64(h + 8, S.ckpt_len); wr_u64(h + 16, S.blocks_len);

    uint8_t *body = blob + S.header;
    uint8_t *ca = body, *mult = ca + S.ca, *kt = mult + S.mult, *sa_out = kt + S.kt;
    uint8_t *sent = sa_out + S.sa, *ckpt = sent + S.sent, *blocks = ckpt + S.ckpt;

    /* 2) count_and_encode_text — count_array.rs:78-136 */
    uint8_t *t = (uint8_t *)malloc(n + 1);
    uint64_t *cnt = (uint64_t *)calloc(W, 8);
    uint64_t *kc = (uint64_t *)calloc(wk, 8);
    uint64_t *mul = (uint64_t *)malloc(8 * (k ? k : 1));
    if (!t || !cnt || !kc || !mul) { free(t); free(cnt); free(kc); free(mul); return ORC_E_CONFIG; }
    { uint64_t p = 1; for (uint32_t i = 0; i < k; ++i) { mul[k - 1 - i] = p; p *= W; } }
    uint64_t tix = 0;
    for (uint64_t ii = n; ii-- > 0;) {
        uint32_t s = table ? table[text[ii]] : text[ii];
        if (s >= sigma) { free(t); free(cnt); free(kc); free(mul); return ORC_E_SYMBOL; }
        t[ii] = (uint8_t)(s + 1);
        cnt[s + 1]++;
        tix /= W;
        tix += mul[0] * (s + 1);
        kc[tix]++;
    }
    t[n] = 0; /* SENTINEL_SYMBOL (crate_bio_manual/mod.rs:5,10) */
    uint64_t acc = 0;
    for (uint64_t c = 0; c < W; ++c) { acc += cnt[c]; wr_p(ca, c, (uint32_t)pb, acc); }
    acc = 0;
    for (uint64_t c = 0; c < wk; ++c) { acc += kc[c]; wr_p(kt, c, (uint32_t)pb, acc); }
    for (uint32_t i = 0; i < k; ++i) wr_u64(mult + 8 * i, mul[i]);
    free(cnt); free(kc); free(mul);

    /* 3) suffix array + BWT (crate_bio_manual/mod.rs:8-23, bwt.rs:14-24) */
    uint64_t *sa = (uint64_t *)malloc((n + 1) * 8);
    if (!sa) { free(t); return ORC_E_CONFIG; }
    orc_suffix_array(t, n + 1, (uint32_t)W, sa);
    uint8_t *bwt = (uint8_t *)malloc(n + 1);
    uint64_t pidx = 0;
    int found = 0;
    for (uint64_t r = 0; r <= n; ++r) {
        bwt[r] = sa[r] > 0 ? t[sa[r] - 1] : t[n];
        if (!found && bwt[r] == 0) { pidx = r; found = 1; }
    }
    memmove(bwt + pidx, bwt + pidx + 1, n - pidx); /* bwt.remove(pidx) */
    /* SA.remove(0), then step_by(sr) */
    for (uint64_t j = 0; j < S.sa_len; ++j) wr_p(sa_out, j, (uint32_t)pb, sa[1 + j * sr]);
    free(sa);
    free(t);

    /* 4) encode_bwm_body — bwm/mod.rs:91-143 with Block::vectorize
     * (block3.rs:18-36) and shift_last_offset (:37-39). */
    wr_p(sent, 0, (uint32_t)pb, pidx);
    uint64_t pre[64] = {0};
    const uint32_t vb = (uint32_t)(BL / 8), bb = L.planes * vb;
    for (uint64_t q = 0; q < S.blocks_len; ++q) {
        for (uint32_t c = 0; c < sigma; ++c) wr_p(ckpt, q * sigma + c, (uint32_t)pb, pre[c]);
        u128 planes[6] = {0, 0, 0, 0, 0, 0};
        uint64_t b0 = q * BL, e0 = b0 + BL < n ? b0 + BL : n;
        for (uint64_t p = b0; p < e0; ++p) {
            uint32_t s = (uint32_t)bwt[p] - 1; /* sentinel's idx is 0 */
            pre[s]++;
            uint32_t bit = (uint32_t)(BL - 1 - (p - b0));
            for (uint32_t j = 0; j < L.planes; ++j)
                if ((s >> j) & 1) planes[j] |= (u128)1 << bit;
        }
        for (uint32_t j = 0; j < L.planes; ++j) memcpy(blocks + q * bb + j * vb, &planes[j], vb);
    }
    free(bwt);
    return ORC_OK;
}
