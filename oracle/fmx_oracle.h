/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of baku4/sview-fmindex's query path (k-mer seed,
 * LF-mapping backward search over the bit-sliced Block<V> occ arrays, sampled-SA
 * locate walk) and of its blob builder.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library, and only as the
 * checker / CPU baseline — never as the product path.
 *
 * Parity pins: the reference's README known-answer test
 * (sview-fmindex/src/tests/readme/mod.rs:29-44) is committed as
 * tests/golden/readme.json, and the reference's accuracy contract
 * (src/tests/get_accurate_result/mod.rs:136-140: sorted locate == all
 * occurrences) is checked by brute force in tests/test_oracle.py.
 * Blob bytes and the unsorted (suffix-array-row) locate order are pinned only
 * by this restatement ("parity unpinned" against a real reference run: the
 * Rust toolchain is absent).
 */
#ifndef FMX_ORACLE_H
#define FMX_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Layout tags (the reference's generic parameters P, B=BlockN<V>, E). */
typedef struct {
    uint32_t pos_bytes; /* Position P: 4 (u32) or 8 (u64)   text_length.rs:10-129 */
    uint32_t planes;    /* N of BlockN: 2..6                 blocks/mod.rs:1-30     */
    uint32_t vec_bits;  /* V: 32, 64 or 128                  blocks/vector.rs:11-79 */
    uint32_t encoder;   /* 0 = EncodingTable, 1 = PassThrough text_encoder/        */
} orc_layout;

enum {
    ORC_OK = 0,
    ORC_E_FORMAT = 1,        /* LoadError::InvalidFormat            load_from_blob.rs:16-24 */
    ORC_E_SIZE = 2,          /* LoadError::MismatchedBlobSize        load_from_blob.rs:46-58 */
    ORC_E_ALIGN = 3,         /* BuildError::NotAlignedBlob           builder/mod.rs:197-202  */
    ORC_E_LAYOUT = 4,        /* inconsistent header / bad layout tag                        */
    ORC_E_EMPTY_PATTERN = 5, /* reference panics (count_array.rs:211)                      */
    ORC_E_SYMBOL = 6,        /* PassThrough byte >= symbol_count; BuildError::SymbolCountOver */
    ORC_E_CAPACITY = 7,
    ORC_E_CONFIG = 10,       /* BuildError::InvalidConfig / UnmatchedTextLength / InvalidBlobSize */
};

/* A loaded index: parsed headers + pointers into the caller's blob (zero-copy,
 * as FmIndex borrows &'a [u8], lib.rs:14-28). */
typedef struct {
    orc_layout L;
    const uint8_t *blob;
    uint64_t blob_len;
    uint8_t enc[256];         /* EncodingTable bytes, or the identity for PassThrough */
    uint32_t sigma;           /* CountArrayHeader.symbol_count */
    uint32_t k;               /* lookup_table_kmer_size */
    uint32_t sr;              /* SuffixArrayHeader.sampling_ratio */
    uint32_t bl;              /* BLOCK_LEN = vec_bits */
    uint32_t align;           /* ALIGN_SIZE: 8 (u32/u64 vectors) or 16 (u128) */
    uint32_t block_bytes;     /* planes * vec_bits / 8 */
    uint64_t n;               /* text length = C[sigma] */
    uint64_t count_array[65]; /* C-array, sigma+1 entries (copied, count_array.rs:187) */
    uint64_t mult[64];        /* kmer_multiplier (copied, count_array.rs:188) */
    const uint8_t *kmer_table; uint64_t kmer_len;
    const uint8_t *sa;         uint64_t sa_len;
    uint64_t sentinel;        /* BwmView.sentinel_index */
    const uint8_t *ckpt;       uint64_t ckpt_len;
    const uint8_t *blocks;     uint64_t blocks_len;
    /* byte offsets of each section inside the blob (for tests / device upload) */
    uint64_t off_count_array, off_mult, off_kmer, off_sa, off_sentinel, off_ckpt, off_blocks;
} orc_index;

int orc_load(const uint8_t *blob, uint64_t len, orc_layout L, orc_index *out,
             uint64_t *expected_total, uint64_t *actual_total);

/* FmIndex::count / locate (locate/with_slice.rs:5-18).  Locations are written
 * in suffix-array-row order, exactly as write_locations_to_buffer emits them. */
int orc_count(const orc_index *ix, const uint8_t *pat, uint64_t m, uint64_t *out_count);
int orc_locate(const orc_index *ix, const uint8_t *pat, uint64_t m,
               uint64_t *out_locs, uint64_t cap, uint64_t *out_count);
/* The *_rev_iter forms (locate/with_rev_iter.rs:5-38): the pattern is given
 * already reversed (rev[0] is the pattern's last byte). */
int orc_count_rev(const orc_index *ix, const uint8_t *rev, uint64_t m, uint64_t *out_count);

/* Batches over ragged patterns (bytes + offsets[n+1]); `threads` CPU threads
 * each take a contiguous slab of patterns. Outputs are P-wide (ix->L.pos_bytes). */
int orc_count_batch(const orc_index *ix, const uint8_t *bytes, const uint64_t *offsets,
                    uint64_t n, void *out_counts, int threads);
int orc_locate_batch(const orc_index *ix, const uint8_t *bytes, const uint64_t *offsets,
                     uint64_t n, uint64_t *out_loc_offsets, void *out_locs,
                     uint64_t cap, uint64_t *needed, int threads);

/* Builder (builder/mod.rs:165-264). k = lookup_table_kmer_size (1 = None),
 * sr = sampling ratio (1 = Uncompressed).  table == NULL selects PassThrough. */
int orc_blob_size(uint64_t text_len, uint32_t sigma, orc_layout L, uint32_t k, uint32_t sr,
                  uint64_t *out_size);
int orc_build(const uint8_t *text, uint64_t n, const uint8_t *table, uint32_t sigma,
              orc_layout L, uint32_t k, uint32_t sr, uint8_t *blob, uint64_t blob_len);

/* Suffix array of t[0..len) (len includes the trailing unique 0 sentinel), by
 * prefix doubling.  Exposed for tests. */
int orc_suffix_array(const uint8_t *t, uint64_t len, uint32_t alphabet, uint64_t *sa);

#ifdef __cplusplus
}
#endif
#endif
