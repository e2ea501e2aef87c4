/*
 * fmx.h — C ABI of the MI355X-native batched FM-index count/locate engine.
 *
 * This is the drop-in boundary for baku4/sview-fmindex's query hot path.  The
 * reference has no FFI of its own: its surface is the Rust generic API
 * `FmIndex<'a, P: Position, B: Block, E: TextEncoder>` (sview-fmindex/src/lib.rs:14-28)
 * over the blob byte layout written by `FmIndexBuilder::build`
 * (src/builder/mod.rs:187-264).  Each entry point below names the reference
 * item it replaces; INTEGRATION.md shows the Rust `extern "C"` binding a
 * maintainer would add to restore `FmIndex::count/locate` on top of it.
 *
 * Conventions
 *  - Plain pointers and sizes only.  "Host" buffers are ordinary CPU memory;
 *    "device" buffers are HIP device pointers on the index's device.
 *  - P-wide outputs (counts, locations) are uint32_t when layout.pos_bytes == 4
 *    and uint64_t when 8, exactly the reference's `P` (src/text_length.rs:10-129).
 *  - Locations of one pattern are emitted in suffix-array-row order, the order
 *    `FmIndex::locate` returns them in (src/locate/mod.rs:14-37).
 *  - No entry point aborts: every failure the reference reports as an error or
 *    a panic is returned as an fmx_status.
 */
#ifndef FMX_H
#define FMX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FMX_ABI_VERSION 8u

typedef enum fmx_status {
    FMX_OK = 0,
    FMX_E_FORMAT = 1,        /* LoadError::InvalidFormat (src/load_from_blob.rs:16-19, 31-33)          */
    FMX_E_SIZE = 2,          /* LoadError::MismatchedBlobSize(expected, actual) (load_from_blob.rs:20-23, 46-58) */
    FMX_E_ALIGN = 3,         /* misaligned blob: reference panics (bwm/mod.rs:172-181); BuildError::NotAlignedBlob */
    FMX_E_LAYOUT = 4,        /* layout tag inconsistent with the blob's headers (P/B/E are not stored in the blob) */
    FMX_E_EMPTY_PATTERN = 5, /* empty pattern: reference panics (components/count_array.rs:211)            */
    FMX_E_SYMBOL = 6,        /* PassThrough byte >= symbol_count; BuildError::SymbolCountOver (builder/mod.rs:71-73) */
    FMX_E_CAPACITY = 7,      /* locate output buffer smaller than the number of occurrences ("needed")   */
    FMX_E_DEVICE = 8,        /* HIP runtime error, or no GPU                                               */
    FMX_E_ARG = 9,           /* null pointer or invalid argument                                           */
    FMX_E_CONFIG = 10        /* BuildError::{InvalidConfig, UnmatchedTextLength, InvalidBlobSize}          */
} fmx_status;

/* The reference's type parameters, which the blob does not record
 * (only sizes are checked, src/load_from_blob.rs:40-58). */
typedef struct fmx_layout {
    uint32_t pos_bytes; /* P: 4 = u32, 8 = u64                      (src/text_length.rs:10-129)   */
    uint32_t planes;    /* B = BlockN<V>: N in 2..6                  (components/bwm/blocks/mod.rs)  */
    uint32_t vec_bits;  /* V: 32, 64 or 128 = BLOCK_LEN              (components/bwm/blocks/vector.rs:11-79) */
    uint32_t encoder;   /* E: FMX_ENC_TABLE or FMX_ENC_PASS          (components/text_encoder/)      */
} fmx_layout;

#define FMX_ENC_TABLE 0u /* EncodingTable([u8; 256])  text_encoders/encoding_table.rs:7-11 */
#define FMX_ENC_PASS 1u  /* PassThrough               text_encoders/pass_through.rs:6-12   */

/* Query flags */
#define FMX_PATTERN_REVERSED 1u /* patterns are given last byte first: the *_rev_iter forms
                                   (src/locate/with_rev_iter.rs:5-38)                          */
#define FMX_HINT_LONG_PATTERNS 2u /* performance hint: patterns average more than 64 bytes; the
                                   kernels stage each workgroup's patterns in 56 KB of LDS
                                   instead of 16 KB                                            */
/* Performance hint: stage each 256-pattern tile in kb KB of LDS (1..56): the
 * most bytes any tile's patterns span.  A tile that does not fit is read from
 * HBM instead (same results).  Less LDS per workgroup = more workgroups per
 * CU.  Overrides FMX_HINT_LONG_PATTERNS; the host-buffer calls set it exactly. */
#define FMX_HINT_STAGE_KB(kb) ((((uint32_t)(kb)) & 0xffu) << 8)
/* Performance hint: every pattern is m bytes (1..65535) and d_offsets[i] ==
 * i * m, so the kernels address each pattern's bytes without first reading
 * the offsets (one dependent HBM round trip fewer per workgroup).  The
 * offsets are still read alongside and checked: a batch that disagrees is
 * reported as FMX_E_ARG (its outputs are then undefined).  Because the bytes
 * are read before that check, a hint larger than the true length is
 * undefined behaviour for the reads: the kernels read up to n_patterns * m
 * bytes from d_bytes, which must be that large.  The host-buffer calls set
 * the hint themselves when every pattern has the same length. */
#define FMX_HINT_FIXED_LEN(m) ((((uint32_t)(m)) & 0xffffu) << 16)

/* Load options: device-side structures derived from the blob at load time.
 * Results are identical with any combination; they trade HBM for fewer
 * dependent random reads per pattern. */
#define FMX_OCC_BLOB 0u        /* kernels read the blob's rank_checkpoints / blocks as laid out   */
#define FMX_OCC_INTERLEAVED 1u /* checkpoints + bit planes re-laid out into one HBM line per block */
#define FMX_OPT_DEEP_LUT 2u    /* a K-mer interval table (K > the blob's k), built on the GPU by
                                  breadth-first backward search; replaces the first LF steps.
                                  Indexed by the S symbols that occur in the text: K = the
                                  largest with S^K * 2P bytes <= FMX_DEEP_LUT_MB (environment;
                                  default 163840, capped at half the free HBM) */
#define FMX_OPT_FULL_SA 4u     /* the full suffix array (n x P), recovered on the GPU by walking every
                                  row to its sample: a location is one read, no walk            */
#define FMX_OPT_TEXT 8u        /* the text (n symbol indices), recovered from the full SA; once an
                                  interval is a single row, the rest of the pattern is compared
                                  against the text instead of LF-stepped (needs FMX_OPT_FULL_SA) */
#define FMX_OPT_ROW_CONTEXT 16u /* full SA stored as row records {SA[r], ctx[r]} (2P per row), ctx =
                                  the up to context_len symbols preceding the suffix, packed base
                                  sigma+1; an interval of at most FMX_SCAN_ROWS rows (environment,
                                  default 32) is finished by one contiguous scan of its records
                                  instead of LF steps (implies FMX_OPT_FULL_SA | FMX_OPT_TEXT)    */
#define FMX_OPT_LUT_ROWS 32u   /* deep-table entries whose interval is a single row hold that row's
                                  SA value and the symbols preceding its suffix instead of the
                                  interval: such a pattern is settled by that one read (plus a
                                  text compare beyond the packed symbols).  Needs FMX_OPT_DEEP_LUT
                                  and FMX_OPT_TEXT, and n < 2^31 for u32 positions            */
/* The default: the blob's own structures, its occ planes and checkpoints
 * re-laid out as one record per block — the reference's index and algorithm
 * (FmIndex::load is a zero-copy view, load_from_blob.rs:28-85; this is one
 * device copy plus a 1/2.7 size re-layout, milliseconds at 1 Gbp). */
#define FMX_OPT_DEFAULT FMX_OCC_INTERLEAVED
/* Every derived structure: ~55x the blob's HBM at C2 (147 GB) and seconds of
 * load time, paid back only after ~10^10 patterns (bench.py "derived"). */
#define FMX_OPT_DERIVED (FMX_OCC_INTERLEAVED | FMX_OPT_DEEP_LUT | FMX_OPT_FULL_SA | FMX_OPT_TEXT | \
                         FMX_OPT_ROW_CONTEXT | FMX_OPT_LUT_ROWS)
/* fmx_load_file only: read the blob's body with O_DIRECT, bypassing the page
 * cache — a cold load from storage, what the reference bench measures after
 * dropping the caches (bench/run_benchmark.sh:53-56).  FMX_E_ARG if the
 * file system refuses O_DIRECT (tmpfs does). */
#define FMX_LOAD_DIRECT (1u << 16)

typedef struct fmx_index fmx_index; /* opaque; one per (blob, device) */

typedef struct fmx_index_info {
    uint64_t text_len;       /* C[symbol_count]                                   */
    uint64_t sentinel_index; /* BwmView.sentinel_index                            */
    uint64_t blob_len;
    uint64_t device_bytes;   /* HBM held by the index (blob + derived structures) */
    uint32_t symbol_count;
    uint32_t kmer_size;      /* lookup_table_kmer_size                            */
    uint32_t sampling_ratio;
    uint32_t block_len;      /* BLOCK_LEN = vec_bits                              */
    uint32_t options;        /* FMX_OCC_* | FMX_OPT_* in effect                   */
    uint32_t deep_lut_k;     /* K of the deep k-mer table (0 = none)              */
    int32_t device;
    uint32_t context_len;    /* symbols per row context (0 = no row records)      */
    uint32_t scan_rows;      /* largest interval finished by a record scan        */
    uint32_t occ_record;     /* occ record encoding: 0 blob layout, 64/128 interleaved
                                records, | 1 paired-chunk, | 2 symbol-mask records
                                                                     */
    uint32_t group_key_len;  /* grouped launches: the key's last symbols (0: none) */
    uint32_t group_key_base; /* ... as digits over this many symbols               */
    uint64_t grouped_min;    /* fixed-length launches of at least this many
                                patterns are grouped (UINT64_MAX: never)            */
    uint64_t launches_grouped;      /* locate launches of this index so far, by the
                                       path they took: grouped with packed records, */
    uint64_t launches_grouped_raw;  /* grouped with id-only records,                  */
    uint64_t launches_ordered;      /* in launch order,                               */
    uint64_t launches_fused;        /* of those, as one kernel (k_locate: search,
                                       offsets and locations; FMX_FUSED=0: never)   */
    uint64_t launches_chained;      /* grouped launches ended by k_emit_chain (tile
                                       counts handed from tile to tile in-kernel)    */
} fmx_index_info;

typedef struct fmx_kernel_timing {
    char name[32];
    uint64_t launches;
    double total_ms;         /* summed hipEvent durations on the launch stream    */
    uint64_t units;          /* patterns (count) or occurrences (locate) processed */
} fmx_kernel_timing;

/* ---------------------------------------------------------------- version */
uint32_t fmx_abi_version(void);
const char *fmx_status_str(fmx_status s);
int fmx_device_count(void);

/* ------------------------------------------------------------------- load */

/* FmIndex::load (src/load_from_blob.rs:28-85).  Validates the blob exactly as
 * the reference does (magic + version, header sizes, exact body size) plus the
 * consistency checks the reference leaves to the type system, then copies the
 * blob to HBM of `device` once.  The host blob is borrowed for fmx_blob() only.
 * On FMX_E_SIZE, *expected_total / *actual_total receive the two sizes.
 * options: FMX_OCC_* | FMX_OPT_* (FMX_OPT_DEFAULT: the blob's own structures). */
fmx_status fmx_load(const uint8_t *blob, uint64_t blob_len, fmx_layout layout, int device,
                    uint32_t options, fmx_index **out, uint64_t *expected_total,
                    uint64_t *actual_total);

/* Same, for a blob already resident in HBM of `device` (e.g. written by
 * fmx_build_device).  The device blob is borrowed and must outlive the index.
 * Starts after all work already queued on the device: it calls
 * hipDeviceSynchronize, which also waits for unrelated work on other streams
 * (other threads' queries, pending collectives) — load before serving starts,
 * or order the blob's writer yourself and accept that wait once. */
fmx_status fmx_load_device(const uint8_t *d_blob, uint64_t blob_len, fmx_layout layout, int device,
                           uint32_t options, fmx_index **out, uint64_t *expected_total,
                           uint64_t *actual_total);

/* Blob ingest from a file (the bench's mmap / read-whole-file loaders,
 * bench/src/locate/sview_mmap.rs:17-45 and sview_memory.rs:17-20, then
 * FmIndex::load).  The header is read and validated first (same checks and
 * codes as fmx_load; the file size is the blob length); the body is then
 * streamed file -> a ring of four pinned host chunks -> HBM, each chunk read
 * by several threads while earlier chunks are in flight, so no host copy of
 * the whole blob is ever held.  chunk_bytes = 0 picks the default (16 MiB:
 * pinning larger buffers costs more than it saves).  FMX_E_ARG if the file cannot
 * be opened or read.  fmx_blob() returns NULL for such an index. */
fmx_status fmx_load_file(const char *path, fmx_layout layout, int device, uint32_t options,
                         uint64_t chunk_bytes, fmx_index **out, uint64_t *expected_total,
                         uint64_t *actual_total);

void fmx_free(fmx_index *ix);

/* FmIndex::blob (src/reference_to_source_blob.rs:9-11).  NULL for device loads. */
const uint8_t *fmx_blob(const fmx_index *ix, uint64_t *len);

fmx_status fmx_info(const fmx_index *ix, fmx_index_info *out);

/* ---------------------------------------------- queries on host buffers
 * Synchronous.  Patterns are ragged: pattern i is bytes[offsets[i] .. offsets[i+1]). */

/* FmIndex::count / count_rev_iter (locate/with_slice.rs:5-8, with_rev_iter.rs:5-9), batched. */
fmx_status fmx_count_batch(fmx_index *ix, const uint8_t *bytes, const uint64_t *offsets,
                           uint64_t n_patterns, uint32_t flags, void *out_counts);

/* FmIndex::locate / locate_rev_iter (with_slice.rs:10-13, with_rev_iter.rs:10-14),
 * batched: the locations of pattern i are out_locs[out_loc_offsets[i] ..
 * out_loc_offsets[i+1]) in suffix-array-row order.  *needed receives the total;
 * if it exceeds cap, nothing past cap is written and FMX_E_CAPACITY is returned. */
fmx_status fmx_locate_batch(fmx_index *ix, const uint8_t *bytes, const uint64_t *offsets,
                            uint64_t n_patterns, uint32_t flags, uint64_t *out_loc_offsets,
                            void *out_locs, uint64_t cap, uint64_t *needed);

/* ---------------------------------------------- queries on device buffers
 * Asynchronous on `stream` (a hipStream_t; NULL = the index's own stream).
 * Inputs and outputs live in HBM of the index's device.  Errors detected on
 * the device (empty pattern, PassThrough symbol) are latched in a status word
 * read by fmx_sync().  Only `stream` orders the launch: the index's own
 * stream is non-blocking (not ordered with the caller's streams, nor with the
 * legacy default stream), so buffers written on another stream must be
 * complete first — pass the writers' stream, or synchronise. */

fmx_status fmx_count_batch_async(fmx_index *ix, const uint8_t *d_bytes, const uint64_t *d_offsets,
                                 uint64_t n_patterns, uint32_t flags, void *d_counts, void *stream);

/* Workspace for fmx_locate_batch_async, in bytes, for up to n_patterns patterns:
 * [256 B][32 KiB of key counters][58 KiB batch table of a grouped launch]
 * [tile counts][tile offsets][one search record per pattern][to 16 B][one
 * 16-B sorted-order record per pattern].
 * The workspace must be 16-byte aligned (FMX_E_ARG otherwise: the grouped
 * passes read and write it as 16-B vectors; hipMalloc gives 256-B alignment).
 * A workspace needs no initialisation (a grouped launch zeroes its key
 * counters on its stream first; only the FMX_SEARCH_PERSISTENT=1 A/B variant
 * wants its first 4 bytes zero) and belongs to this index: its launches are
 * ordered on one stream at a time.  A locate is k_search + k_emit.  A
 * grouped locate first deals the launch's patterns out in the order of their
 * last symbols, so that patterns whose backward searches share their first
 * LF steps run side by side, and searches them in that order — same
 * results.  Grouped by default: launches (a group call's batches together) of
 * at least 3 x 2^20 fixed-length patterns that pack into 96 bits, on the
 * faithful index, when the key spans at least 5 symbols (DNA: 6), of at
 * least 2^26 when it spans fewer (20 residues: 3; environment
 * at load: FMX_GROUPED=0 never, =1 always — longer patterns too, with
 * id-only records —, FMX_GROUPED_MIN=<patterns>, FMX_GROUPED_RAW=1 id-only
 * records, FMX_GROUP_REFINE_MIN=<patterns> re-sorts each key's run by the
 * next symbols, FMX_GROUPED_WSORT=0 turns off the search's in-workgroup sort
 * by the next symbols, FMX_GROUP_CHECK=1 checks each launch's sorted order on
 * the device before its search — a violation is FMX_E_DEVICE; debug).  One
 * kernel makes workgroups wait on others: the fused launch in launch order
 * (k_locate, fmx_index_info.launches_fused; FMX_FUSED=0 never) — a workgroup
 * answers the tile of its ticket (the number of its batch's workgroups that
 * started before it) and waits only for the earlier tiles of its batch, whose
 * workgroups are therefore already running; bounded (FMX_FUSED_TIMEOUT_MS,
 * default 4 s, then FMX_E_DEVICE).  The key counters and the batch table of a
 * grouped launch are in its first batch's workspace. */
fmx_status fmx_locate_workspace_size(fmx_index *ix, uint64_t n_patterns, uint64_t *bytes);

/* The same size without an index (ABI 8): for n_patterns patterns of an
 * index with pos_bytes-wide positions (4 or 8; FMX_E_ARG otherwise) — what a
 * caller sizing HBM before it loads an index (e.g. the per-rank accounting of
 * a sharded job) needs.  Equal to fmx_locate_workspace_size on such an index. */
fmx_status fmx_workspace_bytes(uint64_t n_patterns, uint32_t pos_bytes, uint64_t *bytes);

/* d_loc_offsets has n_patterns+1 entries; d_counts (optional, may be NULL)
 * receives P-wide counts; d_needed (device uint64) receives the total. */
fmx_status fmx_locate_batch_async(fmx_index *ix, const uint8_t *d_bytes, const uint64_t *d_offsets,
                                  uint64_t n_patterns, uint32_t flags, void *d_counts,
                                  uint64_t *d_loc_offsets, void *d_locs, uint64_t cap,
                                  uint64_t *d_needed, void *d_workspace, uint64_t workspace_bytes,
                                  void *stream);

/* A queue of locate batches submitted in one call (a serving loop's batches
 * in flight): job i is exactly fmx_locate_batch_async(ix, jobs[i].d_bytes,
 * ...), issued in order, each on its own stream; the call returns after the
 * last launch is queued (or at the first error, which it returns). */
typedef struct fmx_locate_job {
    const uint8_t *d_bytes;
    const uint64_t *d_offsets;
    uint64_t n_patterns;
    uint32_t flags;
    uint32_t reserved;         /* 0 */
    void *d_counts;            /* optional */
    uint64_t *d_loc_offsets;
    void *d_locs;
    uint64_t cap;
    uint64_t *d_needed;
    void *d_workspace;
    uint64_t workspace_bytes;
    void *stream;              /* hipStream_t; NULL = the index's own stream */
} fmx_locate_job;

fmx_status fmx_locate_jobs_async(fmx_index *ix, const fmx_locate_job *jobs, uint64_t n_jobs);

/* The same batches run together: up to 1,024 per launch on `stream` (each
 * batch keeps its own patterns, outputs and workspace; the jobs' own stream
 * fields are ignored), so that small batches fill the GPU the way one large
 * batch does — a grouped launch searches all of them in one order (kernels
 * take at most 256 batches as arguments: the launch-order path runs one
 * launch per 256).  The jobs' workspaces must be distinct and no two jobs may share
 * an output buffer (they run concurrently).  The results are those of
 * fmx_locate_batch_async on each job. */
fmx_status fmx_locate_group_async(fmx_index *ix, const fmx_locate_job *jobs, uint64_t n_jobs, void *stream);

/* Wait for `stream` and return (and clear) the latched device status. */
fmx_status fmx_sync(fmx_index *ix, void *stream);

/* The caller is done with `stream` (e.g. before hipStreamDestroy): wait for it,
 * return (and clear) its latched status like fmx_sync, and free its status
 * word for reuse.  Optional: an index holds 1024 status words and recycles
 * the least recently used one whose stream has no launch in flight, so a
 * caller that makes a stream per request never runs out; bits latched on a
 * recycled word and never read are dropped.  A destroyed stream's handle may
 * be reused by a new stream, which then shares the old status word — release
 * (or sync) a stream before destroying it. */
fmx_status fmx_stream_release(fmx_index *ix, void *stream);

/* ----------------------------------------------------- several GPUs, one handle
 * The device mask of SURVEY §8(b) for a single-process caller (no process
 * group): one replica of the index per entry of `devices` (a device may be
 * listed more than once: replicas on one GPU run concurrently).  The blob is
 * validated like fmx_load (same codes), copied to HBM of devices[0] once and
 * from there device-to-device to the other replicas (hipMemcpyPeer: xGMI
 * between MI355X GPUs); each replica is an fmx_load_device index.  A host
 * batch is cut into n_replicas contiguous shards (sizes differ by at most
 * one) answered concurrently, and the results are concatenated in order:
 * exactly what fmx_count_batch / fmx_locate_batch on one device return for
 * the whole batch (same capacity contract: offsets and *needed are written,
 * FMX_E_CAPACITY if the total exceeds cap). */
typedef struct fmx_multi fmx_multi;

fmx_status fmx_multi_load(const uint8_t *blob, uint64_t blob_len, fmx_layout layout, const int *devices,
                          int n_devices, uint32_t options, fmx_multi **out, uint64_t *expected_total,
                          uint64_t *actual_total);
void fmx_multi_free(fmx_multi *m);
int fmx_multi_replicas(const fmx_multi *m);
/* Replica i's own index (for the device-buffer calls on its device); owned by m. */
fmx_index *fmx_multi_replica(fmx_multi *m, int i);
fmx_status fmx_multi_count_batch(fmx_multi *m, const uint8_t *bytes, const uint64_t *offsets,
                                 uint64_t n_patterns, uint32_t flags, void *out_counts);
fmx_status fmx_multi_locate_batch(fmx_multi *m, const uint8_t *bytes, const uint64_t *offsets,
                                  uint64_t n_patterns, uint32_t flags, uint64_t *out_loc_offsets,
                                  void *out_locs, uint64_t cap, uint64_t *needed);

/* --------------------------------------------------------------- timing
 * enable = k > 0: every k-th kernel launch (k = 1: every launch) is bracketed
 * by hipEvents on its stream; 0: off.  fmx_timing_read sums the bracketed
 * durations per kernel since timing was last enabled (enabling resets the
 * totals; fmx_timing_read synchronises).  An event pair costs the stream
 * several microseconds, so throughput runs sample (k > 1).  Timers: "count",
 * "locate" (a whole locate launch) and, for fmx_locate_group_async, its two
 * kernels "locate.search" (k_search) and "locate.emit" (k_emit). */
fmx_status fmx_timing_enable(fmx_index *ix, int enable);
fmx_status fmx_timing_read(fmx_index *ix, fmx_kernel_timing *out, int max_entries, int *n_entries);

/* --------------------------------------------------------------- builder
 * FmIndexBuilder (src/builder/mod.rs): blob_size (:165-181) and build (:187-264),
 * on the GPU.  kmer_size 1 = LookupTableConfig::None, >= 2 = KmerSize(k);
 * sampling_ratio 1 = SuffixArrayConfig::Uncompressed, >= 2 = Compressed(r).
 * table: 256-byte EncodingTable (host memory), or NULL for PassThrough. */
fmx_status fmx_build_blob_size(uint64_t text_len, uint32_t symbol_count, fmx_layout layout,
                               uint32_t kmer_size, uint32_t sampling_ratio, uint64_t *out_size);

/* d_text and d_blob are device buffers on `device`; d_blob must be 16-B aligned
 * and exactly fmx_build_blob_size bytes.  Synchronous: starts after all work
 * already queued on the device (whichever stream wrote d_text) and returns
 * when the blob is complete. */
fmx_status fmx_build_device(const uint8_t *d_text, uint64_t text_len, const uint8_t *table,
                            uint32_t symbol_count, fmx_layout layout, uint32_t kmer_size,
                            uint32_t sampling_ratio, uint8_t *d_blob, uint64_t blob_len, int device);

/* Host-buffer convenience: uploads the text, builds on `device`, downloads the blob. */
fmx_status fmx_build(const uint8_t *text, uint64_t text_len, const uint8_t *table,
                     uint32_t symbol_count, fmx_layout layout, uint32_t kmer_size,
                     uint32_t sampling_ratio, uint8_t *blob, uint64_t blob_len, int device);

#ifdef __cplusplus
}
#endif
#endif /* FMX_H */
