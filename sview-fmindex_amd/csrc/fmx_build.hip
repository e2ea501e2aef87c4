// fmx_build.hip — the blob builder on the GPU (FmIndexBuilder::build,
// sview-fmindex/src/builder/mod.rs:187-264), producing byte-for-byte the blob
// the reference writes into a zeroed buffer:
//
//   1. encode + count      count_and_encode_text      components/count_array.rs:78-136
//   2. suffix array        get_compressed_suffix_array_and_pidx_while_bwt
//                          (crate_bio_manual/mod.rs:8-23) — here by prefix doubling
//                          over 64-bit packed keys with rocPRIM radix sorts.  The SA of a
//                          string with a unique smallest sentinel is unique, so the
//                          construction algorithm does not change a byte.
//   3. BWT, pidx, sampled SA (crate_bio_manual/mod.rs:10-21, bwt.rs:14-24)
//   4. occ encoding        BwmHeader::encode_bwm_body (bwm/mod.rs:91-143) with
//                          Block::vectorize / shift_last_offset (blocks/block3.rs:18-39)
//
// Sizes: n + 1 < 2^32 with 32-bit suffix indices (about 40 B per text byte of
// transient HBM at the peak: keys, values and their double buffers); larger
// texts take the bucketed 64-bit path (suffix_array64: ~17 B per text byte
// plus ~49 B per element of the largest first-two-symbol bucket and 56 B per
// suffix still unresolved in a doubling round).
#include <cstring>
#include <rocprim/rocprim.hpp>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "fmx_internal.hpp"

namespace fmx {

#define BCK(x)                                                                                       \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) {                                                                      \
            fprintf(stderr, "fmx build: %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return FMX_E_DEVICE;                                                                     \
        }                                                                                            \
    } while (0)

struct DBuf {
    void *p = nullptr;
    size_t bytes = 0;
    DBuf() = default;
    DBuf(const DBuf &) = delete;
    ~DBuf() { if (p) hipFree(p); }
    hipError_t alloc(size_t b) {
        if (p) hipFree(p);
        p = nullptr;
        bytes = b;
        return hipMalloc(&p, b ? b : 16);
    }
    template <class T> T *as() const { return (T *)p; }
};

static unsigned grid_of(uint64_t n, unsigned cap = 1u << 20) {
    uint64_t g = (n + 255) / 256;
    if (g == 0) g = 1;
    return (unsigned)(g < cap ? g : cap);
}

// ------------------------------------------------------------ 1. encode

struct EncTable { uint8_t v[256]; };

// t[i] = idx(text[i]) + 1, t[n] = 0 (count_array.rs:112-118, crate_bio_manual/mod.rs:10)
__global__ __launch_bounds__(256) void k_encode(const uint8_t *__restrict__ text, uint64_t n, EncTable enc,
                                                uint32_t sigma, uint8_t *__restrict__ t,
                                                unsigned long long *__restrict__ sym_counts, uint32_t *status) {
    __shared__ uint32_t hist[kMaxSigma];
    __shared__ uint8_t s_enc[256];
    s_enc[threadIdx.x] = enc.v[threadIdx.x];
    if (threadIdx.x < kMaxSigma) hist[threadIdx.x] = 0;
    __syncthreads();
    uint32_t bad = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint32_t c = s_enc[text[i]];
        if (c >= sigma) { bad = 1; t[i] = 1; continue; }
        t[i] = (uint8_t)(c + 1);
        atomicAdd(&hist[c], 1u);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) t[n] = 0;
    if (bad) atomicOr(status, kStatusSymbol);
    __syncthreads();
    if (threadIdx.x < sigma && hist[threadIdx.x]) atomicAdd(&sym_counts[threadIdx.x], (unsigned long long)hist[threadIdx.x]);
}

// k-mer code of every text position (count_array.rs:110-123): digits are the
// (idx+1) of t[i..i+k), 0 past the end, most significant first.
__global__ __launch_bounds__(256) void k_kmer_hist(const uint8_t *__restrict__ t, uint64_t n, uint32_t k, uint64_t W,
                                                   uint64_t bins, unsigned long long *__restrict__ hist) {
    extern __shared__ uint32_t lh[];
    const bool use_lds = bins <= 8192;
    if (use_lds) {
        for (uint64_t b = threadIdx.x; b < bins; b += 256) lh[b] = 0;
        __syncthreads();
    }
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        uint64_t code = 0;
        for (uint32_t j = 0; j < k; ++j) {
            const uint64_t x = i + j;
            code = code * W + (x < n ? t[x] : 0);
        }
        if (use_lds) atomicAdd(&lh[code], 1u);
        else atomicAdd(&hist[code], 1ull);
    }
    if (use_lds) {
        __syncthreads();
        for (uint64_t b = threadIdx.x; b < bins; b += 256)
            if (lh[b]) atomicAdd(&hist[b], (unsigned long long)lh[b]);
    }
}

template <typename P>
__global__ void k_narrow(const uint64_t *__restrict__ in, uint64_t n, P *__restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) out[i] = (P)in[i];
}

// ---------------------------------------------------- 2. suffix array

// Packed first-K0-symbols key of suffix i (b bits per symbol, 0 past the end).
__global__ __launch_bounds__(256) void k_init_keys(const uint8_t *__restrict__ t, uint64_t n1, uint32_t b, uint32_t K0,
                                                   uint64_t *__restrict__ keys, uint32_t *__restrict__ vals) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n1; i += (uint64_t)gridDim.x * 256) {
        uint64_t key = 0;
        for (uint32_t j = 0; j < K0; ++j) {
            const uint64_t x = i + j;
            key = (key << b) | (x < n1 ? t[x] : 0);
        }
        keys[i] = key;
        vals[i] = (uint32_t)i;
    }
}

// hv[r] = r if r starts a new key group, else 0 (max-scan gives the group head)
__global__ __launch_bounds__(256) void k_heads(const uint64_t *__restrict__ keys, uint64_t m, uint32_t *__restrict__ hv,
                                               uint8_t *__restrict__ active) {
    for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r < m; r += (uint64_t)gridDim.x * 256) {
        const uint64_t k = keys[r];
        const bool eq_prev = r > 0 && keys[r - 1] == k;
        const bool eq_next = r + 1 < m && keys[r + 1] == k;
        hv[r] = eq_prev ? 0u : (uint32_t)r;
        active[r] = (eq_prev || eq_next) ? 1 : 0;
    }
}

// initial ranks: ISA[SA[r]] = head slot of r's group
__global__ __launch_bounds__(256) void k_isa_init(const uint32_t *__restrict__ sa, const uint32_t *__restrict__ grp,
                                                  uint64_t m, uint32_t *__restrict__ isa) {
    for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r < m; r += (uint64_t)gridDim.x * 256) isa[sa[r]] = grp[r];
}

__global__ __launch_bounds__(256) void k_iota(uint32_t *__restrict__ v, uint64_t m) {
    for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r < m; r += (uint64_t)gridDim.x * 256) v[r] = (uint32_t)r;
}

// doubling round keys: (rank of i, rank of i+h) for each unresolved slot
__global__ __launch_bounds__(256) void k_round_keys(const uint32_t *__restrict__ act, uint64_t m,
                                                    const uint32_t *__restrict__ sa, const uint32_t *__restrict__ isa,
                                                    uint64_t h, uint64_t *__restrict__ keys, uint32_t *__restrict__ vals) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) {
        const uint32_t i = sa[act[j]];
        keys[j] = ((uint64_t)isa[i] << 32) | isa[(uint64_t)i + h];
        vals[j] = i;
    }
}

__global__ __launch_bounds__(256) void k_round_write(const uint32_t *__restrict__ act, uint64_t m,
                                                     const uint32_t *__restrict__ vals, const uint32_t *__restrict__ hj,
                                                     uint32_t *__restrict__ sa, uint32_t *__restrict__ isa) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) {
        const uint32_t i = vals[j];
        sa[act[j]] = i;
        isa[i] = act[hj[j]];
    }
}

// ------------------------------------------------------- 3. BWT / SA

template <typename I>
__global__ void k_find_pidx(const I *__restrict__ sa, uint64_t n1, unsigned long long *__restrict__ out) {
    for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r < n1; r += (uint64_t)gridDim.x * 256)
        if (sa[r] == 0) *out = r;
}

// stored BWT = full BWT without the sentinel row pidx (bwt.remove(pidx))
template <typename I>
__global__ __launch_bounds__(256) void k_bwt(const uint8_t *__restrict__ t, const I *__restrict__ sa, uint64_t n,
                                             const unsigned long long *__restrict__ pidx, uint8_t *__restrict__ bwt) {
    const uint64_t pi = *pidx;
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < n; j += (uint64_t)gridDim.x * 256) {
        const uint64_t r = j < pi ? j : j + 1;
        bwt[j] = t[(uint64_t)sa[r] - 1];
    }
}

// sampled SA: SA.remove(0); step_by(sr)  (crate_bio_manual/mod.rs:18-21)
template <typename P, typename I>
__global__ __launch_bounds__(256) void k_sample_sa(const I *__restrict__ sa, uint64_t sa_len, uint64_t sr,
                                                   P *__restrict__ out) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < sa_len; j += (uint64_t)gridDim.x * 256)
        out[j] = (P)sa[1 + j * sr];
}

template <typename P>
__global__ void k_put_pidx(const unsigned long long *__restrict__ pidx, P *__restrict__ out) { *out = (P)*pidx; }

// --------------------------------------------------------- 4. occ encode

// One lane per block: bit planes MSB-first and left-aligned (vectorize +
// shift_last_offset), and the per-symbol counts of the block.
template <int N, int VB>
__global__ __launch_bounds__(256) void k_bwm_blocks(const uint8_t *__restrict__ bwt, uint64_t n, uint64_t blocks_len,
                                                    uint32_t sigma, uint8_t *__restrict__ blocks,
                                                    uint8_t *__restrict__ cnt) {
    for (uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x; q < blocks_len; q += (uint64_t)gridDim.x * 256) {
        uint64_t lo[N], hi[N];
#pragma unroll
        for (int j = 0; j < N; ++j) lo[j] = hi[j] = 0;
        const uint64_t b0 = q * VB;
        const uint32_t len = b0 >= n ? 0 : (uint32_t)(n - b0 < VB ? n - b0 : VB);
        for (uint32_t o = 0; o < len; ++o) {
            const uint32_t s = (uint32_t)bwt[b0 + o] - 1;
            const uint32_t bit = VB - 1 - o;
#pragma unroll
            for (int j = 0; j < N; ++j) {
                if ((s >> j) & 1u) {
                    if (bit >= 64) hi[j] |= 1ull << (bit - 64);
                    else lo[j] |= 1ull << bit;
                }
            }
        }
        // per-symbol counts over the valid (top `len`) bits
        uint64_t vlo, vhi;
        if (VB == 128) {
            vhi = len >= 64 ? ~0ull : (len ? (~0ull << (64 - len)) : 0ull);
            vlo = len > 64 ? (~0ull << (128 - len)) : 0ull;
            if (len == 128) vlo = ~0ull;
        } else {
            vhi = 0;
            vlo = len == 0 ? 0ull : ((VB == 64 ? ~0ull : 0xFFFFFFFFull) & ~((len == VB) ? 0ull : ((1ull << (VB - len)) - 1)));
        }
        for (uint32_t c = 0; c < sigma; ++c) {
            uint64_t ml = vlo, mh = vhi;
#pragma unroll
            for (int j = 0; j < N; ++j) {
                const bool bset = (c >> j) & 1u;
                ml &= bset ? lo[j] : ~lo[j];
                mh &= bset ? hi[j] : ~hi[j];
            }
            cnt[q * sigma + c] = (uint8_t)(__popcll(ml) + __popcll(mh));
        }
        uint8_t *dst = blocks + q * (uint64_t)(N * VB / 8);
#pragma unroll
        for (int j = 0; j < N; ++j) {
            if (VB == 32) reinterpret_cast<uint32_t *>(dst)[j] = (uint32_t)lo[j];
            else if (VB == 64) reinterpret_cast<uint64_t *>(dst)[j] = lo[j];
            else { reinterpret_cast<uint64_t *>(dst)[2 * j] = lo[j]; reinterpret_cast<uint64_t *>(dst)[2 * j + 1] = hi[j]; }
        }
    }
}

// 256-thread block-wide exclusive scan of one u64 per thread.
__device__ uint64_t block_excl_scan(uint64_t v, uint64_t *total, uint64_t *sh /*[4]*/) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    uint64_t before = 0, all = 0;
    for (int i = 0; i < 4; ++i) {
        if (i < w) before += sh[i];
        all += sh[i];
    }
    __syncthreads();
    *total = all;
    return before + x - v;
}

constexpr int kChunkBlocks = 1024;  // 256 threads x 4 blocks

__global__ __launch_bounds__(256) void k_chunk_totals(const uint8_t *__restrict__ cnt, uint64_t blocks_len,
                                                      uint32_t sigma, uint64_t *__restrict__ tot) {
    __shared__ uint64_t sh[4];
    const uint64_t g = blockIdx.x, q0 = g * kChunkBlocks + threadIdx.x * 4;
    for (uint32_t c = 0; c < sigma; ++c) {
        uint64_t s = 0;
        for (int t = 0; t < 4; ++t)
            if (q0 + t < blocks_len) s += cnt[(q0 + t) * sigma + c];
        uint64_t total;
        block_excl_scan(s, &total, sh);
        if (threadIdx.x == 0) tot[g * sigma + c] = total;
    }
}

// rank_checkpoints[q*sigma + c] = occurrences of c before block q (bwm/mod.rs:121-135)
template <typename P>
__global__ __launch_bounds__(256) void k_ckpt(const uint8_t *__restrict__ cnt, uint64_t blocks_len, uint32_t sigma,
                                              const uint64_t *__restrict__ base, P *__restrict__ ckpt) {
    __shared__ uint64_t sh[4];
    const uint64_t g = blockIdx.x, q0 = g * kChunkBlocks + threadIdx.x * 4;
    for (uint32_t c = 0; c < sigma; ++c) {
        uint8_t v[4];
        uint64_t s = 0;
        for (int t = 0; t < 4; ++t) {
            v[t] = q0 + t < blocks_len ? cnt[(q0 + t) * sigma + c] : 0;
            s += v[t];
        }
        uint64_t total;
        uint64_t run = base[g * sigma + c] + block_excl_scan(s, &total, sh);
        for (int t = 0; t < 4; ++t) {
            if (q0 + t < blocks_len) ckpt[(q0 + t) * sigma + c] = (P)run;
            run += v[t];
        }
    }
}

// ------------------------------------------------------------------ driver

template <class F>
static hipError_t with_temp(size_t bytes, F &&f) {
    DBuf tmp;
    hipError_t e = tmp.alloc(bytes);
    if (e != hipSuccess) return e;
    return f(tmp.p);
}

static hipError_t sort_pairs(uint64_t *&keys, uint64_t *&keys_alt, uint32_t *&vals, uint32_t *&vals_alt, size_t m,
                             unsigned begin_bit, unsigned end_bit, hipStream_t s) {
    rocprim::double_buffer<uint64_t> kb(keys, keys_alt);
    rocprim::double_buffer<uint32_t> vb(vals, vals_alt);
    size_t tb = 0;
    hipError_t e = rocprim::radix_sort_pairs(nullptr, tb, kb, vb, m, begin_bit, end_bit, s);
    if (e != hipSuccess) return e;
    e = with_temp(tb, [&](void *tmp) { return rocprim::radix_sort_pairs(tmp, tb, kb, vb, m, begin_bit, end_bit, s); });
    if (e != hipSuccess) return e;
    if (kb.current() != keys) { std::swap(keys, keys_alt); }
    if (vb.current() != vals) { std::swap(vals, vals_alt); }
    return hipSuccess;
}

static hipError_t max_scan(const uint32_t *in, uint32_t *out, size_t m, hipStream_t s) {
    size_t tb = 0;
    hipError_t e = rocprim::inclusive_scan(nullptr, tb, in, out, m, rocprim::maximum<uint32_t>(), s);
    if (e != hipSuccess) return e;
    return with_temp(tb, [&](void *tmp) {
        return rocprim::inclusive_scan(tmp, tb, in, out, m, rocprim::maximum<uint32_t>(), s);
    });
}

static hipError_t select_active(const uint32_t *in, const uint8_t *flags, uint32_t *out, size_t m, uint64_t *d_count,
                                uint64_t *h_count, Stage &io, hipStream_t s) {
    size_t tb = 0;
    hipError_t e = rocprim::select(nullptr, tb, in, flags, out, d_count, m, s);
    if (e != hipSuccess) return e;
    e = with_temp(tb, [&](void *tmp) { return rocprim::select(tmp, tb, in, flags, out, d_count, m, s); });
    if (e != hipSuccess) return e;
    return io.d2h(h_count, d_count, 8, s);  // (synchronous)
}

// Suffix array of t[0..n1) (t[n1-1] == 0 unique) into sa (u32), by prefix
// doubling: sort by the packed first K0 symbols, then repeatedly re-sort only
// the unresolved groups by (rank[i], rank[i+h]), h = K0, 2K0, 4K0, ...
// Ranks are group-head slots, so every key fits 32 + 32 bits.
static fmx_status suffix_array(const uint8_t *t, uint64_t n1, uint32_t alphabet, uint32_t *sa, Stage &io,
                               hipStream_t s) {
    uint32_t b = 1;
    while ((1u << b) < alphabet) ++b;
    const uint32_t K0 = 64 / b;
    DBuf kA, kB, vA, vB, isa, hv, hjb, act, act2, flg, cntd;
    BCK(kA.alloc(n1 * 8)); BCK(kB.alloc(n1 * 8)); BCK(vA.alloc(n1 * 4)); BCK(vB.alloc(n1 * 4));
    BCK(isa.alloc(n1 * 4)); BCK(hv.alloc(n1 * 4)); BCK(hjb.alloc(n1 * 4)); BCK(act.alloc(n1 * 4));
    BCK(act2.alloc(n1 * 4)); BCK(flg.alloc(n1)); BCK(cntd.alloc(8));
    uint32_t *HV = hv.as<uint32_t>(), *HJ = hjb.as<uint32_t>(), *ISA = isa.as<uint32_t>();
    uint8_t *FL = flg.as<uint8_t>();
    {
        uint64_t *k1 = kA.as<uint64_t>(), *k2 = kB.as<uint64_t>();
        uint32_t *v1 = vA.as<uint32_t>(), *v2 = vB.as<uint32_t>();
        hipLaunchKernelGGL(k_init_keys, dim3(grid_of(n1)), dim3(256), 0, s, t, n1, b, K0, k1, v1);
        BCK(hipGetLastError());
        BCK(sort_pairs(k1, k2, v1, v2, n1, 0, b * K0, s));
        BCK(hipMemcpyAsync(sa, v1, n1 * 4, hipMemcpyDeviceToDevice, s));
        hipLaunchKernelGGL(k_heads, dim3(grid_of(n1)), dim3(256), 0, s, k1, n1, HV, FL);
        BCK(max_scan(HV, HJ, n1, s));
        hipLaunchKernelGGL(k_isa_init, dim3(grid_of(n1)), dim3(256), 0, s, sa, HJ, n1, ISA);
        hipLaunchKernelGGL(k_iota, dim3(grid_of(n1)), dim3(256), 0, s, HV, n1);
        BCK(hipGetLastError());
    }
    uint64_t m = 0;
    uint32_t *A = act.as<uint32_t>(), *A2 = act2.as<uint32_t>();
    BCK(select_active(HV, FL, A, n1, cntd.as<uint64_t>(), &m, io, s));
    for (uint64_t h = K0; m > 0; h *= 2) {
        if (h >= n1) return FMX_E_CONFIG;  // impossible with a unique sentinel
        uint64_t *k1 = kA.as<uint64_t>(), *k2 = kB.as<uint64_t>();
        uint32_t *v1 = vA.as<uint32_t>(), *v2 = vB.as<uint32_t>();
        hipLaunchKernelGGL(k_round_keys, dim3(grid_of(m)), dim3(256), 0, s, A, m, sa, ISA, h, k1, v1);
        BCK(hipGetLastError());
        BCK(sort_pairs(k1, k2, v1, v2, m, 0, 64, s));
        hipLaunchKernelGGL(k_heads, dim3(grid_of(m)), dim3(256), 0, s, k1, m, HV, FL);
        BCK(max_scan(HV, HJ, m, s));
        hipLaunchKernelGGL(k_round_write, dim3(grid_of(m)), dim3(256), 0, s, A, m, v1, HJ, sa, ISA);
        BCK(hipGetLastError());
        uint64_t m2 = 0;
        BCK(select_active(A, FL, A2, m, cntd.as<uint64_t>(), &m2, io, s));
        std::swap(A, A2);
        m = m2;
    }
    BCK(hipStreamSynchronize(s));
    return FMX_OK;
}


// ---------------------------------------------- 2b. suffix array, 64-bit
//
// For n + 1 >= 2^32 (or FMX_BUILD_SA64=1): the same prefix doubling with
// 64-bit suffix indices and ranks, made to fit HBM by bucketing the first
// sort.  Positions are counting-sorted by their first two symbols into `sa`
// (one bucket = one contiguous slot range); each bucket is then sorted alone
// by the packed first K0 symbols (64-bit keys), which assigns every slot its
// group-head rank.  The doubling rounds sort only the unresolved groups: by
// rank(i + h), then stably by rank(i) (both 64-bit keys, two stable radix
// sorts: a 128-bit key in two passes).  Transient HBM: t + sa + isa (17 B per
// text byte) plus ~49 B per element of the largest bucket (first sort) and
// 56 B per unresolved slot in a doubling round (six 8-B buffers reused across
// the round's steps + the slot list).

__global__ __launch_bounds__(256) void k_bucket_of(const uint8_t *__restrict__ t, uint64_t n1, uint32_t W,
                                                   uint32_t *__restrict__ hist) {
    extern __shared__ uint32_t lh[];
    for (uint32_t b = threadIdx.x; b < W * W; b += 256) lh[b] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n1; i += (uint64_t)gridDim.x * 256) {
        const uint32_t b = t[i] * W + (i + 1 < n1 ? t[i + 1] : 0);
        atomicAdd(&lh[b], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < W * W; b += 256) hist[(uint64_t)blockIdx.x * W * W + b] = lh[b];
}

// scatter positions into their bucket's slots; base[g * W*W + b] = first slot
// of workgroup g's positions in bucket b (exclusive scan over (b, g))
__global__ __launch_bounds__(256) void k_bucket_scatter(const uint8_t *__restrict__ t, uint64_t n1, uint32_t W,
                                                        const uint64_t *__restrict__ base, uint64_t *__restrict__ sa) {
    extern __shared__ unsigned long long cur[];
    for (uint32_t b = threadIdx.x; b < W * W; b += 256) cur[b] = base[(uint64_t)blockIdx.x * W * W + b];
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n1; i += (uint64_t)gridDim.x * 256) {
        const uint32_t b = t[i] * W + (i + 1 < n1 ? t[i + 1] : 0);
        sa[atomicAdd(&cur[b], 1ull)] = i;
    }
}

__global__ __launch_bounds__(256) void k_keys64(const uint8_t *__restrict__ t, uint64_t n1, uint32_t b, uint32_t K0,
                                                const uint64_t *__restrict__ pos, uint64_t m,
                                                uint64_t *__restrict__ keys, uint64_t *__restrict__ vals) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) {
        const uint64_t i = pos[j];
        uint64_t key = 0;
        for (uint32_t q = 0; q < K0; ++q) key = (key << b) | (i + q < n1 ? t[i + q] : 0);
        keys[j] = key;
        vals[j] = i;
    }
}

// head flags of a sorted run: hv[j] = j at a group start (keys differ from
// j-1), else 0; single[j] = the group has one member
__global__ __launch_bounds__(256) void k_heads64(const uint64_t *__restrict__ k1, const uint64_t *__restrict__ k2,
                                                 uint64_t m, uint64_t *__restrict__ hv, uint8_t *__restrict__ active) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) {
        const bool eq_prev = j > 0 && k1[j - 1] == k1[j] && (!k2 || k2[j - 1] == k2[j]);
        const bool eq_next = j + 1 < m && k1[j + 1] == k1[j] && (!k2 || k2[j + 1] == k2[j]);
        hv[j] = eq_prev ? 0ull : j;
        active[j] = (eq_prev || eq_next) ? 1 : 0;
    }
}

// first pass of one bucket (slots s0..s0+m): sa = sorted positions, isa =
// global slot of the group head, act = 1 on unresolved slots
__global__ __launch_bounds__(256) void k_bucket_write(const uint64_t *__restrict__ vals, const uint64_t *__restrict__ hj,
                                                      const uint8_t *__restrict__ flags, uint64_t m, uint64_t s0,
                                                      uint64_t *__restrict__ sa, uint64_t *__restrict__ isa,
                                                      uint8_t *__restrict__ act) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) {
        sa[s0 + j] = vals[j];
        isa[vals[j]] = s0 + hj[j];
        act[s0 + j] = flags[j];
    }
}

// a doubling round's keys for active slot list A: secondary = rank of i + h
__global__ __launch_bounds__(256) void k_round_sec(const uint64_t *__restrict__ A, uint64_t m,
                                                   const uint64_t *__restrict__ sa, const uint64_t *__restrict__ isa,
                                                   uint64_t h, uint64_t *__restrict__ keys, uint64_t *__restrict__ vals) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) {
        const uint64_t i = sa[A[j]];
        keys[j] = isa[i + h];
        vals[j] = i;
    }
}

// primary = current group-head rank of each position (after the secondary sort)
__global__ __launch_bounds__(256) void k_round_pri(const uint64_t *__restrict__ vals, uint64_t m,
                                                   const uint64_t *__restrict__ isa, uint64_t *__restrict__ pri,
                                                   uint64_t *__restrict__ idx) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) {
        pri[j] = isa[vals[j]];
        idx[j] = j;
    }
}

__global__ __launch_bounds__(256) void k_gather2(const uint64_t *__restrict__ perm, uint64_t m,
                                                 const uint64_t *__restrict__ a, const uint64_t *__restrict__ b,
                                                 uint64_t *__restrict__ ao, uint64_t *__restrict__ bo) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) {
        ao[j] = a[perm[j]];
        bo[j] = b[perm[j]];
    }
}

__global__ __launch_bounds__(256) void k_round_write64(const uint64_t *__restrict__ A, uint64_t m,
                                                       const uint64_t *__restrict__ vals, const uint64_t *__restrict__ hj,
                                                       uint64_t *__restrict__ sa, uint64_t *__restrict__ isa) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) {
        sa[A[j]] = vals[j];
        isa[vals[j]] = A[hj[j]];
    }
}

__global__ __launch_bounds__(256) void k_iota64(uint64_t *__restrict__ v, uint64_t s0, uint64_t m) {
    for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r < m; r += (uint64_t)gridDim.x * 256) v[r] = s0 + r;
}

template <class K, class V>
static hipError_t sort_pairs_db(K *&keys, K *&keys_alt, V *&vals, V *&vals_alt, size_t m, unsigned begin_bit,
                                unsigned end_bit, hipStream_t s) {
    rocprim::double_buffer<K> kb(keys, keys_alt);
    rocprim::double_buffer<V> vb(vals, vals_alt);
    size_t tb = 0;
    hipError_t e = rocprim::radix_sort_pairs(nullptr, tb, kb, vb, m, begin_bit, end_bit, s);
    if (e != hipSuccess) return e;
    e = with_temp(tb, [&](void *tmp) { return rocprim::radix_sort_pairs(tmp, tb, kb, vb, m, begin_bit, end_bit, s); });
    if (e != hipSuccess) return e;
    if (kb.current() != keys) std::swap(keys, keys_alt);
    if (vb.current() != vals) std::swap(vals, vals_alt);
    return hipSuccess;
}

static hipError_t max_scan64(const uint64_t *in, uint64_t *out, size_t m, hipStream_t s) {
    size_t tb = 0;
    hipError_t e = rocprim::inclusive_scan(nullptr, tb, in, out, m, rocprim::maximum<uint64_t>(), s);
    if (e != hipSuccess) return e;
    return with_temp(tb, [&](void *tmp) {
        return rocprim::inclusive_scan(tmp, tb, in, out, m, rocprim::maximum<uint64_t>(), s);
    });
}

// slots j in [s0, s0 + m) with flags[j] set, appended to out[*count...]
static hipError_t select_slots(const uint8_t *flags, uint64_t s0, uint64_t m, uint64_t *out, uint64_t *d_count,
                               uint64_t *h_count, Stage &io, hipStream_t s) {
    DBuf idx;
    hipError_t e = idx.alloc(m * 8);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_iota64, dim3(grid_of(m)), dim3(256), 0, s, idx.as<uint64_t>(), s0, m);
    size_t tb = 0;
    e = rocprim::select(nullptr, tb, idx.as<uint64_t>(), flags + s0, out, d_count, m, s);
    if (e != hipSuccess) return e;
    e = with_temp(tb, [&](void *tmp) {
        return rocprim::select(tmp, tb, idx.as<uint64_t>(), flags + s0, out, d_count, m, s);
    });
    if (e != hipSuccess) return e;
    return io.d2h(h_count, d_count, 8, s);  // (synchronous)
}

static fmx_status suffix_array64(const uint8_t *t, uint64_t n1, uint32_t alphabet, uint64_t *sa, Stage &io,
                                 hipStream_t s) {
    uint32_t b = 1;
    while ((1u << b) < alphabet) ++b;
    const uint32_t K0 = 64 / b, W = alphabet, B2 = W * W;
    DBuf isa, act;
    BCK(isa.alloc(n1 * 8));
    BCK(act.alloc(n1));
    uint64_t *ISA = isa.as<uint64_t>();
    uint8_t *ACT = act.as<uint8_t>();
    // ---- bucket by the first two symbols (counting sort into sa) ----------
    std::vector<uint64_t> bstart(B2 + 1, 0);
    {
        const unsigned G = grid_of(n1, 4096);
        DBuf hist, base;
        BCK(hist.alloc((uint64_t)G * B2 * 4));
        BCK(base.alloc((uint64_t)G * B2 * 8));
        hipLaunchKernelGGL(k_bucket_of, dim3(G), dim3(256), B2 * 4, s, t, n1, W, hist.as<uint32_t>());
        BCK(hipGetLastError());
        std::vector<uint32_t> hh((size_t)G * B2);
        BCK(io.d2h(hh.data(), hist.p, hh.size() * 4, s));
        std::vector<uint64_t> hb((size_t)G * B2);
        uint64_t run = 0;
        for (uint32_t bk = 0; bk < B2; ++bk) {
            bstart[bk] = run;
            for (unsigned g = 0; g < G; ++g) {
                hb[(size_t)g * B2 + bk] = run;
                run += hh[(size_t)g * B2 + bk];
            }
        }
        bstart[B2] = run;
        BCK(io.h2d(base.p, hb.data(), hb.size() * 8, s));
        hipLaunchKernelGGL(k_bucket_scatter, dim3(G), dim3(256), B2 * 8, s, t, n1, W, base.as<uint64_t>(), sa);
        BCK(hipGetLastError());
        BCK(hipStreamSynchronize(s));
    }
    // ---- each bucket sorted by its packed first K0 symbols -----------------
    uint64_t mb = 0;
    for (uint32_t bk = 0; bk < B2; ++bk) mb = std::max(mb, bstart[bk + 1] - bstart[bk]);
    {
        DBuf kA, kB, vA, vB, hv, hj, fl;
        BCK(kA.alloc(mb * 8)); BCK(kB.alloc(mb * 8)); BCK(vA.alloc(mb * 8)); BCK(vB.alloc(mb * 8));
        BCK(hv.alloc(mb * 8)); BCK(hj.alloc(mb * 8)); BCK(fl.alloc(mb));
        for (uint32_t bk = 0; bk < B2; ++bk) {
            const uint64_t s0 = bstart[bk], m = bstart[bk + 1] - s0;
            if (!m) continue;
            uint64_t *k1 = kA.as<uint64_t>(), *k2 = kB.as<uint64_t>(), *v1 = vA.as<uint64_t>(), *v2 = vB.as<uint64_t>();
            hipLaunchKernelGGL(k_keys64, dim3(grid_of(m)), dim3(256), 0, s, t, n1, b, K0, sa + s0, m, k1, v1);
            BCK(hipGetLastError());
            BCK(sort_pairs_db(k1, k2, v1, v2, m, 0, b * K0, s));
            hipLaunchKernelGGL(k_heads64, dim3(grid_of(m)), dim3(256), 0, s, k1, (const uint64_t *)nullptr, m,
                               hv.as<uint64_t>(), fl.as<uint8_t>());
            BCK(max_scan64(hv.as<uint64_t>(), hj.as<uint64_t>(), m, s));
            hipLaunchKernelGGL(k_bucket_write, dim3(grid_of(m)), dim3(256), 0, s, v1, hj.as<uint64_t>(),
                               fl.as<uint8_t>(), m, s0, sa, ISA, ACT);
            BCK(hipGetLastError());
        }
        BCK(hipStreamSynchronize(s));
    }
    // ---- active slots (unresolved groups), collected bucket by bucket ------
    uint64_t m = 0;
    DBuf alist, cntd;
    BCK(cntd.alloc(8));
    {
        // size the list: count the flags first (bounded per-bucket selects)
        std::vector<uint64_t> part(B2, 0);
        uint64_t total = 0;
        DBuf tmpl;
        BCK(tmpl.alloc(std::max<uint64_t>(mb, 1) * 8));
        for (uint32_t bk = 0; bk < B2; ++bk) {
            const uint64_t s0 = bstart[bk], mm = bstart[bk + 1] - s0;
            if (!mm) continue;
            BCK(select_slots(ACT, s0, mm, tmpl.as<uint64_t>(), cntd.as<uint64_t>(), &part[bk], io, s));
            total += part[bk];
        }
        BCK(alist.alloc(std::max<uint64_t>(total, 1) * 8));
        for (uint32_t bk = 0; bk < B2; ++bk) {
            const uint64_t s0 = bstart[bk], mm = bstart[bk + 1] - s0;
            if (!part[bk]) continue;
            uint64_t got = 0;
            BCK(select_slots(ACT, s0, mm, alist.as<uint64_t>() + m, cntd.as<uint64_t>(), &got, io, s));
            m += got;
        }
    }
    act.alloc(0);
    // ---- doubling rounds over the unresolved groups -------------------------
    uint64_t *A = alist.as<uint64_t>();
    for (uint64_t h = K0; m > 0; h *= 2) {
        if (h >= n1) return FMX_E_CONFIG;  // impossible with a unique sentinel
        // six buffers of m words, reused across the round's steps (48 B per
        // active slot, + 8 B of the slot list): after each double-buffered
        // sort the alternate buffers are free and take the next step's output
        DBuf kA, kB, vA, vB, xA, xB;
        BCK(kA.alloc(m * 8)); BCK(kB.alloc(m * 8)); BCK(vA.alloc(m * 8)); BCK(vB.alloc(m * 8));
        BCK(xA.alloc(m * 8)); BCK(xB.alloc(m * 8));
        uint64_t *k1 = kA.as<uint64_t>(), *k2 = kB.as<uint64_t>(), *v1 = vA.as<uint64_t>(), *v2 = vB.as<uint64_t>();
        hipLaunchKernelGGL(k_round_sec, dim3(grid_of(m)), dim3(256), 0, s, A, m, sa, ISA, h, k1, v1);
        BCK(hipGetLastError());
        BCK(sort_pairs_db(k1, k2, v1, v2, m, 0, 64, s));  // by rank(i + h); k2, v2 now free
        uint64_t *p1 = xA.as<uint64_t>(), *p2 = k2, *i1 = xB.as<uint64_t>(), *i2 = v2;
        hipLaunchKernelGGL(k_round_pri, dim3(grid_of(m)), dim3(256), 0, s, v1, m, ISA, p1, i1);
        BCK(hipGetLastError());
        BCK(sort_pairs_db(p1, p2, i1, i2, m, 0, 64, s));  // stably by rank(i): groups stay in slot order
        uint64_t *val2 = i2, *sec2 = p2;                    // (the second sort's free buffers)
        hipLaunchKernelGGL(k_gather2, dim3(grid_of(m)), dim3(256), 0, s, i1, m, v1, k1, val2, sec2);
        BCK(hipGetLastError());
        uint64_t *hv = v1, *hj = k1;                        // (free once gathered)
        uint8_t *fl = reinterpret_cast<uint8_t *>(i1);
        hipLaunchKernelGGL(k_heads64, dim3(grid_of(m)), dim3(256), 0, s, p1, sec2, m, hv, fl);
        BCK(max_scan64(hv, hj, m, s));
        hipLaunchKernelGGL(k_round_write64, dim3(grid_of(m)), dim3(256), 0, s, A, m, val2, hj, sa, ISA);
        BCK(hipGetLastError());
        // the next round's active slots: A[j] where fl[j] (into hv: scanned already)
        uint64_t *A2 = hv;
        uint64_t m2 = 0;
        {
            size_t tb = 0;
            BCK(rocprim::select(nullptr, tb, A, fl, A2, cntd.as<uint64_t>(), m, s));
            BCK(with_temp(tb, [&](void *tmp) {
                return rocprim::select(tmp, tb, A, fl, A2, cntd.as<uint64_t>(), m, s);
            }));
            BCK(io.d2h(&m2, cntd.p, 8, s));
        }
        BCK(hipMemcpyAsync(A, A2, m2 * 8, hipMemcpyDeviceToDevice, s));
        m = m2;
    }
    BCK(hipStreamSynchronize(s));
    return FMX_OK;
}

template <typename P>
static fmx_status build_typed(const uint8_t *d_text, uint64_t n, const uint8_t *table, uint32_t sigma, fmx_layout L,
                              uint32_t k, uint32_t sr, uint8_t *d_blob, const BlobSizes &S, Stage &io,
                              hipStream_t s) {
    const uint64_t W = sigma + 1, n1 = n + 1;
    // ---- headers (builder/mod.rs:211-231) -------------------------------
    std::vector<uint8_t> hdr(S.header, 0);
    uint8_t *h = hdr.data();
    h[0] = 'F'; h[1] = 'I'; h[2] = '0'; h[3] = '0';
    h += S.magic;
    EncTable enc;
    if (table) { memcpy(h, table, 256); memcpy(enc.v, table, 256); h += S.enc; }
    else for (int i = 0; i < 256; ++i) enc.v[i] = (uint8_t)i;
    auto w32 = [](uint8_t *p, uint32_t v) { memcpy(p, &v, 4); };
    auto w64 = [](uint8_t *p, uint64_t v) { memcpy(p, &v, 8); };
    w32(h, sigma); w32(h + 4, k); w32(h + 8, (uint32_t)W); w32(h + 12, k); w64(h + 16, S.kt_len);
    h += S.cah;
    w32(h, sr); w64(h + 8, S.sa_len);
    h += S.sah;
    w32(h, sigma); w64(h + 8, S.ckpt_len); w64(h + 16, S.blocks_len);
    BCK(hipMemsetAsync(d_blob, 0, S.total, s));
    BCK(io.h2d(d_blob, hdr.data(), S.header, s));
    uint8_t *body = d_blob + S.header;
    uint8_t *ca = body, *mult = ca + S.ca, *kt = mult + S.mult, *sa_out = kt + S.kt;
    uint8_t *sent = sa_out + S.sa, *ckpt = sent + S.sent, *blocks = ckpt + S.ckpt;

    // ---- 1. encode + count (count_array.rs:78-136) ------------------------
    DBuf tb, symc, st, kh, khs;
    BCK(tb.alloc(n1)); BCK(symc.alloc(kMaxSigma * 8)); BCK(st.alloc(4));
    BCK(hipMemsetAsync(symc.p, 0, kMaxSigma * 8, s));
    BCK(hipMemsetAsync(st.p, 0, 4, s));
    uint8_t *t = tb.as<uint8_t>();
    hipLaunchKernelGGL(k_encode, dim3(grid_of(n, 8192)), dim3(256), 0, s, d_text, n, enc, sigma, t,
                       symc.as<unsigned long long>(), st.as<uint32_t>());
    BCK(hipGetLastError());
    uint32_t hstatus = 0;
    uint64_t hsym[kMaxSigma];
    BCK(io.d2h(&hstatus, st.p, 4, s));
    BCK(io.d2h(hsym, symc.p, kMaxSigma * 8, s));
    if (hstatus) return FMX_E_SYMBOL;  // idx >= symbol_count: the reference panics
    std::vector<uint8_t> cah(W * sizeof(P)), mh(k * 8);
    uint64_t acc = 0;
    for (uint64_t c = 0; c < W; ++c) {  // accumulate_count_array (count_array.rs:139-145)
        P v = (P)acc;
        memcpy(&cah[c * sizeof(P)], &v, sizeof(P));
        if (c < sigma) acc += hsym[c];
    }
    for (uint32_t i = 0; i < k; ++i) {  // kmer_multiplier = [W^(k-1) .. W^0]
        uint64_t p = 1;
        for (uint32_t j = 0; j < k - 1 - i; ++j) p *= W;
        memcpy(&mh[i * 8], &p, 8);
    }
    BCK(io.h2d(ca, cah.data(), cah.size(), s));
    BCK(io.h2d(mult, mh.data(), mh.size(), s));
    BCK(kh.alloc(S.kt_len * 8)); BCK(khs.alloc(S.kt_len * 8));
    BCK(hipMemsetAsync(kh.p, 0, S.kt_len * 8, s));
    const size_t lds = S.kt_len <= 8192 ? S.kt_len * 4 : 0;
    if (n) hipLaunchKernelGGL(k_kmer_hist, dim3(grid_of(n, 8192)), dim3(256), lds, s, t, n, k, W, S.kt_len,
                              kh.as<unsigned long long>());
    BCK(hipGetLastError());
    {
        size_t tbytes = 0;
        BCK(rocprim::inclusive_scan(nullptr, tbytes, kh.as<uint64_t>(), khs.as<uint64_t>(), S.kt_len,
                                    rocprim::plus<uint64_t>(), s));
        BCK(with_temp(tbytes, [&](void *tmp) {
            return rocprim::inclusive_scan(tmp, tbytes, kh.as<uint64_t>(), khs.as<uint64_t>(), S.kt_len,
                                           rocprim::plus<uint64_t>(), s);
        }));
        hipLaunchKernelGGL(k_narrow<P>, dim3(grid_of(S.kt_len)), dim3(256), 0, s, khs.as<uint64_t>(), S.kt_len, (P *)kt);
        BCK(hipGetLastError());
    }
    kh.alloc(0); khs.alloc(0);

    // ---- 2. suffix array (crate_bio_manual/mod.rs:11-12) -----------------
    // 32-bit suffix indices while n + 1 < 2^32, else the bucketed 64-bit path
    const char *force64 = getenv("FMX_BUILD_SA64");
    const bool sa64 = n1 >= 0xFFFFFFFFull || (force64 && atoi(force64) != 0);
    DBuf sab;
    BCK(sab.alloc(n1 * (sa64 ? 8 : 4)));
    fmx_status fs = sa64 ? suffix_array64(t, n1, (uint32_t)W, sab.as<uint64_t>(), io, s)
                         : suffix_array(t, n1, (uint32_t)W, sab.as<uint32_t>(), io, s);
    if (fs) return fs;

    // ---- 3. pidx, stored BWT, sampled SA ----------------------------------
    DBuf pid, bw;
    BCK(pid.alloc(8)); BCK(bw.alloc(n ? n : 1));
    auto bwt_sa = [&](auto *sa_t) {
        using I = std::remove_const_t<std::remove_pointer_t<decltype(sa_t)>>;
        hipLaunchKernelGGL(k_find_pidx<I>, dim3(grid_of(n1)), dim3(256), 0, s, sa_t, n1, pid.as<unsigned long long>());
        if (n) hipLaunchKernelGGL(k_bwt<I>, dim3(grid_of(n)), dim3(256), 0, s, t, sa_t, n,
                                  pid.as<unsigned long long>(), bw.as<uint8_t>());
        if (S.sa_len) hipLaunchKernelGGL((k_sample_sa<P, I>), dim3(grid_of(S.sa_len)), dim3(256), 0, s, sa_t,
                                         S.sa_len, (uint64_t)sr, (P *)sa_out);
    };
    if (sa64) bwt_sa(sab.as<uint64_t>());
    else bwt_sa(sab.as<uint32_t>());
    hipLaunchKernelGGL(k_put_pidx<P>, dim3(1), dim3(1), 0, s, pid.as<unsigned long long>(), (P *)sent);
    BCK(hipGetLastError());
    BCK(hipStreamSynchronize(s));
    sab.alloc(0);
    tb.alloc(0);

    // ---- 4. occ blocks + checkpoints (bwm/mod.rs:91-143) ------------------
    DBuf cnt;
    BCK(cnt.alloc(S.blocks_len * sigma));
    {
        const fmx_layout &LL = L;
#define FMX_BWM(NN, VV)                                                                                     \
    hipLaunchKernelGGL((k_bwm_blocks<NN, VV>), dim3(grid_of(S.blocks_len)), dim3(256), 0, s, bw.as<uint8_t>(), \
                       n, S.blocks_len, sigma, blocks, cnt.as<uint8_t>())
#define FMX_BWM_V(NN)                                      \
    switch (LL.vec_bits) {                                 \
        case 32: FMX_BWM(NN, 32); break;                   \
        case 64: FMX_BWM(NN, 64); break;                   \
        default: FMX_BWM(NN, 128); break;                  \
    }
        switch (LL.planes) {
            case 2: FMX_BWM_V(2) break;
            case 3: FMX_BWM_V(3) break;
            case 4: FMX_BWM_V(4) break;
            case 5: FMX_BWM_V(5) break;
            default: FMX_BWM_V(6) break;
        }
#undef FMX_BWM_V
#undef FMX_BWM
        BCK(hipGetLastError());
    }
    const uint64_t chunks = (S.blocks_len + kChunkBlocks - 1) / kChunkBlocks;
    DBuf tot;
    BCK(tot.alloc(chunks * sigma * 8));
    hipLaunchKernelGGL(k_chunk_totals, dim3((unsigned)chunks), dim3(256), 0, s, cnt.as<uint8_t>(), S.blocks_len, sigma,
                       tot.as<uint64_t>());
    BCK(hipGetLastError());
    std::vector<uint64_t> htot(chunks * sigma);
    BCK(io.d2h(htot.data(), tot.p, htot.size() * 8, s));
    {
        std::vector<uint64_t> run(sigma, 0);
        for (uint64_t g = 0; g < chunks; ++g)
            for (uint32_t c = 0; c < sigma; ++c) {
                const uint64_t v = htot[g * sigma + c];
                htot[g * sigma + c] = run[c];
                run[c] += v;
            }
    }
    BCK(io.h2d(tot.p, htot.data(), htot.size() * 8, s));
    hipLaunchKernelGGL(k_ckpt<P>, dim3((unsigned)chunks), dim3(256), 0, s, cnt.as<uint8_t>(), S.blocks_len, sigma,
                       tot.as<uint64_t>(), (P *)ckpt);
    BCK(hipGetLastError());
    BCK(hipStreamSynchronize(s));
    return FMX_OK;
}

fmx_status build_device(const uint8_t *d_text, uint64_t n, const uint8_t *table, uint32_t sigma, fmx_layout L,
                        uint32_t k, uint32_t sr, uint8_t *d_blob, uint64_t blob_len, hipStream_t s) {
    L.encoder = table ? FMX_ENC_TABLE : FMX_ENC_PASS;
    BlobSizes S;
    fmx_status st = blob_sizes(n, sigma, L, k, sr, &S);
    if (st) return st;
    if (blob_len != S.total) return FMX_E_CONFIG;                      // BuildError::InvalidBlobSize
    if (((uintptr_t)d_blob) % (L.vec_bits == 128 ? 16 : 8)) return FMX_E_ALIGN;  // NotAlignedBlob
    // every host <-> device copy of the build (headers, counts, totals)
    // through a pinned stage; its destructor waits for the copies still in
    // flight, on every return path
    Stage io(1ull << 20);
    if (L.pos_bytes == 4) return build_typed<uint32_t>(d_text, n, table, sigma, L, k, sr, d_blob, S, io, s);
    return build_typed<uint64_t>(d_text, n, table, sigma, L, k, sr, d_blob, S, io, s);
}

}  // namespace fmx
