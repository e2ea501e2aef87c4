// fmx_layout.hip — the layout-dependent kernels of one (P, N, V) triple:
// compiled once per triple (-DFMX_LAYOUT_P=4|8 -DFMX_LAYOUT_N=2..6
// -DFMX_LAYOUT_VB=32|64|128, csrc/Makefile: 30 objects built in parallel), each
// exporting its LayoutOps table layout_ops_<P>_<N>_<V>.  Within a triple the
// occ record encoding (blob layout, 64-B or
// 128-B interleaved records: plain, paired-chunk or symbol-mask) are dispatched
// at run time.
#include "fmx_kernels.hpp"

#if !defined(FMX_LAYOUT_P) || !defined(FMX_LAYOUT_N) || !defined(FMX_LAYOUT_VB)
#error "build with -DFMX_LAYOUT_P=4|8 -DFMX_LAYOUT_N=2..6 -DFMX_LAYOUT_VB=32|64|128"
#endif

namespace fmx {
namespace {

using P = std::conditional_t<FMX_LAYOUT_P == 4, uint32_t, uint64_t>;
constexpr int N = FMX_LAYOUT_N;

template <int VB, int R, class F>
hipError_t disp_if(F &&f) {
    if constexpr (rec_fits(sizeof(P), N, VB, R)) return f.template operator()<VB, R>();
    else return hipErrorInvalidValue;
}

template <int VB, class F>
hipError_t disp_rec(uint32_t rec, F &&f) {
    switch (rec) {
        case 0: return f.template operator()<VB, 0>();
        case 64: return disp_if<VB, 64>(f);
        case 128: return disp_if<VB, 128>(f);
        case 64 | kRecPaired: return disp_if<VB, 64 | kRecPaired>(f);
        case 128 | kRecPaired: return disp_if<VB, 128 | kRecPaired>(f);
        case 64 | kRecOneHot: return disp_if<VB, 64 | kRecOneHot>(f);
        case 128 | kRecOneHot: return disp_if<VB, 128 | kRecOneHot>(f);
        case 256 | kRecOneHot: return disp_if<VB, 256 | kRecOneHot>(f);
        case 384 | kRecOneHot: return disp_if<VB, 384 | kRecOneHot>(f);
        case 512 | kRecOneHot: return disp_if<VB, 512 | kRecOneHot>(f);
        case 256 | kRecOneHot | kRecWalk: return disp_if<VB, 256 | kRecOneHot | kRecWalk>(f);
        case 384 | kRecOneHot | kRecWalk: return disp_if<VB, 384 | kRecOneHot | kRecWalk>(f);
        case 512 | kRecOneHot | kRecWalk: return disp_if<VB, 512 | kRecOneHot | kRecWalk>(f);
        default: return hipErrorInvalidValue;
    }
}

// Multi-line symbol-mask records are picked for the faithful index only
// (fmx_load): their kernels exist in the faithful variant alone.
constexpr bool faithful_only(int rec) { return (rec & kRecOneHot) != 0 && (rec & ~15) > 128; }

// f.template operator()<VB, REC>() for this object's vector width and the record size
template <class F>
hipError_t disp(uint32_t vb, uint32_t rec, F &&f) {
    if (vb != FMX_LAYOUT_VB) return hipErrorInvalidValue;
    return disp_rec<FMX_LAYOUT_VB>(rec, f);
}

[[maybe_unused]] hipError_t op_count(const QueryArgs &qa, uint32_t vb, uint32_t rec, int var, const uint8_t *bytes,
                    const uint64_t *offs, uint64_t n, uint32_t flags, void *counts, uint32_t sb, hipStream_t s) {
    return disp(vb, rec, [&]<int VB, int R>() {
        const uint32_t lds = sb + qa.kt_lds_bytes;
        const dim3 g(grid_for(n)), b(256);
        if (var == kVarFaithful) {
            hipLaunchKernelGGL((k_count<P, N, VB, R, kVarFaithful>), g, b, lds, s, qa, bytes, offs, n, flags,
                               (P *)counts, sb);
        } else if constexpr (faithful_only(R)) {
            return hipErrorInvalidValue;
        } else if (var == kVarDerived) {
            hipLaunchKernelGGL((k_count<P, N, VB, R, kVarDerived>), g, b, lds, s, qa, bytes, offs, n, flags,
                               (P *)counts, sb);
        } else {
            hipLaunchKernelGGL((k_count<P, N, VB, R, kVarDerivedLong>), g, b, lds, s, qa, bytes, offs, n, flags,
                               (P *)counts, sb);
        }
        return hipGetLastError();
    });
}

[[maybe_unused]] hipError_t op_search(const QueryArgs &qa, uint32_t vb, uint32_t rec, int var, const LocateGroup &grp,
                     uint32_t tiles, uint32_t sb, hipStream_t s) {
    return disp(vb, rec, [&]<int VB, int R>() {
        const uint32_t lds = sb + qa.kt_lds_bytes;
        if (var == kVarFaithful && grp.tile_ctr) {
            // resident-sized grid: workgroups per CU at this LDS size x CUs
            int per_cu = 0, dev = 0, cus = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_search_tiles<P, N, VB, R, kVarFaithful>, 256,
                                                             lds) != hipSuccess ||
                hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
                return hipErrorInvalidValue;
            const uint32_t grid = std::min<uint32_t>(tiles, (uint32_t)std::max(1, per_cu * cus));
            hipLaunchKernelGGL((k_search_tiles<P, N, VB, R, kVarFaithful>), dim3(grid), dim3(256), lds, s, qa, grp, sb,
                               tiles);
        } else if (var == kVarFaithful) {
            hipLaunchKernelGGL((k_search<P, N, VB, R, kVarFaithful>), dim3(tiles), dim3(256), lds, s, qa, grp, sb);
        } else if constexpr (faithful_only(R)) {
            return hipErrorInvalidValue;
        } else if (var == kVarDerived) {
            hipLaunchKernelGGL((k_search<P, N, VB, R, kVarDerived>), dim3(tiles), dim3(256), lds, s, qa, grp, sb);
        } else {
            hipLaunchKernelGGL((k_search<P, N, VB, R, kVarDerivedLong>), dim3(tiles), dim3(256), lds, s, qa, grp,
                               sb);
        }
        return hipGetLastError();
    });
}

[[maybe_unused]] hipError_t op_emit(const QueryArgs &qa, uint32_t vb, uint32_t rec, const LocateGroup &grp, uint32_t tiles,
                   uint32_t fold, hipStream_t s) {
    return disp(vb, rec, [&]<int VB, int R>() {
        hipLaunchKernelGGL((k_emit<P, N, VB, R>), dim3(tiles), dim3(256), 0, s, qa, grp, fold);
        return hipGetLastError();
    });
}

[[maybe_unused]] hipError_t op_search_grouped(const QueryArgs &qa, uint32_t vb, uint32_t rec, const LocateGroup &grp,
                                              uint64_t total, uint32_t cap, uint32_t pair, uint32_t opts,
                                              hipStream_t s) {
    return disp(vb, rec, [&]<int VB, int R>() {
        const uint32_t per = pair ? 512u : 256u;
        const uint64_t grid = (total + per - 1) / per;
        if (grid == 0 || grid > 0x7FFFFFFFull || cap == 0 || cap > kGroupRawStage) return hipErrorInvalidValue;
        if (pair)
            hipLaunchKernelGGL((k_search_grouped<P, N, VB, R, 2>), dim3((uint32_t)grid), dim3(256),
                               grouped_pat_bytes(2, cap, 0) + qa.kt_lds_bytes, s, qa, grp, total, cap, opts & 0xffu);
        else
            hipLaunchKernelGGL((k_search_grouped<P, N, VB, R, 1>), dim3((uint32_t)grid), dim3(256),
                               grouped_pat_bytes(1, cap, opts >> 8) + qa.kt_lds_bytes, s, qa, grp, total, cap,
                               opts);
        return hipGetLastError();
    });
}

[[maybe_unused]] hipError_t op_dlut_level(const QueryArgs &qa, uint32_t vb, uint32_t rec, const void *parent, uint64_t np,
                         void *child, hipStream_t s) {
    return disp(vb, rec, [&]<int VB, int R>() {
        if constexpr (faithful_only(R)) {
            return hipErrorInvalidValue;
        } else {
            hipLaunchKernelGGL((k_dlut_level<P, N, VB, R>), dim3(grid_dlut(np)), dim3(256), 0, s, qa,
                               (const P *)parent, np, (P *)child);
            return hipGetLastError();
        }
    });
}

[[maybe_unused]] hipError_t op_full_sa(const QueryArgs &qa, uint32_t vb, uint32_t rec, uint64_t n, void *sa_out, uint32_t stride,
                      hipStream_t s) {
    return disp(vb, rec, [&]<int VB, int R>() {
        if constexpr (faithful_only(R)) {
            return hipErrorInvalidValue;
        } else {
            hipLaunchKernelGGL((k_full_sa<P, N, VB, R>), dim3(grid_stride_for(n)), dim3(256), 0, s, qa, n,
                               (P *)sa_out, stride);
            return hipGetLastError();
        }
    });
}

[[maybe_unused]] hipError_t op_relayout(const QueryArgs &qa, uint32_t vb, uint32_t rec, uint64_t blocks_len, uint8_t *occ,
                       hipStream_t s) {
    return disp(vb, rec, [&]<int VB, int R>() {
        if constexpr (R != 0) {
            hipLaunchKernelGGL((k_relayout<P, N, VB, R>), dim3(grid_for(blocks_len)), dim3(256), 0, s, qa,
                               blocks_len, occ);
            return hipGetLastError();
        } else {
            return hipErrorInvalidValue;
        }
    });
}

[[maybe_unused]] hipError_t op_locate(const QueryArgs &qa, uint32_t vb, uint32_t rec, int var, const LocateGroup &grp,
                                      uint32_t tiles, uint32_t sb, uint64_t tag, uint64_t late_ticks, hipStream_t s) {
    return disp(vb, rec, [&]<int VB, int R>() {
        const uint32_t lds = sb + qa.kt_lds_bytes;
        if (var == kVarFaithful) {
            hipLaunchKernelGGL((k_locate<P, N, VB, R, kVarFaithful>), dim3(tiles), dim3(256), lds, s, qa, grp, sb, tag,
                               late_ticks);
        } else if constexpr (faithful_only(R)) {
            return hipErrorInvalidValue;
        } else if (var == kVarDerived) {
            hipLaunchKernelGGL((k_locate<P, N, VB, R, kVarDerived>), dim3(tiles), dim3(256), lds, s, qa, grp, sb, tag,
                               late_ticks);
        } else {
            hipLaunchKernelGGL((k_locate<P, N, VB, R, kVarDerivedLong>), dim3(tiles), dim3(256), lds, s, qa, grp, sb,
                               tag, late_ticks);
        }
        return hipGetLastError();
    });
}

[[maybe_unused]] hipError_t op_emit_chain(const QueryArgs &qa, uint32_t vb, uint32_t rec, const LocateGroup &grp,
                                          uint32_t tiles, uint64_t tag, uint64_t late_ticks, hipStream_t s) {
    return disp(vb, rec, [&]<int VB, int R>() {
        hipLaunchKernelGGL((k_emit_chain<P, N, VB, R>), dim3(tiles), dim3(256), 0, s, qa, grp, tag, late_ticks);
        return hipGetLastError();
    });
}

}  // namespace

#if !defined(__HIP_DEVICE_COMPILE__)  // a host table (the device pass only instantiates the kernels)
#define FMX_OPS_NAME2(p, n, v) layout_ops_##p##_##n##_##v
#define FMX_OPS_NAME(p, n, v) FMX_OPS_NAME2(p, n, v)
extern const LayoutOps FMX_OPS_NAME(FMX_LAYOUT_P, FMX_LAYOUT_N, FMX_LAYOUT_VB);
const LayoutOps FMX_OPS_NAME(FMX_LAYOUT_P, FMX_LAYOUT_N, FMX_LAYOUT_VB) = {op_count, op_search, op_emit, op_search_grouped,
                                                           op_dlut_level, op_full_sa, op_relayout, op_locate,
                                                           op_emit_chain};
#endif

}  // namespace fmx
