// TEST INFRASTRUCTURE — what libfmx_simt.so leaves out: the GPU blob builder
// (fmx_build.hip, rocPRIM radix sorts) is not emulated; the CPU tests build
// their blobs with the oracle's builder (oracle/fmx_oracle.c).
#include "../../sview-fmindex_amd/csrc/fmx_internal.hpp"

namespace fmx {
fmx_status build_device(const uint8_t *, uint64_t, const uint8_t *, uint32_t, fmx_layout, uint32_t, uint32_t,
                        uint8_t *, uint64_t, hipStream_t) {
    return FMX_E_DEVICE;
}
}  // namespace fmx
