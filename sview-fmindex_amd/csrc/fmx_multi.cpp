// fmx_multi.cpp — one index handle over several GPUs of one process: the
// device mask of the boundary SURVEY §8(b) sketches, for a single-process
// caller of the reference's API (FmIndex::count / locate, lib.rs:14-28) that
// has no process group.  The blob is validated like fmx_load, copied to HBM of
// the first device once and device-to-device to the others (hipMemcpyPeer:
// over xGMI between MI355X GPUs — SURVEY §8(e)'s "H2D to GPU0, then
// broadcast"), and each replica is loaded with fmx_load_device.  A host batch
// is cut into contiguous shards (sizes differ by at most one), answered
// concurrently — one host thread per replica, each through the replica's own
// host-buffer call — and the shards' results are concatenated in order: the
// answer one device gives for the whole batch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "fmx_internal.hpp"

struct fmx_multi {
    std::vector<int> devices;
    std::vector<uint8_t *> d_blobs;  // one replica per entry (owned)
    std::vector<fmx_index *> ix;
    uint64_t blob_len = 0;
    uint32_t pos_bytes = 4;
};

namespace {

using namespace fmx;

// shard p of `parts` over [0, n): contiguous, sizes differ by at most one
void shard_of(uint64_t n, uint64_t parts, uint64_t p, uint64_t &s, uint64_t &e) {
    const uint64_t base = n / parts, extra = n % parts;
    s = p * base + std::min(p, extra);
    e = s + base + (p < extra ? 1 : 0);
}

struct CurrentDevice {  // restores the caller's current device
    int prev = -1;
    CurrentDevice() {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    }
    ~CurrentDevice() {
        if (prev >= 0) hipSetDevice(prev);
    }
};

void free_multi(fmx_multi *m) {
    if (!m) return;
    for (fmx_index *x : m->ix) fmx_free(x);
    for (size_t d = 0; d < m->d_blobs.size(); ++d)
        if (m->d_blobs[d] && hipSetDevice(m->devices[d]) == hipSuccess) hipFree(m->d_blobs[d]);
    delete m;
}

// run(d) for every replica, replica 0 on the calling thread, the others on
// threads of their own (or here, one after another, if no thread can start)
template <class F>
void for_each_replica(size_t D, F &&run) {
    std::vector<std::thread> th;
    size_t d = 1;
    try {
        for (; d < D; ++d) th.emplace_back(run, d);
    } catch (...) {
        for (; d < D; ++d) run(d);
    }
    run(0);
    for (auto &t : th) t.join();
}

}  // namespace

extern "C" {

fmx_status fmx_multi_load(const uint8_t *blob, uint64_t blob_len, fmx_layout layout, const int *devices,
                          int n_devices, uint32_t options, fmx_multi **out, uint64_t *expected_total,
                          uint64_t *actual_total) {
    if (!out || !devices || n_devices <= 0 || n_devices > 64 || (!blob && blob_len)) return FMX_E_ARG;
    *out = nullptr;
    BlobView bv;
    BlobReader rd = [&](uint64_t off, uint64_t len, void *dst) {
        if (off + len > blob_len) return false;
        memcpy(dst, blob + off, len);
        return true;
    };
    fmx_status st = parse_blob(rd, blob_len, layout, &bv, expected_total, actual_total);
    if (st) return st;
    if (((uintptr_t)blob) % bv.align != 0) return FMX_E_ALIGN;
    CurrentDevice keep;
    fmx_multi *m = new (std::nothrow) fmx_multi();
    if (!m) return FMX_E_DEVICE;
    m->devices.assign(devices, devices + n_devices);
    m->d_blobs.assign(n_devices, nullptr);
    m->blob_len = blob_len;
    m->pos_bytes = layout.pos_bytes;
    const uint64_t bytes = std::max<uint64_t>(blob_len, 16);
    for (int d = 0; d < n_devices; ++d)
        if (hipSetDevice(devices[d]) != hipSuccess || hipMalloc(&m->d_blobs[d], bytes) != hipSuccess) {
            free_multi(m);
            return FMX_E_DEVICE;
        }
    // host -> the first device once (through a pinned stage: no DMA on the
    // caller's pageable blob); the first device -> every other replica
    hipError_t e = hipSetDevice(devices[0]);
    if (e == hipSuccess && blob_len) {
        Stage up(32ull << 20);
        e = up.h2d(m->d_blobs[0], blob, blob_len, nullptr);
        if (e == hipSuccess) e = up.drain();
        if (e == hipSuccess) e = hipDeviceSynchronize();
    }
    for (int d = 1; d < n_devices && e == hipSuccess; ++d)
        if (blob_len) e = hipMemcpyPeer(m->d_blobs[d], devices[d], m->d_blobs[0], devices[0], blob_len);
    if (e != hipSuccess) {
        free_multi(m);
        return FMX_E_DEVICE;
    }
    for (int d = 0; d < n_devices; ++d) {
        fmx_index *x = nullptr;
        st = fmx_load_device(m->d_blobs[d], blob_len, layout, devices[d], options, &x, nullptr, nullptr);
        if (st) {
            free_multi(m);
            return st;
        }
        m->ix.push_back(x);
    }
    *out = m;
    return FMX_OK;
}

void fmx_multi_free(fmx_multi *m) {
    CurrentDevice keep;
    free_multi(m);
}

int fmx_multi_replicas(const fmx_multi *m) { return m ? (int)m->ix.size() : 0; }

fmx_index *fmx_multi_replica(fmx_multi *m, int i) {
    return (m && i >= 0 && i < (int)m->ix.size()) ? m->ix[i] : nullptr;
}

fmx_status fmx_multi_count_batch(fmx_multi *m, const uint8_t *bytes, const uint64_t *offsets, uint64_t n,
                                 uint32_t flags, void *out_counts) {
    if (!m || (n && (!offsets || !out_counts))) return FMX_E_ARG;
    if (n == 0) return FMX_OK;
    if (offsets[0] != 0) return FMX_E_ARG;
    const size_t D = m->ix.size();
    std::vector<fmx_status> st(D, FMX_OK);
    for_each_replica(D, [&](size_t d) {
        uint64_t s, e;
        shard_of(n, D, d, s, e);
        if (e == s) return;
        std::vector<uint64_t> off(e - s + 1);
        for (uint64_t i = 0; i <= e - s; ++i) off[i] = offsets[s + i] - offsets[s];
        st[d] = fmx_count_batch(m->ix[d], bytes + offsets[s], off.data(), e - s, flags,
                                (uint8_t *)out_counts + s * m->pos_bytes);
    });
    for (fmx_status x : st)
        if (x) return x;
    return FMX_OK;
}

fmx_status fmx_multi_locate_batch(fmx_multi *m, const uint8_t *bytes, const uint64_t *offsets, uint64_t n,
                                  uint32_t flags, uint64_t *out_loc_offsets, void *out_locs, uint64_t cap,
                                  uint64_t *needed) {
    if (!m || !out_loc_offsets || (n && !offsets) || (cap && !out_locs)) return FMX_E_ARG;
    if (needed) *needed = 0;
    if (n == 0) {
        out_loc_offsets[0] = 0;
        return FMX_OK;
    }
    if (offsets[0] != 0) return FMX_E_ARG;
    const size_t D = m->ix.size();
    const uint64_t pb = m->pos_bytes;
    struct Part {
        uint64_t s = 0, e = 0, need = 0;
        std::vector<uint64_t> loff;
        std::vector<uint8_t> locs;
        fmx_status st = FMX_OK;
    };
    std::vector<Part> parts(D);
    for_each_replica(D, [&](size_t d) {
        Part &p = parts[d];
        shard_of(n, D, d, p.s, p.e);
        const uint64_t k = p.e - p.s;
        if (!k) return;
        std::vector<uint64_t> off(k + 1);
        for (uint64_t i = 0; i <= k; ++i) off[i] = offsets[p.s + i] - offsets[p.s];
        p.loff.resize(k + 1);
        uint64_t c = k + k / 8 + 64;  // a guess; the exact room if the shard has more occurrences
        p.locs.resize(c * pb);
        p.st = fmx_locate_batch(m->ix[d], bytes + offsets[p.s], off.data(), k, flags, p.loff.data(), p.locs.data(),
                                c, &p.need);
        if (p.st == FMX_E_CAPACITY) {
            c = p.need;
            p.locs.resize(std::max<uint64_t>(c, 1) * pb);
            p.st = fmx_locate_batch(m->ix[d], bytes + offsets[p.s], off.data(), k, flags, p.loff.data(),
                                    p.locs.data(), c, &p.need);
        }
    });
    for (const Part &p : parts)
        if (p.st) return p.st;
    // the batch's offsets (written whatever the capacity, as fmx_locate_batch does)
    uint64_t base = 0;
    out_loc_offsets[0] = 0;
    for (const Part &p : parts) {
        for (uint64_t i = 1; i <= p.e - p.s; ++i) out_loc_offsets[p.s + i] = base + p.loff[i];
        base += p.need;
    }
    if (needed) *needed = base;
    if (base > cap) return FMX_E_CAPACITY;
    base = 0;
    for (const Part &p : parts) {
        if (p.need) memcpy((uint8_t *)out_locs + base * pb, p.locs.data(), p.need * pb);
        base += p.need;
    }
    return FMX_OK;
}

}  // extern "C"
