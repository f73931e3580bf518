// compact.hip — drop the bytes of failing records from an encoded batch
// (onc_compact / onc_compact_iov, include/onc_rpc.h).
//
// The reference's serialise_into writes nothing for a message that fails:
// its construction and auth checks panic before a byte is written
// (unix_params.rs:47,149, flavor.rs:110), and a receiver frames the stream
// record by record (expected_message_len, rpc_message.rs:343-367). The batch
// encode keeps one kind of failing record in the output: a declared
// AUTH_UNIX credential failing its deferred block check keeps its extent as
// a framable placeholder (include/onc_rpc.h onc_auth), so that the records
// after it stay where the length pass placed them. These kernels take those
// extents out afterwards, so that the buffer holds exactly the stream the
// reference's per-message loop would have written for the OK messages.
//
//   compact_lens    kept length of every record (0 for status != OK) and the
//                   first record with an extent to drop (atomicMin)
//   (scan)          onc_scan_lengths of the kept lengths: the new offsets
//   compact_info    one lane: the moved range, into mapped host memory
//   compact_gather  wave per 64-record tile of the moved records: their kept
//                   bytes packed into scratch, 16-byte chunks (one unaligned
//                   dwordx4 load when the chunk lies in one record)
//   (copy)          scratch -> the buffer at the first dropped extent
//   compact_offsets the new offsets into rec_off
// Only the records from the first dropped extent on move; a batch without
// one moves nothing.
#include "common.h"
#include "kernels.h"

namespace onc {

constexpr int kCmpThreads = 256;

__global__ __launch_bounds__(kCmpThreads) void compact_lens_kernel(const uint64_t* rec_off, const int32_t* status,
                                                                   uint64_t n, uint32_t* lens,
                                                                   unsigned long long* first_drop) {
    const uint64_t i = uint64_t(blockIdx.x) * kCmpThreads + threadIdx.x;
    if (i >= n) return;
    const uint64_t len = rec_off[i + 1] - rec_off[i];
    const bool ok = status[i] == ONC_OK;
    lens[i] = ok ? uint32_t(len) : 0u;
    if (!ok && len != 0) atomicMin(first_drop, static_cast<unsigned long long>(i));
}

// info[0] first dropped record (n: none), [1] rec_off[0], [2] its old start,
// [3] old end (rec_off[n]), [4] new end
__global__ void compact_info_kernel(const uint64_t* rec_off, const uint64_t* new_off, uint64_t n,
                                    const unsigned long long* first_drop, uint64_t* info) {
    if (threadIdx.x != 0) return;
    const uint64_t fb = min(uint64_t(*first_drop), n);
    const uint64_t base = rec_off[0];
    info[0] = fb;
    info[1] = base;
    info[2] = rec_off[fb];
    info[3] = rec_off[n];
    info[4] = base + new_off[n];
}

// Wave per tile of 64 records from `fb` on: the tile's kept bytes, in record
// order, into scratch at (base + new_off[r]) - lo (lo: the first dropped
// record's old start = where the moved bytes begin in both layouts).
__global__ __launch_bounds__(kCmpThreads) void compact_gather_kernel(const uint8_t* out, const uint64_t* rec_off,
                                                                     const uint64_t* new_off, uint64_t fb, uint64_t n,
                                                                     uint64_t base, uint64_t lo, uint8_t* scratch) {
    __shared__ uint64_t s_dst[kCmpThreads / 64][65];
    __shared__ uint64_t s_src[kCmpThreads / 64][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t r0 = fb + (uint64_t(blockIdx.x) * (kCmpThreads / 64) + wv) * 64;
    if (r0 >= n) return;                                   // wave-uniform
    const int nrec = int(min(uint64_t(64), n - r0));
    uint64_t* dst = s_dst[wv];
    uint64_t* src = s_src[wv];
    if (lane < nrec) {
        dst[lane] = base + new_off[r0 + lane] - lo;        // scratch coordinates
        src[lane] = rec_off[r0 + lane];
    }
    if (lane == 0) dst[nrec] = base + new_off[r0 + nrec] - lo;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t D0 = dst[0], D1 = dst[nrec];
    if (D1 <= D0) return;
    const uintptr_t ob = reinterpret_cast<uintptr_t>(out);
    for (uint64_t c = (D0 >> 4) + lane; c <= (D1 - 1) >> 4; c += 64) {
        const uint64_t cb = c << 4;
        const uint64_t a = max(cb, D0), e = min(cb + 16, D1);
        // record holding byte a: the last one starting at or before it (a
        // dropped record has no bytes: it starts where the next kept one does)
        int j = 0;
        for (int step = 32; step; step >>= 1)
            if (j + step < nrec && dst[j + step] <= a) j += step;
        uint32_t v[4] = {0u, 0u, 0u, 0u};
        if (e - a == 16 && dst[j + 1] >= e) {
            load16_unaligned(ob + src[j] + (a - dst[j]), v);
            *reinterpret_cast<uint4*>(scratch + cb) = make_uint4(v[0], v[1], v[2], v[3]);
            continue;
        }
        for (uint64_t p = a; p < e; ++p) {
            while (p >= dst[j + 1]) ++j;
            scratch[p] = out[src[j] + (p - dst[j])];
        }
    }
}

__global__ __launch_bounds__(kCmpThreads) void compact_offsets_kernel(uint64_t* rec_off, const uint64_t* new_off,
                                                                      uint64_t fb, uint64_t n, uint64_t base) {
    const uint64_t i = fb + uint64_t(blockIdx.x) * kCmpThreads + threadIdx.x;
    if (i <= n) rec_off[i] = base + new_off[i];
}

// onc_compact_iov: kept (header + payload) lengths; then, with their scan,
// the entries rewritten: a failing record's lengths 0, every wire_off the
// kept bytes before it; totals = {kept header bytes, kept wire bytes}.
__global__ __launch_bounds__(kCmpThreads) void compact_iov_lens_kernel(const onc_iov_rec* iov, const int32_t* status,
                                                                       uint64_t n, uint32_t* lens) {
    const uint64_t i = uint64_t(blockIdx.x) * kCmpThreads + threadIdx.x;
    if (i >= n) return;
    const onc_iov_rec r = iov[i];
    lens[i] = status[i] == ONC_OK ? r.hdr_len + r.payload_len : 0u;
}

__global__ __launch_bounds__(kCmpThreads) void compact_iov_apply_kernel(onc_iov_rec* iov, const int32_t* status,
                                                                        uint64_t n, const uint64_t* new_off,
                                                                        unsigned long long* totals) {
    __shared__ uint64_t s_wave[kCmpThreads / 64];
    const uint64_t i = uint64_t(blockIdx.x) * kCmpThreads + threadIdx.x;
    uint64_t hdr = 0;
    if (i < n) {
        onc_iov_rec r = iov[i];
        if (status[i] != ONC_OK) {
            r.hdr_len = 0;
            r.payload_len = 0;
        }
        hdr = r.hdr_len;
        r.wire_off = new_off[i];
        iov[i] = r;
        if (i + 1 == n && totals) totals[1] = new_off[n];
    }
    uint64_t total;
    block_excl_scan_u64<kCmpThreads>(hdr, s_wave, &total);
    if (threadIdx.x == 0 && totals && total) atomicAdd(totals, static_cast<unsigned long long>(total));
}

static uint32_t blocks_of(uint64_t n) { return uint32_t((n + kCmpThreads - 1) / kCmpThreads); }

hipError_t launch_compact_lens(const uint64_t* rec_off, const int32_t* status, uint64_t n, uint32_t* lens,
                               uint64_t* first_drop, hipStream_t s) {
    ONC_LAUNCH(compact_lens_kernel, dim3(blocks_of(n)), dim3(kCmpThreads), 0, s, rec_off, status, n, lens,
               reinterpret_cast<unsigned long long*>(first_drop));
    return hipGetLastError();
}

hipError_t launch_compact_info(const uint64_t* rec_off, const uint64_t* new_off, uint64_t n,
                               const uint64_t* first_drop, uint64_t* info, hipStream_t s) {
    ONC_LAUNCH(compact_info_kernel, dim3(1), dim3(64), 0, s, rec_off, new_off, n,
               reinterpret_cast<const unsigned long long*>(first_drop), info);
    return hipGetLastError();
}

hipError_t launch_compact_gather(const uint8_t* out, const uint64_t* rec_off, const uint64_t* new_off, uint64_t fb,
                                 uint64_t n, uint64_t base, uint64_t lo, uint8_t* scratch, hipStream_t s) {
    const uint64_t tiles = (n - fb + 63) / 64;
    ONC_LAUNCH(compact_gather_kernel, dim3(uint32_t((tiles + 3) / 4)), dim3(kCmpThreads), 0, s, out, rec_off, new_off,
               fb, n, base, lo, scratch);
    return hipGetLastError();
}

hipError_t launch_compact_offsets(uint64_t* rec_off, const uint64_t* new_off, uint64_t fb, uint64_t n, uint64_t base,
                                  hipStream_t s) {
    ONC_LAUNCH(compact_offsets_kernel, dim3(blocks_of(n - fb + 1)), dim3(kCmpThreads), 0, s, rec_off, new_off, fb, n,
               base);
    return hipGetLastError();
}

hipError_t launch_compact_iov_lens(const onc_iov_rec* iov, const int32_t* status, uint64_t n, uint32_t* lens,
                                   hipStream_t s) {
    ONC_LAUNCH(compact_iov_lens_kernel, dim3(blocks_of(n)), dim3(kCmpThreads), 0, s, iov, status, n, lens);
    return hipGetLastError();
}

hipError_t launch_compact_iov_apply(onc_iov_rec* iov, const int32_t* status, uint64_t n, const uint64_t* new_off,
                                    uint64_t* totals, hipStream_t s) {
    ONC_LAUNCH(compact_iov_apply_kernel, dim3(blocks_of(n)), dim3(kCmpThreads), 0, s, iov, status, n, new_off,
               reinterpret_cast<unsigned long long*>(totals));
    return hipGetLastError();
}

}  // namespace onc
