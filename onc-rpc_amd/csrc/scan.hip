// scan.hip — record-offset placement (exclusive prefix sums of lengths).
//
// Variable record lengths are placed by a two-level scan: a per-tile
// (256 records, 4 waves) wavefront __shfl scan combined through LDS, and a
// single-workgroup scan of the tile totals. The encoder fuses the per-tile
// level into enc_len / enc_emit; onc_scan_lengths (decode input framing)
// uses lenblk -> lenoff up to 8M records, len_tiles -> scan_tiles ->
// len_apply beyond.
#include "common.h"
#include "kernels.h"

namespace onc {

// Exclusive scan of `count` u64 totals by one 1024-thread workgroup, in
// rows of 1024 x 16 values: each thread loads its 16 contiguous values of
// the row at once (8 dwordx4, 128 contiguous bytes per lane), keeps them in
// registers, and the per-thread sums go through the wavefront __shfl + LDS
// block scan; one memory latency per row (one row covers 16K workgroup
// totals = 16M records at 1024 records per enc_len workgroup).
constexpr int kScanPer = 16;
__global__ __launch_bounds__(kScanThreads) void scan_tiles_kernel(const uint64_t* in, uint64_t* out,
                                                                    uint64_t count, uint64_t base,
                                                                    uint64_t* total_out) {
    __shared__ uint64_t s_wave[kScanThreads / 64];
    uint64_t carry = base;
    const bool vec = ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) == 0;
    for (uint64_t row = 0; row < count; row += uint64_t(kScanThreads) * kScanPer) {
        const uint64_t lo = row + uint64_t(threadIdx.x) * kScanPer;
        uint64_t v[kScanPer];
        if (vec && lo + kScanPer <= count) {
            const ulonglong2* src = reinterpret_cast<const ulonglong2*>(in + lo);
#pragma unroll
            for (int k = 0; k < kScanPer / 2; ++k) {
                const ulonglong2 w = src[k];
                v[2 * k] = w.x;
                v[2 * k + 1] = w.y;
            }
        } else {
#pragma unroll
            for (int k = 0; k < kScanPer; ++k) v[k] = lo + k < count ? in[lo + k] : 0;
        }
        uint64_t sum = 0;
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) sum += v[k];
        uint64_t total;
        uint64_t run = carry + block_excl_scan_u64<kScanThreads>(sum, s_wave, &total);
        if (vec && lo + kScanPer <= count) {
            ulonglong2* dst = reinterpret_cast<ulonglong2*>(out + lo);
#pragma unroll
            for (int k = 0; k < kScanPer / 2; ++k) {
                const uint64_t r0 = run;
                run += v[2 * k];
                dst[k] = make_ulonglong2(r0, run);
                run += v[2 * k + 1];
            }
        } else {
#pragma unroll
            for (int k = 0; k < kScanPer; ++k) {
                if (lo + k < count) out[lo + k] = run;
                run += v[k];
            }
        }
        carry += total;
    }
    if (threadIdx.x == 0 && total_out) *total_out = carry;
}

__global__ __launch_bounds__(kTile) void len_tiles_kernel(const uint32_t* len, uint64_t n, uint64_t* tile_sum) {
    __shared__ uint64_t s_wave[kTile / 64];
    const uint64_t i = uint64_t(blockIdx.x) * kTile + threadIdx.x;
    const uint64_t v = i < n ? len[i] : 0;
    uint64_t total;
    block_excl_scan_u64<kTile>(v, s_wave, &total);
    if (threadIdx.x == 0) tile_sum[blockIdx.x] = total;
}

__global__ __launch_bounds__(kTile) void len_apply_kernel(const uint32_t* len, uint64_t n,
                                                          const uint64_t* tile_base, uint64_t* rec_off) {
    __shared__ uint64_t s_wave[kTile / 64];
    const uint64_t i = uint64_t(blockIdx.x) * kTile + threadIdx.x;
    const uint64_t v = i < n ? len[i] : 0;
    uint64_t total;
    const uint64_t excl = block_excl_scan_u64<kTile>(v, s_wave, &total);
    if (i < n) rec_off[i] = tile_base[blockIdx.x] + excl;
}

// Two-launch form of onc_scan_lengths for up to kLenBlk * kLenBlkMax
// records (8M): lenblk sums each 4096-record block; lenoff gives every
// block its base by summing the block totals before it itself (at most
// kLenBlkMax / 256 loads per thread, L2-resident) and scans its own 4096
// lengths — one launch and one dependent round trip fewer than len_tiles ->
// scan_tiles -> len_apply. Each thread owns 16 consecutive records (four
// dwordx4 length loads, eight 16-byte offset stores).
constexpr int kLenBlk = 4096;
constexpr int kLenBlkMax = 2048;
constexpr int kLenPerThread = kLenBlk / kTile;   // 16
static_assert(kLenPerThread == 16, "four uint4 loads per thread below");

__device__ __forceinline__ void load_lens16(const uint32_t* len, uint64_t n, uint64_t lo, uint32_t v[16]) {
    if (lo + 16 <= n && (reinterpret_cast<uintptr_t>(len + lo) & 15) == 0) {
        const uint4* p = reinterpret_cast<const uint4*>(len + lo);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 w = p[k];
            v[4 * k] = w.x; v[4 * k + 1] = w.y; v[4 * k + 2] = w.z; v[4 * k + 3] = w.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = lo + k < n ? len[lo + k] : 0u;
    }
}

__global__ __launch_bounds__(kTile) void lenblk_kernel(const uint32_t* len, uint64_t n, uint64_t* blk_sum) {
    __shared__ uint64_t s_wave[kTile / 64];
    uint32_t v[16];
    load_lens16(len, n, uint64_t(blockIdx.x) * kLenBlk + 16ull * threadIdx.x, v);
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) sum += v[k];
    uint64_t total;
    block_excl_scan_u64<kTile>(sum, s_wave, &total);
    if (threadIdx.x == 0) blk_sum[blockIdx.x] = total;
}

__global__ __launch_bounds__(kTile) void lenoff_kernel(const uint32_t* len, uint64_t n, const uint64_t* blk_sum,
                                                       uint64_t base, uint64_t* rec_off) {
    __shared__ uint64_t s_wave[kTile / 64];
    const uint64_t blk = blockIdx.x;
    const uint64_t lo = blk * kLenBlk + 16ull * threadIdx.x;
    uint32_t v[16];
    load_lens16(len, n, lo, v);                           // issued with the block-total loads below
    uint64_t pre = 0;
#pragma unroll
    for (int k = 0; k < kLenBlkMax / kTile; ++k) {
        const uint64_t j = uint64_t(threadIdx.x) + uint64_t(k) * kTile;
        if (j < blk) pre += blk_sum[j];
    }
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) sum += v[k];
    uint64_t pre_total, total;
    block_excl_scan_u64<kTile>(pre, s_wave, &pre_total);   // the block's base
    uint64_t run = base + pre_total + block_excl_scan_u64<kTile>(sum, s_wave, &total);
    if (lo + 16 <= n && (reinterpret_cast<uintptr_t>(rec_off + lo) & 15) == 0) {
        ulonglong2* dst = reinterpret_cast<ulonglong2*>(rec_off + lo);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint64_t r0 = run;
            run += v[2 * k];
            dst[k] = make_ulonglong2(r0, run);
            run += v[2 * k + 1];
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (lo + k < n) rec_off[lo + k] = run;
            run += v[k];
        }
    }
    // the grand total: rec_off[n] (the thread whose range ends at n)
    if (lo < n && lo + 16 >= n) rec_off[n] = run;
}

hipError_t launch_scan_tiles(const uint64_t* in, uint64_t* out_excl, uint64_t count, uint64_t base,
                             uint64_t* total_out, hipStream_t s) {
    ONC_LAUNCH(scan_tiles_kernel, dim3(1), dim3(kScanThreads), 0, s, in, out_excl, count, base,
                       total_out);
    return hipGetLastError();
}

hipError_t launch_len_tiles(const uint32_t* len, uint64_t n, uint64_t* tile_sum, hipStream_t s) {
    ONC_LAUNCH(len_tiles_kernel, dim3(uint32_t(num_tiles(n))), dim3(kTile), 0, s, len, n, tile_sum);
    return hipGetLastError();
}

hipError_t launch_len_apply(const uint32_t* len, uint64_t n, const uint64_t* tile_base, uint64_t* rec_off,
                            hipStream_t s) {
    ONC_LAUNCH(len_apply_kernel, dim3(uint32_t(num_tiles(n))), dim3(kTile), 0, s, len, n, tile_base,
                       rec_off);
    return hipGetLastError();
}

// rec_off[0] = base of an empty scan (a kernel rather than a copy from the
// host stack: no synchronisation, capturable)
__global__ void store_u64_kernel(uint64_t* p, uint64_t v) { *p = v; }

hipError_t launch_store_u64(uint64_t* p, uint64_t v, hipStream_t s) {
    ONC_LAUNCH(store_u64_kernel, dim3(1), dim3(1), 0, s, p, v);
    return hipGetLastError();
}

bool scan_lengths_fused_ok(uint64_t n) { return (n + kLenBlk - 1) / kLenBlk <= kLenBlkMax; }

hipError_t launch_lenblk(const uint32_t* len, uint64_t n, uint64_t* blk_sum, hipStream_t s) {
    ONC_LAUNCH(lenblk_kernel, dim3(uint32_t((n + kLenBlk - 1) / kLenBlk)), dim3(kTile), 0, s, len, n, blk_sum);
    return hipGetLastError();
}

hipError_t launch_lenoff(const uint32_t* len, uint64_t n, const uint64_t* blk_sum, uint64_t base, uint64_t* rec_off,
                         hipStream_t s) {
    ONC_LAUNCH(lenoff_kernel, dim3(uint32_t((n + kLenBlk - 1) / kLenBlk)), dim3(kTile), 0, s, len, n, blk_sum,
                       base, rec_off);
    return hipGetLastError();
}

}  // namespace onc
