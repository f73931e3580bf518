// scan.hip — record-offset placement (exclusive prefix sums of lengths).
//
// Variable record lengths are placed by a two-level scan: a per-tile
// (256 records, 4 waves) wavefront __shfl scan combined through LDS, and a
// single-workgroup scan of the tile totals. The encoder fuses the per-tile
// level into enc_len / enc_emit; onc_scan_lengths (decode input framing)
// uses len_tiles -> scan_tiles -> len_apply.
#include "common.h"
#include "kernels.h"

namespace onc {

// Exclusive scan of `count` u64 totals by one 1024-thread workgroup. Each
// thread owns a contiguous segment and reads it in batches of 8 independent
// loads (one memory latency per batch, not per element); the per-thread
// sums are combined by the wavefront __shfl + LDS block scan.
__global__ __launch_bounds__(kScanThreads) void scan_tiles_kernel(const uint64_t* in, uint64_t* out,
                                                                    uint64_t count, uint64_t base,
                                                                    uint64_t* total_out) {
    __shared__ uint64_t s_wave[kScanThreads / 64];
    constexpr int kB = 8;
    const uint64_t per = (count + kScanThreads - 1) / kScanThreads;
    const uint64_t lo = min(count, uint64_t(threadIdx.x) * per);
    const uint64_t hi = min(count, lo + per);
    uint64_t sum = 0;
    for (uint64_t j = lo; j < hi; j += kB) {
        uint64_t v[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) v[k] = j + k < hi ? in[j + k] : 0;
#pragma unroll
        for (int k = 0; k < kB; ++k) sum += v[k];
    }
    uint64_t total;
    const uint64_t excl = block_excl_scan_u64<kScanThreads>(sum, s_wave, &total);
    uint64_t run = base + excl;
    for (uint64_t j = lo; j < hi; j += kB) {
        uint64_t v[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) v[k] = j + k < hi ? in[j + k] : 0;
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            if (j + k < hi) out[j + k] = run;
            run += v[k];
        }
    }
    if (threadIdx.x == 0 && total_out) *total_out = base + total;
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

hipError_t launch_scan_tiles(const uint64_t* in, uint64_t* out_excl, uint64_t count, uint64_t base,
                             uint64_t* total_out, hipStream_t s) {
    hipLaunchKernelGGL(scan_tiles_kernel, dim3(1), dim3(kScanThreads), 0, s, in, out_excl, count, base,
                       total_out);
    return hipGetLastError();
}

hipError_t launch_len_tiles(const uint32_t* len, uint64_t n, uint64_t* tile_sum, hipStream_t s) {
    hipLaunchKernelGGL(len_tiles_kernel, dim3(uint32_t(num_tiles(n))), dim3(kTile), 0, s, len, n, tile_sum);
    return hipGetLastError();
}

hipError_t launch_len_apply(const uint32_t* len, uint64_t n, const uint64_t* tile_base, uint64_t* rec_off,
                            hipStream_t s) {
    hipLaunchKernelGGL(len_apply_kernel, dim3(uint32_t(num_tiles(n))), dim3(kTile), 0, s, len, n, tile_base,
                       rec_off);
    return hipGetLastError();
}

}  // namespace onc
