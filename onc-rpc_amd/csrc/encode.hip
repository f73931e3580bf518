// encode.hip — batch RpcMessage::serialise_into for gfx950.
//
// Reference: RpcMessage::serialise_into (src/rpc_message.rs:136-164) and the
// serialise_into/serialised_len chain it calls (call_body.rs:98-119,
// auth/flavor.rs:106-174, auth/unix_params.rs:162-245, opaque.rs:38-63,
// reply/*). The reference is called once per message by the user's loop;
// here one launch encodes a whole batch into one contiguous send buffer.
//
// Pipeline (3 launches on one stream):
//   enc_len   lane per record: plan_record() = serialised_len + validation,
//             per-tile (256-record) byte totals.
//   scan      exclusive scan of tile totals -> tile base offsets.
//   enc_emit  per tile: block scan of record lengths (wavefront __shfl scan
//             + LDS across the 4 waves) -> record offsets; descriptors
//             staged in LDS; then the tile's output byte range is produced
//             in 16-byte aligned chunks, one chunk per lane per step, and
//             stored with global_store_dwordx4 (fully coalesced: a wave
//             writes 1 KiB contiguous per instruction). Each chunk finds its
//             record by binary search over the LDS offsets; pure-payload
//             chunks are an unaligned 16-byte copy (5 dword loads + 4
//             v_alignbyte); chunks touching header words or a record
//             boundary evaluate the XDR words directly (record_word()).
//             Chunks that straddle a tile boundary are written with byte
//             stores of only this tile's bytes, so tiles never exchange data.
#include "common.h"
#include "kernels.h"

namespace onc {

__global__ __launch_bounds__(kTile) void enc_len_kernel(EncArgs a) {
    __shared__ uint64_t s_wave[kTile / 64];
    const uint64_t r = uint64_t(blockIdx.x) * kTile + threadIdx.x;
    uint64_t len = 0;
    if (r < a.n) {
        const onc_msg d = a.msgs[r];
        const RecPlan p = plan_record(d, a.unix);
        len = p.len;
        a.status[r] = p.status;
        if (a.rec_len) a.rec_len[r] = uint32_t(len);
    }
    uint64_t total;
    block_excl_scan_u64<kTile>(len, s_wave, &total);
    if (threadIdx.x == 0) a.tile_sum[blockIdx.x] = total;
}

// Largest r in [0, nrec) with s_start[r] <= x (s_start ascending). Records
// of length 0 share their successor's start and are therefore never chosen
// for an x inside the tile.
__device__ __forceinline__ int find_rec(const uint64_t* s_start, int nrec, uint64_t x) {
    int lo = 0, hi = nrec - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_start[mid] <= x) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// The 16 stream bytes of record r that fall at output offsets [o, o+16)
// (bytes outside the record read as 0). rel = o - start may be negative.
__device__ __forceinline__ void record_chunk(const onc_msg& d, uint64_t start, uint32_t len, uint32_t meta,
                                             uint64_t o, const EncSrc& s, uint32_t out[4]) {
    const int64_t rel = int64_t(o) - int64_t(start);
    const int64_t k0 = rel >> 2;              // floor division
    const uint32_t sh = uint32_t(rel & 3);
    uint32_t w[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) w[i] = record_word(d, len, meta, k0 + i, s);
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i] = funnel(w[i], w[i + 1], sh);
}

__global__ __launch_bounds__(kTile) void enc_emit_kernel(EncArgs a) {
    __shared__ onc_msg s_desc[kTile];
    __shared__ uint64_t s_start[kTile + 1];
    __shared__ uint32_t s_meta[kTile];
    __shared__ uint64_t s_wave[kTile / 64];

    const int t = threadIdx.x;
    const uint64_t r0 = uint64_t(blockIdx.x) * kTile;
    const int nrec = int(min(uint64_t(kTile), a.n - r0));
    const uint64_t tile_base = a.tile_base[blockIdx.x];

    uint64_t len = 0;
    uint32_t meta = 0;
    if (t < nrec) {
        const onc_msg d = a.msgs[r0 + t];
        const RecPlan p = plan_record(d, a.unix);
        len = p.len;
        meta = p.meta;
        s_desc[t] = d;
    }
    uint64_t total;
    const uint64_t excl = block_excl_scan_u64<kTile>(len, s_wave, &total);
    const uint64_t start = tile_base + excl;
    if (t < nrec) {
        s_start[t] = start;
        s_meta[t] = meta;
        a.rec_off[r0 + t] = start;
        if (len != 0 && start + len > a.out_cap) a.status[r0 + t] = ONC_ENC_WRITE_ZERO;
    }
    if (t == 0) s_start[nrec] = tile_base + total;
    __syncthreads();

    const uint64_t T0 = s_start[0];
    const uint64_t T1 = s_start[nrec];
    const uint64_t E = min(T1, a.out_cap);
    if (E <= T0) return;

    const EncSrc src{a.unix, reinterpret_cast<uintptr_t>(a.auth_arena),
                     reinterpret_cast<uintptr_t>(a.payload_arena)};
    const uint64_t c_begin = T0 >> 4;
    const uint64_t c_end = (E + 15) >> 4;

    for (uint64_t c = c_begin + t; c < c_end; c += kTile) {
        const uint64_t o = c << 4;
        const uint64_t lo = max(o, T0);
        const uint64_t hi = min(o + 16, E);
        const int r = find_rec(s_start, nrec, lo);
        const uint64_t st = s_start[r];
        const uint64_t en = s_start[r + 1];
        const uint32_t rlen = uint32_t(en - st);
        const uint32_t rmeta = s_meta[r];
        const uint64_t pst = st + 4ull * meta_hw(rmeta);
        uint32_t v[4];
        if (o >= pst && o + 16 <= en) {
            // Pure payload: unaligned 16-byte copy, every byte valid.
            const uintptr_t addr = src.payload_arena + s_desc[r].payload_off + (o - pst);
            const uintptr_t al = addr & ~uintptr_t(3);
            const uint32_t sh = uint32_t(addr & 3);
            const uint32_t* p = reinterpret_cast<const uint32_t*>(al);
            const uint32_t w0 = p[0], w1 = p[1], w2 = p[2], w3 = p[3];
            const uint32_t w4 = sh ? p[4] : 0u;
            v[0] = funnel(w0, w1, sh);
            v[1] = funnel(w1, w2, sh);
            v[2] = funnel(w2, w3, sh);
            v[3] = funnel(w3, w4, sh);
        } else {
            record_chunk(s_desc[r], st, rlen, rmeta, o, src, v);
            if (o + 16 > en && en < T1) {
                // The chunk runs into the next record of this tile.
                const int r2 = find_rec(s_start, nrec, en);
                uint32_t b[4];
                record_chunk(s_desc[r2], s_start[r2], uint32_t(s_start[r2 + 1] - s_start[r2]), s_meta[r2], o,
                             src, b);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int64_t na = int64_t(en) - int64_t(o + 4 * i);
                    const uint32_t m = na >= 4 ? 0xFFFFFFFFu : (na <= 0 ? 0u : ((1u << (8 * uint32_t(na))) - 1u));
                    v[i] = (v[i] & m) | (b[i] & ~m);
                }
            }
        }
        if (lo == o && hi == o + 16) {
            *reinterpret_cast<uint4*>(a.out + o) = make_uint4(v[0], v[1], v[2], v[3]);
        } else {
            // Tile-boundary or capacity-boundary chunk: only this tile's bytes.
            for (uint64_t bpos = lo; bpos < hi; ++bpos) {
                const uint32_t j = uint32_t(bpos - o);
                a.out[bpos] = uint8_t(v[j >> 2] >> (8 * (j & 3)));
            }
        }
    }
}

hipError_t launch_enc_len(const EncArgs& a, hipStream_t s) {
    const uint64_t tiles = num_tiles(a.n);
    hipLaunchKernelGGL(enc_len_kernel, dim3(uint32_t(tiles)), dim3(kTile), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_enc_emit(const EncArgs& a, hipStream_t s) {
    const uint64_t tiles = num_tiles(a.n);
    hipLaunchKernelGGL(enc_emit_kernel, dim3(uint32_t(tiles)), dim3(kTile), 0, s, a);
    return hipGetLastError();
}

}  // namespace onc
