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

// Per-record plan + per-tile (kEmitRecs records) byte totals. One 256-thread
// block covers kTile records = 2 emit tiles; tile totals come from the four
// wave sums.
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
    const uint64_t incl = wave_incl_scan_u64(len);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 63) s_wave[wave] = incl;
    __syncthreads();
    if (threadIdx.x < kTile / kEmitRecs) {
        constexpr int wpt = kEmitRecs / 64;   // waves per emit tile
        uint64_t t = 0;
#pragma unroll
        for (int w = 0; w < wpt; ++w) t += s_wave[threadIdx.x * wpt + w];
        const uint64_t tile = uint64_t(blockIdx.x) * (kTile / kEmitRecs) + threadIdx.x;
        if (tile * kEmitRecs < a.n) a.tile_sum[tile] = t;
    }
}

// Largest r in [0, nrec) with start[r] <= x (start ascending). Records of
// length 0 share their successor's start and are never chosen for an x
// inside the tile.
__device__ __forceinline__ int find_rec(const uint64_t* start, int nrec, uint64_t x) {
    int lo = 0, hi = nrec - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (start[mid] <= x) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// Header word of a record whose header did not fit the tile's LDS budget
// (kept out of line: rare, and large when inlined).
__device__ __noinline__ uint32_t header_word_slow(const onc_msg* d, uint32_t len, uint32_t meta, uint32_t k,
                                                 const EncSrc* src) {
    return header_word(*d, len, meta, k, *src);
}

constexpr int kHdrCap = 4096;                 // header words staged per tile (16 KiB of LDS)
constexpr int kMapCap = 4096;                 // 64-byte output granules mapped per tile (256 KiB)
constexpr uint32_t kNotStaged = 0xFFFFFFFFu;

struct EmitTile {
    uint64_t start[kEmitRecs + 1];   // output offset of each record (+ tile end)
    uint64_t poff[kEmitRecs];        // payload arena offset
    uint32_t meta[kEmitRecs];        // plan_record() meta (header words etc.)
    uint32_t hoff[kEmitRecs];        // staged header: word offset in hdr[], or kNotStaged
    uint32_t hdr[kHdrCap];           // header words of the tile's records (stream order)
    uint8_t map[kMapCap];            // granule g -> record holding byte 64*(G0+g) (or record 0)
};

// Record holding output byte x (T0 <= x < T1): granule map + short walk
// over the records that start inside the granule; binary search beyond the
// mapped range.
__device__ __forceinline__ int locate(const EmitTile& T, int nrec, uint64_t G0, uint64_t x) {
    const uint64_t g = (x >> 6) - G0;
    if (g >= uint64_t(kMapCap)) return find_rec(T.start, nrec, x);
    int r = T.map[g];
    while (r + 1 < nrec && T.start[r + 1] <= x) ++r;
    return r;
}

__device__ __forceinline__ uint32_t hdr_word(const EmitTile& T, const EncArgs& a, const EncSrc& src, uint64_t r0,
                                             int r, uint32_t len, uint32_t meta, uint32_t k) {
    const uint32_t ho = T.hoff[r];
    if (ho != kNotStaged) return T.hdr[ho + k];
    return header_word_slow(a.msgs + r0 + r, len, meta, k, &src);
}

// Stream word k of tile record r; 0 outside [0, len).
__device__ __forceinline__ uint32_t tile_word(const EmitTile& T, const EncArgs& a, const EncSrc& src,
                                              uint64_t r0, int r, int64_t k) {
    const uint64_t st = T.start[r];
    const uint32_t len = uint32_t(T.start[r + 1] - st);
    if (k < 0 || 4 * k >= int64_t(len)) return 0u;
    const uint32_t meta = T.meta[r];
    const uint32_t hw = meta_hw(meta);
    if (uint64_t(k) < hw) return hdr_word(T, a, src, r0, r, len, meta, uint32_t(k));
    const uintptr_t b = src.payload_arena + T.poff[r];
    return load4_masked(b + 4 * (uint64_t(k) - hw), b + (len - 4 * hw));
}

// Byte-granular chunk: the 16 stream bytes of tile record r at output
// offsets [o, o+16) (bytes outside the record read as 0).
__device__ __forceinline__ void tile_chunk(const EmitTile& T, const EncArgs& a, const EncSrc& src, uint64_t r0,
                                           int r, uint64_t o, uint32_t out[4]) {
    const int64_t rel = int64_t(o) - int64_t(T.start[r]);
    const int64_t k0 = rel >> 2;                 // floor division
    const uint32_t sh = uint32_t(rel & 3);
    uint32_t w[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) w[i] = tile_word(T, a, src, r0, r, k0 + i);
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i] = funnel(w[i], w[i + 1], sh);
}

// Word-aligned chunk (every record of the tile starts and ends on a 4-byte
// boundary, payload sources 4-aligned): each output dword is one whole
// stream word of exactly one record.
__device__ __forceinline__ void aligned_chunk(const EmitTile& T, const EncArgs& a, const EncSrc& src, uint64_t r0,
                                              int nrec, int r, uint64_t o, uint32_t v[4]) {
    uint64_t st = T.start[r], en = T.start[r + 1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint64_t p = o + 4 * i;
        while (p >= en && r + 1 < nrec) {
            ++r;
            st = en;
            en = T.start[r + 1];
        }
        uint32_t w = 0;
        if (p >= st && p < en) {
            const uint32_t k = uint32_t((p - st) >> 2);
            const uint32_t meta = T.meta[r];
            const uint32_t hw = meta_hw(meta);
            if (k < hw) w = hdr_word(T, a, src, r0, r, uint32_t(en - st), meta, k);
            else w = gload<uint32_t>(src.payload_arena + T.poff[r] + 4ull * (k - hw));
        }
        v[i] = w;
    }
}

// enc_emit: one 256-thread workgroup per tile of kEmitRecs records.
//  1. lane per record: plan_record() again (same function as enc_len, so the
//     lengths agree), one block scan places output bytes and LDS header
//     words, the record's header words are serialised into LDS, and its
//     64-byte output granules are claimed in the granule map.
//  2. the tile's output bytes [T0, T1) are produced in 16-byte aligned
//     chunks, one chunk per lane per step, stored with global_store_dwordx4
//     (a wave writes 1 KiB contiguous per instruction). Pure-payload chunks
//     are one (unaligned) 16-byte load; other chunks assemble stream words
//     from the LDS header image and the payload arena. Chunks straddling a
//     tile boundary are written with byte stores of only this tile's bytes.
__global__ __launch_bounds__(kTile) void enc_emit_kernel(EncArgs a) {
    __shared__ EmitTile T;
    __shared__ uint64_t s_wave[kTile / 64];

    const int t = threadIdx.x;
    const uint64_t r0 = uint64_t(blockIdx.x) * kEmitRecs;
    const int nrec = int(min(uint64_t(kEmitRecs), a.n - r0));
    const uint64_t tile_base = a.tile_base[blockIdx.x];
    const EncSrc src{a.unix, reinterpret_cast<uintptr_t>(a.auth_arena),
                     reinterpret_cast<uintptr_t>(a.payload_arena)};

    onc_msg d;
    uint64_t len = 0;
    uint32_t meta = 0, hw = 0;
    bool word_aligned = true;
    if (t < nrec) {
        d = a.msgs[r0 + t];
        const RecPlan p = plan_record(d, a.unix);
        len = p.len;
        meta = p.meta;
        hw = len ? meta_hw(meta) : 0;
        word_aligned = (len & 3) == 0 && (len == 4ull * hw || ((src.payload_arena + d.payload_off) & 3) == 0);
    }
    // One scan places both the output bytes and the LDS header words:
    // (len << 16 | hw); per-tile header words < 128 * 181 < 2^16.
    uint64_t total;
    const uint64_t excl = block_excl_scan_u64<kTile>((len << 16) | hw, s_wave, &total);
    const uint64_t start = tile_base + (excl >> 16);
    const uint64_t T0 = tile_base;
    const uint64_t T1 = tile_base + (total >> 16);
    const uint64_t G0 = T0 >> 6;
    const uint32_t hoff = uint32_t(excl & 0xFFFFu);
    if (t < nrec) {
        T.start[t] = start;
        T.poff[t] = d.payload_off;
        T.meta[t] = meta;
        const bool staged = hoff + hw <= uint32_t(kHdrCap);
        T.hoff[t] = staged ? hoff : kNotStaged;
        if (len != 0 && staged) put_header_words(d, uint32_t(len), src, &T.hdr[hoff]);
        // claim the granules whose first byte lies in this record
        if (len != 0) {
            const uint64_t g_hi = min((start + len - 1) >> 6, G0 + kMapCap - 1);
            for (uint64_t g = (start + 63) >> 6; g <= g_hi; ++g) T.map[g - G0] = uint8_t(t);
        }
        a.rec_off[r0 + t] = start;
        if (len != 0 && start + len > a.out_cap) a.status[r0 + t] = ONC_ENC_WRITE_ZERO;
    }
    if (t == 0) {
        T.start[nrec] = T1;
        if (T0 & 63) T.map[0] = 0;      // granule 0 starts before the tile
    }
    const bool tile_aligned = __syncthreads_and(word_aligned) && (T0 & 3) == 0;

    const uint64_t E = min(T1, a.out_cap);
    if (E <= T0) return;
    const uint64_t c_begin = T0 >> 4;
    const uint64_t c_end = (E + 15) >> 4;

    for (uint64_t c = c_begin + t; c < c_end; c += kTile) {
        const uint64_t o = c << 4;
        const uint64_t lo = max(o, T0);
        const uint64_t hi = min(o + 16, E);
        const int r = locate(T, nrec, G0, lo);
        const uint64_t st = T.start[r];
        const uint64_t en = T.start[r + 1];
        const uint64_t pst = st + 4ull * meta_hw(T.meta[r]);
        uint32_t v[4];
        if (o >= pst && o + 16 <= en) {
            // Pure payload: one 16-byte copy.
            load16_unaligned(src.payload_arena + T.poff[r] + (o - pst), v);
        } else if (tile_aligned) {
            aligned_chunk(T, a, src, r0, nrec, r, o, v);
        } else {
            tile_chunk(T, a, src, r0, r, o, v);
            if (o + 16 > en && en < T1) {
                // The chunk runs into the next record of this tile; bytes
                // outside a record read as 0, so the two parts OR together.
                const int r2 = locate(T, nrec, G0, en);
                uint32_t b[4];
                tile_chunk(T, a, src, r0, r2, o, b);
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] |= b[i];
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
    const uint64_t tiles = num_emit_tiles(a.n);
    hipLaunchKernelGGL(enc_emit_kernel, dim3(uint32_t(tiles)), dim3(kTile), 0, s, a);
    return hipGetLastError();
}

}  // namespace onc
