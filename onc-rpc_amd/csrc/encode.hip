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

// Per-record plan + per-tile byte totals: tile = kEmitRecs (64) records =
// one wavefront (its inclusive __shfl scan, lane 63 writes the total), and
// per-workgroup totals (kTile = 256 records = 4 tiles) for the scan.
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
    const uint64_t tile = r / kEmitRecs;
    if ((threadIdx.x & 63) == 63) {
        if (tile * kEmitRecs < a.n) a.tile_sum[tile] = incl;
        s_wave[threadIdx.x >> 6] = incl;
    }
    if (r == 0) *a.defer_count = 0;   // enc_emit appends to the deferred-tile list
    __syncthreads();
    if (threadIdx.x == 0 && a.block_sum) a.block_sum[blockIdx.x] = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
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

constexpr int kHdrCap = 768;                  // header words staged per wave tile (3 KiB)
constexpr int kMapCap = 512;                  // 64-byte output granules mapped per wave tile (32 KiB)
constexpr uint16_t kNone16 = 0xFFFFu;

// Per-record LDS entry, read with two ds_read_b128.
struct RecEnt {
    uint64_t start;     // first output byte
    uint64_t pst;       // first payload byte (start + 4 * header words)
    uint64_t en;        // one past the last byte
    uint64_t srcbase;   // payload byte at output offset o lives at srcbase + o
};

// One wavefront's tile: kEmitRecs records, no workgroup barriers anywhere.
struct WaveTile {
    RecEnt ent[kEmitRecs + 1];       // [nrec] = sentinel {T1, T1, T1, 0}
    uint32_t meta[kEmitRecs];        // plan_record() meta (header words etc.)
    uint16_t hoff[kEmitRecs];        // staged header: word offset in hdr[], or kNone16
    uint32_t hdr[kHdrCap];           // header words of the tile's records (stream order)
    uint8_t map[kMapCap];            // granule g -> record holding byte 64*(G0+g) (or record 0)
};

// LDS writes of one lane become visible to the other lanes of the wave.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xC07F);      // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int find_ent(const RecEnt* ent, int nrec, uint64_t x) {
    int lo = 0, hi = nrec - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (ent[mid].start <= x) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ uint32_t hdr_word(const WaveTile& T, const EncArgs& a, const EncSrc& src, uint64_t r0,
                                             int r, uint32_t len, uint32_t k) {
    const uint16_t ho = T.hoff[r];
    if (ho != kNone16) return T.hdr[ho + k];
    return header_word_slow(a.msgs + r0 + r, len, T.meta[r], k, &src);
}

// Stream word k of tile record r; 0 outside [0, len).
__device__ __forceinline__ uint32_t tile_word(const WaveTile& T, const EncArgs& a, const EncSrc& src,
                                              uint64_t r0, int r, int64_t k) {
    const RecEnt& e = T.ent[r];
    const uint32_t len = uint32_t(e.en - e.start);
    if (k < 0 || 4 * k >= int64_t(len)) return 0u;
    const uint32_t hw = uint32_t((e.pst - e.start) >> 2);
    if (uint64_t(k) < hw) return hdr_word(T, a, src, r0, r, len, uint32_t(k));
    return load4_masked(e.srcbase + e.start + 4 * uint64_t(k), e.srcbase + e.en);
}

// Byte-granular: the 16 stream bytes of tile record r at output offsets
// [o, o+16) (bytes outside the record read as 0).
__device__ __forceinline__ void tile_chunk(const WaveTile& T, const EncArgs& a, const EncSrc& src, uint64_t r0,
                                           int r, uint64_t o, uint32_t out[4]) {
    const int64_t rel = int64_t(o) - int64_t(T.ent[r].start);
    const int64_t k0 = rel >> 2;                 // floor division
    const uint32_t sh = uint32_t(rel & 3);
    uint32_t w[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) w[i] = tile_word(T, a, src, r0, r, k0 + i);
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i] = funnel(w[i], w[i + 1], sh);
}

// Next record after r with bytes (skips zero-length records); nrec if none.
__device__ __forceinline__ int next_rec(const WaveTile& T, int nrec, int r) {
    ++r;
    while (r < nrec && T.ent[r].en == T.ent[r].start) ++r;
    return r;
}

// Byte-granular special chunk owned by r (tiles holding a record that does
// not start or end on a 4-byte boundary: unpadded odd-length payloads).
// Out of line: large, and rare in XDR traffic.
__device__ __noinline__ void byte_chunk(const WaveTile* Tp, const EncArgs* ap, const EncSrc* srcp, uint64_t r0,
                                        int nrec, int r, uint64_t o, uint32_t* v) {
    const WaveTile& T = *Tp;
    uint32_t w[4];
    tile_chunk(T, *ap, *srcp, r0, r, o, w);
    if (o + 16 > T.ent[r].en) {
        const int r2 = next_rec(T, nrec, r);
        if (r2 < nrec) {
            // bytes outside a record read as 0, so the parts OR together
            uint32_t b[4];
            tile_chunk(T, *ap, *srcp, r0, r2, o, b);
#pragma unroll
            for (int i = 0; i < 4; ++i) w[i] |= b[i];
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = w[i];
}

// Word-aligned special chunk owned by r (every record of the tile starts
// and ends on a 4-byte boundary and reads a 4-aligned payload): each output
// dword is one whole stream word of r or of the next record.
__device__ __forceinline__ void aligned_special(const WaveTile& T, const EncArgs& a, const EncSrc& src, uint64_t r0,
                                                int nrec, int r, const RecEnt& e, uint64_t o, uint32_t v[4]) {
    int rn = -1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint64_t p = o + 4 * i;
        uint32_t w = 0;
        if (p >= e.start && p < e.pst) {
            w = hdr_word(T, a, src, r0, r, uint32_t(e.en - e.start), uint32_t((p - e.start) >> 2));
        } else if (p >= e.pst && p < e.en) {
            w = gload<uint32_t>(e.srcbase + p);
        } else if (p >= e.en) {
            // first words of the next record (always header: >= 24 B)
            if (rn < 0) rn = next_rec(T, nrec, r);
            if (rn < nrec) {
                const RecEnt& f = T.ent[rn];
                w = hdr_word(T, a, src, r0, rn, uint32_t(f.en - f.start), uint32_t((p - f.start) >> 2));
            }
        }
        v[i] = w;
    }
}

__device__ __forceinline__ void store_chunk(uint8_t* out, uint64_t o, uint64_t lo, uint64_t hi, const uint32_t v[4]) {
    if (lo == o && hi == o + 16) {
        *reinterpret_cast<uint4*>(out + o) = make_uint4(v[0], v[1], v[2], v[3]);
    } else {
        // Tile-boundary or capacity-boundary chunk: only this tile's bytes.
        for (uint64_t bpos = lo; bpos < hi; ++bpos) {
            const uint32_t j = uint32_t(bpos - o);
            out[bpos] = uint8_t(v[j >> 2] >> (8 * (j & 3)));
        }
    }
}

// enc_fixup: the tiles enc_emit deferred (a record that is not 4-byte
// aligned — unpadded odd-length payloads — or headers beyond the fast
// kernel's LDS budget). One wavefront per tile, single chunk pass: every
// chunk (payload-only or special) is computed by its lane and all chunks of
// a step are stored by one global_store_dwordx4, so 128-byte lines are
// always written whole.
__global__ __launch_bounds__(kTile) void enc_fixup_kernel(EncArgs a) {
    __shared__ WaveTile s_tiles[kTile / 64];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    WaveTile& T = s_tiles[wv];
    const uint32_t ndef = *a.defer_count;
    const uint64_t nwaves = uint64_t(gridDim.x) * (kTile / 64);
    const EncSrc src{a.unix, reinterpret_cast<uintptr_t>(a.auth_arena),
                     reinterpret_cast<uintptr_t>(a.payload_arena)};
    for (uint64_t i = uint64_t(blockIdx.x) * (kTile / 64) + wv; i < ndef; i += nwaves) {
        const uint64_t tile = a.defer_list[i];
        const uint64_t r0 = tile * kEmitRecs;
        const int nrec = int(min(uint64_t(kEmitRecs), a.n - r0));
        const uint64_t tile_base = a.tile_base[tile];
        wave_lds_sync();   // the previous tile's readers are done with T

        uint64_t len = 0, srcbase = 0;
        uint32_t hw = 0;
        bool word_aligned = true;
        uint64_t start, en, pst;
        {
            onc_msg d;
            uint32_t meta = 0;
            if (lane < nrec) {
                d = a.msgs[r0 + lane];
                const RecPlan p = plan_record(d, a.unix);
                len = p.len;
                meta = p.meta;
                hw = len ? meta_hw(meta) : 0;
                word_aligned = (len & 3) == 0 && (len == 4ull * hw || ((src.payload_arena + d.payload_off) & 3) == 0);
            }
            const uint64_t v = (len << 16) | hw;
            const uint64_t incl = wave_incl_scan_u64(v);
            const uint64_t excl = incl - v;
            start = tile_base + (excl >> 16);
            en = start + len;
            pst = start + 4ull * hw;
            const uint32_t hoff = uint32_t(excl & 0xFFFFu);
            if (lane < nrec) {
                srcbase = src.payload_arena + d.payload_off - pst;
                T.ent[lane] = RecEnt{start, pst, en, srcbase};
                T.meta[lane] = meta;
                const bool staged = hoff + hw <= uint32_t(kHdrCap);
                T.hoff[lane] = staged ? uint16_t(hoff) : kNone16;
                if (len != 0 && staged) put_header_words(d, uint32_t(len), src, &T.hdr[hoff]);
            }
        }
        const uint64_t T0 = tile_base;
        const uint64_t T1 = __shfl(en, nrec - 1, 64);
        const uint64_t G0 = T0 >> 6;
        if (lane < nrec && len != 0) {
            const uint64_t g_hi = min((en - 1) >> 6, G0 + kMapCap - 1);
            for (uint64_t g = (start + 63) >> 6; g <= g_hi; ++g) T.map[g - G0] = uint8_t(lane);
        }
        if (lane == 0) {
            T.ent[nrec] = RecEnt{T1, T1, T1, 0};
            if (T0 & 63) T.map[0] = 0;
        }
        const bool tile_aligned = __all(word_aligned) && (T0 & 3) == 0;
        wave_lds_sync();

        const uint64_t E = min(T1, a.out_cap);
        if (E <= T0) continue;
        for (uint64_t c = (T0 >> 4) + lane; c < (E + 15) >> 4; c += 64) {
            const uint64_t o = c << 4;
            const uint64_t lo = max(o, T0);
            const uint64_t g = (lo >> 6) - G0;
            int r = g < uint64_t(kMapCap) ? int(T.map[g]) : find_ent(T.ent, nrec, lo);
            RecEnt e = T.ent[r];
            while (lo >= e.en && r + 1 < nrec) e = T.ent[++r];
            uint32_t v[4];
            if (o >= e.pst && o + 16 <= e.en) load16_unaligned(e.srcbase + o, v);
            else if (tile_aligned) aligned_special(T, a, src, r0, nrec, r, e, o, v);
            else byte_chunk(&T, &a, &src, r0, nrec, r, o, v);
            store_chunk(a.out, o, lo, min(o + 16, E), v);
        }
    }
}

// ---------------------------------------------------------------------------
// enc_emit: the hot kernel.
// ---------------------------------------------------------------------------
constexpr int kFastHdrCap = 1024;             // header words per wave tile (4 KiB of LDS)
constexpr int kFastMapCap = 1024;             // output granules per wave tile

// Per-record LDS entry of the fast kernel (two ds_read_b128).
struct FastEnt {
    uint64_t pst;       // first payload byte
    uint64_t en;        // one past the last byte
    uint64_t srcbase;   // payload byte at output offset o lives at srcbase + o
    int32_t dw;         // LDS header word of the output dword at p: ((p - T0) >> 2) + dw
    int32_t dwn;        // the same for the next record
};

struct FastTile {
    FastEnt ent[kEmitRecs + 1];      // [nrec] = sentinel {T1, T1, 0, 0, 0}
    uint32_t hdr[kFastHdrCap];       // header words of the tile's records (stream order)
    uint8_t map[kFastMapCap];        // granule -> record holding its first in-tile byte
};

// enc_emit: every wavefront owns one tile of kEmitRecs = 64 records and
// never waits for another wave (no workgroup barrier), so the staging of one
// wave overlaps the streaming of the others on the same CU.
//  Staging (lane per record): plan_record() again (the same function as
//  enc_len, so lengths agree); one wavefront __shfl scan places output
//  bytes and LDS header words; each record writes its LDS entry, serialises
//  its header words into LDS, and claims its output granules in the
//  granule map (granule = 64 B, doubled until the tile fits the map).
//  Tiles whose records are not all 4-byte aligned, or whose headers exceed
//  the LDS budget, are appended to the deferred list for enc_fixup.
//  Chunk pass (lane per 16-byte output chunk, 1 KiB contiguous per wave):
//  granule map -> record entry; a chunk inside its record's payload is one
//  unaligned 16-byte load; any other chunk takes each of its four dwords
//  from the LDS header image (this record's or the next one's header) or
//  the payload. Every chunk of a step, payload-only or not, is stored by the
//  same global_store_dwordx4, so 128-byte lines are always written whole
//  (a line left partially written costs a read-modify-write at eviction).
//  Chunks straddling a tile boundary are written with byte stores of only
//  this tile's bytes, so tiles never exchange data.
// kLab != 0 only in tools/emit_lab.hip.
template <int kLab>
__global__ __launch_bounds__(kTile) void enc_emit_kernel_t(EncArgs a) {
    __shared__ FastTile s_tiles[kTile / 64];

    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const uint64_t tile = uint64_t(blockIdx.x) * (kTile / 64) + wv;
    const uint64_t r0 = tile * kEmitRecs;
    if (r0 >= a.n) return;
    // tile base = workgroup base (scan of enc_len's workgroup totals) + the
    // totals of the tiles before this one in the workgroup
    uint64_t T0 = a.block_base[blockIdx.x];
    for (int w = 0; w < wv; ++w) T0 += a.tile_sum[uint64_t(blockIdx.x) * (kTile / 64) + w];
    if (lane == 0) a.tile_base[tile] = T0;            // read by enc_fixup
    FastTile& T = s_tiles[wv];
    const int nrec = int(min(uint64_t(kEmitRecs), a.n - r0));
    const uintptr_t payload = reinterpret_cast<uintptr_t>(a.payload_arena);

    onc_msg d;
    uint64_t len = 0;
    uint32_t meta = 0, hw = 0;
    bool word_aligned = true;
    if (lane < nrec) {
        d = a.msgs[r0 + lane];
        const RecPlan p = plan_record(d, a.unix);
        len = p.len;
        meta = p.meta;
        hw = len ? meta_hw(meta) : 0;
        word_aligned = (len & 3) == 0 && (len == 4ull * hw || ((payload + d.payload_off) & 3) == 0);
    }
    // One wave scan places output bytes and LDS header words: (len << 16 | hw).
    const uint64_t sv = (len << 16) | hw;
    const uint64_t incl = wave_incl_scan_u64(sv);
    const uint64_t excl = incl - sv;
    const uint64_t start = T0 + (excl >> 16);
    const uint64_t en = start + len;
    const uint64_t pst = start + 4ull * hw;
    const uint32_t hoff = uint32_t(excl & 0xFFFFu);
    const uint64_t last = __shfl(incl, nrec - 1, 64);
    const uint64_t T1 = T0 + (last >> 16);
    if (lane < nrec) {
        a.rec_off[r0 + lane] = start;
        if (len != 0 && en > a.out_cap) a.status[r0 + lane] = ONC_ENC_WRITE_ZERO;
    }
    const bool fast = __all(word_aligned) && (T0 & 3) == 0 && (last & 0xFFFFu) <= uint64_t(kFastHdrCap);
    if (!fast) {
        if (lane == 0) a.defer_list[atomicAdd(a.defer_count, 1u)] = uint32_t(tile);
        return;
    }
    const int32_t dw = int32_t(hoff) - int32_t((start - T0) >> 2);
    const int32_t dwn_raw = __shfl_down(dw, 1, 64);
    if (lane < nrec) {
        const uint64_t srcbase = payload + d.payload_off - pst;
        T.ent[lane] = FastEnt{pst, en, srcbase, dw, lane + 1 < nrec ? dwn_raw : dw};
        if (len != 0) {
            const EncSrc src{a.unix, reinterpret_cast<uintptr_t>(a.auth_arena), payload};
            put_header_words(d, uint32_t(len), src, &T.hdr[hoff]);
        }
    }
    // granule size: 64 B, doubled until the tile's bytes fit the map
    uint32_t gs = 6;
    while (((T1 - T0) >> gs) >= uint64_t(kFastMapCap)) ++gs;
    const uint64_t G0 = T0 >> gs;
    if (lane < nrec && len != 0) {
        // claim the granules whose first byte lies in this record
        const uint64_t gsz = 1ull << gs;
        for (uint64_t g = (start + gsz - 1) >> gs; g <= (en - 1) >> gs; ++g) T.map[g - G0] = uint8_t(lane);
    }
    if (lane == 0) {
        T.ent[nrec] = FastEnt{T1, T1, 0, 0, 0};
        if (T0 & ((1ull << gs) - 1)) T.map[0] = 0;   // granule 0 starts before the tile
    }
    wave_lds_sync();

    const uint64_t E = min(T1, a.out_cap);
    const uintptr_t dummy = reinterpret_cast<uintptr_t>(a.msgs);   // >= 64 valid bytes
    for (uint64_t c = (T0 >> 4) + lane; c < (E + 15) >> 4; c += 64) {
        const uint64_t o = c << 4;
        const uint64_t lo = max(o, T0);
        int r = T.map[(lo >> gs) - G0];
        FastEnt e = T.ent[r];
        while (lo >= e.en) e = T.ent[++r];            // sentinel en = T1 > lo
        uint32_t v[4];
        if (o >= e.pst && o + 16 <= e.en) {
            load16_unaligned(e.srcbase + o, v);
        } else {
            const int64_t q = (int64_t(o) - int64_t(T0)) >> 2;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint64_t p = o + 4 * i;
                const bool in_pay = p >= e.pst && p < e.en;
                const int64_t hidx = q + i + (p >= e.en ? e.dwn : e.dw);
                const int64_t hcl = hidx < 0 ? 0 : (hidx >= kFastHdrCap ? kFastHdrCap - 1 : hidx);
                const uint32_t h = T.hdr[hcl];
                const uint32_t w = gload<uint32_t>(in_pay ? e.srcbase + p : dummy);
                v[i] = in_pay ? w : h;
            }
        }
        store_chunk(a.out, o, lo, min(o + 16, E), v);
    }
}

hipError_t launch_enc_len(const EncArgs& a, hipStream_t s) {
    const uint64_t tiles = num_tiles(a.n);
    hipLaunchKernelGGL(enc_len_kernel, dim3(uint32_t(tiles)), dim3(kTile), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_enc_emit(const EncArgs& a, hipStream_t s) {
    const uint64_t blocks = (num_emit_tiles(a.n) + kTile / 64 - 1) / (kTile / 64);
    hipLaunchKernelGGL(enc_emit_kernel_t<0>, dim3(uint32_t(blocks)), dim3(kTile), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_enc_fixup(const EncArgs& a, hipStream_t s) {
    uint64_t blocks = (num_emit_tiles(a.n) + kTile / 64 - 1) / (kTile / 64);
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(enc_fixup_kernel, dim3(uint32_t(blocks)), dim3(kTile), 0, s, a);
    return hipGetLastError();
}

}  // namespace onc
