// encode.hip — batch RpcMessage::serialise_into for gfx950.
//
// Reference: RpcMessage::serialise_into (src/rpc_message.rs:136-164) and the
// serialise_into/serialised_len chain it calls (call_body.rs:98-119,
// auth/flavor.rs:106-174, auth/unix_params.rs:162-245, opaque.rs:38-63,
// reply/*). The reference is called once per message by the user's loop;
// here one pass encodes a whole batch into one contiguous send buffer.
//
// Pipeline (4 launches on one stream):
//   enc_len    lane per record: plan_record() = serialised_len + validation;
//              per-64-record-tile and per-256-record-workgroup byte totals.
//   scan       single-workgroup exclusive scan of the workgroup totals.
//   enc_emit   wave per 64-record tile: wavefront __shfl scan places the
//              records; headers staged in LDS; the tile's output bytes are
//              produced in 16-byte chunks, 1 KiB contiguous per wave per step
//              (global_store_dwordx4). Handles tiles whose records are all
//              4-byte aligned (every output dword is wholly header or wholly
//              payload) and whose headers fit LDS; flags the others.
//   enc_fixup  wave per flagged tile (exits at once for the others): the
//              byte-general path — header image pre-shifted to each
//              record's output alignment, payload bytes via clamped dword
//              loads + v_alignbyte, records in sub-tiles when the headers
//              exceed LDS.
#include "common.h"
#include "kernels.h"

namespace onc {

constexpr uint64_t kDeferBit = 1ull << 63;   // tile_base flag: tile left to enc_fixup

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
    __syncthreads();
    if (threadIdx.x == 0) a.block_sum[blockIdx.x] = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
}

// LDS writes of one lane become visible to the other lanes of the wave.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xC07F);      // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Output bytes [lo, hi) of the 16-byte chunk at o (lo >= o, hi <= o + 16).
__device__ __forceinline__ void store_chunk(uint8_t* out, uint64_t o, uint64_t lo, uint64_t hi, const uint32_t v[4]) {
    if (lo == o && hi == o + 16) {
        *reinterpret_cast<uint4*>(out + o) = make_uint4(v[0], v[1], v[2], v[3]);
    } else {
        // Tile/span-boundary or capacity-boundary chunk: only this span's bytes.
        for (uint64_t bpos = lo; bpos < hi; ++bpos) {
            const uint32_t j = uint32_t(bpos - o);
            out[bpos] = uint8_t(v[j >> 2] >> (8 * (j & 3)));
        }
    }
}

// Byte offset of tile `tile` in the output: base of its enc_len workgroup
// (scan of the workgroup totals) + totals of the tiles before it there.
__device__ __forceinline__ uint64_t tile_start(const EncArgs& a, uint64_t tile) {
    const uint64_t blk = tile / (kTile / kEmitRecs);
    uint64_t T0 = a.block_base[blk];
    for (uint64_t t = blk * (kTile / kEmitRecs); t < tile; ++t) T0 += a.tile_sum[t];
    return T0;
}

// ---------------------------------------------------------------------------
// enc_emit: the hot kernel (word-aligned tiles).
// ---------------------------------------------------------------------------
constexpr int kFastHdrCap = 1024;             // header words per span (4 KiB of LDS)
static_assert(8 * (7 + 2 * 52) <= kFastHdrCap, "a span of 8 maximal headers must fit LDS");
constexpr int kFastMapCap = 1024;             // output granules per wave tile
constexpr int kFastWaves = 4;                 // wave tiles per workgroup
constexpr int kEmitUnroll = 1;                // output chunks per lane per step

// Per-record LDS entry of enc_emit (two ds_read_b128).
struct FastEnt {
    uint64_t pst;       // first payload byte
    uint64_t en;        // one past the last byte
    uint64_t srcbase;   // payload byte at output offset o lives at srcbase + o
    int32_t dw;         // LDS header word of the output dword at p: ((p - T0) >> 2) + dw
    int32_t dwn;        // the same for the next record
};

struct FastTile {
    FastEnt ent[kEmitRecs + 1];      // [span records] = sentinel {S1, S1, 0, 0, 0}
    uint32_t hdr[kFastHdrCap];       // header words of the span's records (stream order)
    uint8_t map[kFastMapCap];        // granule -> span record holding its first byte
};

// enc_emit: every wavefront owns one tile of kEmitRecs = 64 records and
// never waits for another wave (no workgroup barrier), so the staging of one
// wave overlaps the streaming of the others on the same CU.
//  Staging (lane per record): plan_record() again (the same function as
//  enc_len, so lengths agree); one wavefront __shfl scan places output
//  bytes and LDS header words; each record writes its LDS entry, serialises
//  its header words into LDS, and claims its output granules in the
//  granule map (granule = 64 B, doubled until the tile fits the map).
//  Tiles whose records are not all 4-byte aligned (unpadded odd-length
//  payloads), or whose headers exceed the LDS budget, are flagged for
//  enc_fixup in tile_base.
//  Chunk pass (lane per 16-byte output chunk, 1 KiB contiguous per wave):
//  granule map -> record entry; a chunk inside its record's payload is one
//  unaligned 16-byte load; any other chunk takes each of its four dwords
//  from the LDS header image (this record's or the next one's header) or
//  the payload. Every chunk of a step, payload-only or not, is stored by the
//  same global_store_dwordx4, so 128-byte lines are always written whole
//  (a line left partially written costs a read-modify-write at eviction).
//  Chunks straddling a tile boundary are written with byte stores of only
//  this tile's bytes, so tiles never exchange data.
template <int kU>
__global__ __launch_bounds__(64 * kFastWaves) void enc_emit_kernel_t(EncArgs a) {
    __shared__ FastTile s_tiles[kFastWaves];

    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const uint64_t tile = uint64_t(blockIdx.x) * kFastWaves + wv;
    const uint64_t r0 = tile * kEmitRecs;
    if (r0 >= a.n) return;
    const uint64_t T0 = tile_start(a, tile);
    FastTile& T = s_tiles[wv];
    const int nrec = int(min(uint64_t(kEmitRecs), a.n - r0));
    const uintptr_t payload = reinterpret_cast<uintptr_t>(a.payload_arena);

    uint64_t len = 0, poff = 0;
    uint32_t hw = 0;
    bool word_aligned = true;
    if (lane < nrec) {
        const onc_msg d = a.msgs[r0 + lane];
        const RecPlan p = plan_record(d, a.unix);
        len = p.len;
        hw = len ? meta_hw(p.meta) : 0;
        poff = d.payload_off;
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
    const uint32_t hincl = uint32_t(incl & 0xFFFFu);
    if (lane < nrec) {
        a.rec_off[r0 + lane] = start;
        if (len != 0 && en > a.out_cap) a.status[r0 + lane] = ONC_ENC_WRITE_ZERO;
    }
    const bool fast = __all(word_aligned) && (T0 & 3) == 0;
    if (lane == 0) a.tile_base[tile] = T0 | (fast ? 0 : kDeferBit);
    if (!fast) return;

    // Spans: the tile's records in groups of S (64, 32, 16 or 8) whose header
    // words fit kFastHdrCap (8 records always fit: <= 111 words each).
    int S = kEmitRecs;
    for (; S > 8; S >>= 1) {
        const int g0 = lane & ~(S - 1);
        const int g1 = min(lane | (S - 1), nrec - 1);
        const uint32_t top = __shfl(hincl, g1, 64);
        const uint32_t bot = __shfl(hoff, g0, 64);
        if (!__any(g0 < nrec && top - bot > uint32_t(kFastHdrCap))) break;
    }
    const uintptr_t dummy = reinterpret_cast<uintptr_t>(a.msgs);   // >= 64 valid bytes
    for (int lo_rec = 0; lo_rec < nrec; lo_rec += S) {
        const int hi_rec = min(nrec, lo_rec + S);
        const int ns = hi_rec - lo_rec;
        const uint64_t S0 = __shfl(start, lo_rec, 64);
        const uint64_t S1 = __shfl(en, hi_rec - 1, 64);
        const uint32_t hb = __shfl(hoff, lo_rec, 64);
        if (lo_rec) wave_lds_sync();                   // the previous span's readers are done
        const bool active = lane >= lo_rec && lane < hi_rec;
        const int j = lane - lo_rec;
        const int32_t dw = int32_t(hoff - hb) - int32_t((start - S0) >> 2);
        const int32_t dwn_raw = __shfl_down(dw, 1, 64);
        if (active) {
            T.ent[j] = FastEnt{pst, en, payload + poff - pst, dw, lane + 1 < hi_rec ? dwn_raw : dw};
            if (len != 0) {
                // descriptor re-read (L2) rather than kept live across the spans
                const onc_msg d = a.msgs[r0 + lane];
                const EncSrc src{a.unix, reinterpret_cast<uintptr_t>(a.auth_arena), payload};
                put_header_words(d, uint32_t(len), src, &T.hdr[hoff - hb]);
            }
        }
        // granule size: 64 B, doubled until the span's bytes fit the map
        uint32_t gs = 6;
        while (((S1 - S0) >> gs) >= uint64_t(kFastMapCap)) ++gs;
        const uint64_t G0 = S0 >> gs;
        if (active && len != 0) {
            // claim the granules whose first byte lies in this record
            const uint64_t gsz = 1ull << gs;
            for (uint64_t g = (start + gsz - 1) >> gs; g <= (en - 1) >> gs; ++g) T.map[g - G0] = uint8_t(j);
        }
        if (lane == 0) {
            T.ent[ns] = FastEnt{S1, S1, 0, 0, 0};
            if (S0 & ((1ull << gs) - 1)) T.map[0] = 0;   // granule 0 starts before the span
        }
        wave_lds_sync();

        const uint64_t E = min(S1, a.out_cap);
        if (E <= S0) continue;                        // no bytes (all records failed, or beyond out_cap)
        // kU chunks per lane per step: their loads are all in flight before
        // the first store.
        const uint64_t cend = (E + 15) >> 4;
        for (uint64_t c = (S0 >> 4) + lane; c < cend; c += 64 * kU) {
            uint32_t v[kU][4];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const uint64_t o = (c + 64 * u) << 4;
                const uint64_t lo = max(o, S0);
                if (c + 64 * u >= cend) break;
                int r = T.map[(lo >> gs) - G0];
                FastEnt e = T.ent[r];
                while (lo >= e.en) e = T.ent[++r];        // sentinel en = S1 > lo
                if (o >= e.pst && o + 16 <= e.en) {
                    load16_unaligned(e.srcbase + o, v[u]);
                } else {
                    const int64_t q = (int64_t(o) - int64_t(S0)) >> 2;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const uint64_t p = o + 4 * i;
                        const bool in_pay = p >= e.pst && p < e.en;
                        const int64_t hidx = q + i + (p >= e.en ? e.dwn : e.dw);
                        const int64_t hcl = hidx < 0 ? 0 : (hidx >= kFastHdrCap ? kFastHdrCap - 1 : hidx);
                        const uint32_t h = T.hdr[hcl];
                        const uint32_t w = gload<uint32_t>(in_pay ? e.srcbase + p : dummy);
                        v[u][i] = in_pay ? w : h;
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const uint64_t o = (c + 64 * u) << 4;
                if (c + 64 * u >= cend) break;
                store_chunk(a.out, o, max(o, S0), min(o + 16, E), v[u]);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// enc_fixup: byte-general path for the tiles enc_emit flagged.
// ---------------------------------------------------------------------------
constexpr int kImgCap = 2048;                 // header image dwords per span (8 KiB of LDS)
constexpr int kSubRecs = 16;                  // records per span when a tile's image exceeds kImgCap
// a record's header is at most 7 + 2 * (2 + 50) words (Call with two 200-byte
// auth bodies), plus one image word for an unaligned start
static_assert(kSubRecs * (7 + 2 * 52 + 1) <= kImgCap, "a span of maximal headers must fit LDS");

// Per-record LDS entry of enc_fixup (two ds_read_b128).
struct GenEnt {
    uint64_t pst;       // first payload byte (output offset)
    uint64_t en;        // one past the last byte
    uint64_t srcbase;   // payload byte at output offset o lives at srcbase + o
    int32_t ib;         // image dword of output dword q: (q - (S0 >> 2)) + ib
    int32_t pad;
};

struct GenTile {
    GenEnt ent[kEmitRecs + 1];       // [span records] = sentinel {S1, S1, 0, 0}
    uint32_t img[kImgCap];           // header bytes at their output-dword positions, zero elsewhere
    uint8_t map[kFastMapCap];        // granule -> span record holding its first byte
};

// One span (records [lo_rec, hi_rec) of the tile, bytes [S0, S1)) of the
// general path. Per record: its header serialised into the LDS image already
// shifted to its output byte alignment (start & 3; bytes outside the header
// are zero), so an output dword's header bytes are one image word; payload
// bytes come from the five aligned source dwords under the chunk, each
// clamped into the dwords that hold this chunk's payload bytes (nothing
// outside the payload is touched), combined by v_alignbyte. An output dword
// is the OR of (this record's image word, the next record's image word,
// this record's masked payload bytes): a 16-byte chunk meets at most one
// payload, since every record has >= 24 header bytes.
__device__ __forceinline__ void gen_span(GenTile& T, const EncArgs& a, const onc_msg& d, int lane, int lo_rec,
                                         int hi_rec, uint64_t len, uint32_t hw, uint64_t start, uint64_t S0,
                                         uint64_t S1) {
    const uintptr_t payload = reinterpret_cast<uintptr_t>(a.payload_arena);
    const bool active = lane >= lo_rec && lane < hi_rec;
    const uint64_t en = start + len;
    const uint64_t pst = start + 4ull * hw;
    const uint32_t m = uint32_t(start & 3);
    const uint32_t iw = active && len ? hw + (m ? 1u : 0u) : 0u;
    const uint64_t iincl = wave_incl_scan_u64(iw);
    const uint32_t ibase = uint32_t(iincl - iw);
    const int j = lane - lo_rec;
    const int nspan = hi_rec - lo_rec;
    if (active) {
        const int32_t ib = int32_t(ibase) - int32_t((start >> 2) - (S0 >> 2));
        T.ent[j] = GenEnt{pst, en, payload + d.payload_off - pst, ib, 0};
        if (len != 0) {
            const EncSrc src{a.unix, reinterpret_cast<uintptr_t>(a.auth_arena), payload};
            if (m == 0) {
                WordSink w{&T.img[ibase]};
                put_header_words(d, uint32_t(len), src, w);
            } else {
                ShiftSink w{&T.img[ibase], 0u, 4u - m};
                put_header_words(d, uint32_t(len), src, w);
                w.finish();
            }
        }
    }
    uint32_t gs = 6;
    while (((S1 - S0) >> gs) >= uint64_t(kFastMapCap)) ++gs;
    const uint64_t G0 = S0 >> gs;
    if (active && len != 0) {
        const uint64_t gsz = 1ull << gs;
        for (uint64_t g = (start + gsz - 1) >> gs; g <= (en - 1) >> gs; ++g) T.map[g - G0] = uint8_t(j);
    }
    if (lane == 0) {
        T.ent[nspan] = GenEnt{S1, S1, 0, 0, 0};
        if (S0 & ((1ull << gs) - 1)) T.map[0] = 0;
    }
    wave_lds_sync();

    const uint64_t E = min(S1, a.out_cap);
    if (E <= S0) return;                              // no bytes (all records failed, or beyond out_cap)
    const int64_t q0 = int64_t(S0 >> 2);
    const uintptr_t dummy = reinterpret_cast<uintptr_t>(a.msgs);
    for (uint64_t c = (S0 >> 4) + lane; c < (E + 15) >> 4; c += 64) {
        const uint64_t o = c << 4;
        const uint64_t lo = max(o, S0);
        int r = T.map[(lo >> gs) - G0];
        GenEnt e = T.ent[r];
        while (lo >= e.en) e = T.ent[++r];            // sentinel en = S1 > lo
        const uint64_t b0 = max(o, e.pst), b1 = min(o + 16, e.en);
        const bool hp = b0 < b1;
        const bool whole = o >= e.pst && o + 16 <= e.en;
        const uintptr_t sb = e.srcbase + o;
        const uintptr_t base = sb & ~uintptr_t(3);
        const uint32_t sh = uint32_t(sb & 3);
        const uintptr_t first = hp ? ((e.srcbase + b0) & ~uintptr_t(3)) : dummy;
        const uintptr_t last = hp ? ((e.srcbase + b1 - 1) & ~uintptr_t(3)) : dummy;
        uint32_t w[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            uintptr_t ad = base + 4 * k;
            ad = ad < first ? first : (ad > last ? last : ad);
            w[k] = gload<uint32_t>(ad);
        }
        uint32_t v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = funnel(w[i], w[i + 1], sh);
        if (!whole) {
            const int32_t ibn = T.ent[r + 1].ib;
            const int64_t q = int64_t(o >> 2) - q0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint64_t p = o + 4 * i;
                const int64_t h0 = q + i + e.ib, h1 = q + i + ibn;
                const uint32_t x0 = T.img[h0 < 0 ? 0 : (h0 >= kImgCap ? kImgCap - 1 : h0)];
                const uint32_t x1 = T.img[h1 < 0 ? 0 : (h1 >= kImgCap ? kImgCap - 1 : h1)];
                // the next record's header (none past the span's last byte)
                const uint32_t hv = (p < e.pst ? x0 : 0u) | (p + 4 > e.en && e.en < S1 ? x1 : 0u);
                const int64_t l8 = int64_t(b0) - int64_t(p), h8 = int64_t(b1) - int64_t(p);
                const uint32_t l = uint32_t(l8 < 0 ? 0 : (l8 > 4 ? 4 : l8));
                const uint32_t h = uint32_t(h8 < 0 ? 0 : (h8 > 4 ? 4 : h8));
                const uint32_t pm = hp ? uint32_t(((1ull << (8 * h)) - 1ull) & ~((1ull << (8 * l)) - 1ull)) : 0u;
                v[i] = hv | (v[i] & pm);
            }
        }
        store_chunk(a.out, o, lo, min(o + 16, E), v);
    }
}

// enc_fixup: one wavefront (= workgroup) per tile; tiles enc_emit handled
// exit after reading their flag.
__global__ __launch_bounds__(64) void enc_fixup_kernel(EncArgs a) {
    __shared__ GenTile T;
    const int lane = threadIdx.x;
    const uint64_t tile = blockIdx.x;
    const uint64_t tb = a.tile_base[tile];
    if (!(tb & kDeferBit)) return;
    const uint64_t T0 = tb & ~kDeferBit;
    const uint64_t r0 = tile * kEmitRecs;
    const int nrec = int(min(uint64_t(kEmitRecs), a.n - r0));

    onc_msg d;
    uint64_t len = 0;
    uint32_t hw = 0;
    if (lane < nrec) {
        d = a.msgs[r0 + lane];
        const RecPlan p = plan_record(d, a.unix);
        len = p.len;
        hw = len ? meta_hw(p.meta) : 0;
    }
    const uint64_t incl = wave_incl_scan_u64(len);
    const uint64_t start = T0 + incl - len;
    // image words of the whole tile (upper bound: one extra per record)
    const uint64_t iall = wave_incl_scan_u64(len ? hw + 1 : 0);
    const bool split = __shfl(iall, nrec - 1, 64) > uint64_t(kImgCap);
    const int step = split ? kSubRecs : kEmitRecs;
    for (int lo_rec = 0; lo_rec < nrec; lo_rec += step) {
        const int hi_rec = min(nrec, lo_rec + step);
        const uint64_t S0 = __shfl(start, lo_rec, 64);
        const uint64_t S1 = __shfl(start + len, hi_rec - 1, 64);
        if (lo_rec) wave_lds_sync();                   // previous span's readers are done
        gen_span(T, a, d, lane, lo_rec, hi_rec, len, hw, start, S0, S1);
    }
}

hipError_t launch_enc_len(const EncArgs& a, hipStream_t s) {
    const uint64_t tiles = num_tiles(a.n);
    hipLaunchKernelGGL(enc_len_kernel, dim3(uint32_t(tiles)), dim3(kTile), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_enc_emit(const EncArgs& a, hipStream_t s) {
    const uint64_t blocks = (num_emit_tiles(a.n) + kFastWaves - 1) / kFastWaves;
    hipLaunchKernelGGL((enc_emit_kernel_t<kEmitUnroll>), dim3(uint32_t(blocks)), dim3(64 * kFastWaves), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_enc_fixup(const EncArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(enc_fixup_kernel, dim3(uint32_t(num_emit_tiles(a.n))), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace onc
