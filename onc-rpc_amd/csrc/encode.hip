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
//              records; the tile's non-pure 16-byte chunks (those holding
//              header bytes) are assembled in an LDS image; the output is
//              streamed chunk by chunk, 1 KiB contiguous per wave per step
//              (global_store_dwordx4): one 16-byte payload load (clamped into
//              the payload, dword-rotated) + one ds_read_b128 per chunk.
//              Handles tiles whose records are all 4-byte aligned; flags the
//              others.
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
// one wavefront scan (lane 63 writes the total); a workgroup of kLenRecs =
// 1024 lanes (16 waves, one record each) writes its total for the scan.
__global__ __launch_bounds__(kLenRecs) void enc_len_kernel(EncArgs a) {
    __shared__ uint64_t s_wave[kLenRecs / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t r = uint64_t(blockIdx.x) * kLenRecs + threadIdx.x;
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
    if (lane == 63) {
        if (tile * kEmitRecs < a.n) a.tile_sum[tile] = incl;
        s_wave[wv] = incl;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint64_t v = threadIdx.x < kLenRecs / 64 ? s_wave[threadIdx.x] : 0;
        const uint64_t t = wave_incl_scan_u64(v);
        if (threadIdx.x == 63) a.block_sum[blockIdx.x] = t;
    }
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
// (scan of the workgroup totals) + totals of the tiles before it there
// (lane i loads tile i of the workgroup; one wave reduction). Wave-uniform.
__device__ __forceinline__ uint64_t tile_start(const EncArgs& a, uint64_t tile) {
    const int lane = threadIdx.x & 63;
    const uint64_t blk = tile / (kLenRecs / kEmitRecs);
    const uint64_t t0 = blk * (kLenRecs / kEmitRecs);
    const uint64_t v = t0 + lane < tile ? a.tile_sum[t0 + lane] : 0;
    const uint64_t base = a.block_base[blk];
    return base + __shfl(wave_incl_scan_u64(v), 63, 64);
}

constexpr int kFastMapCap = 1024;             // output granules per wave tile (enc_fixup)
constexpr int kFastWaves = 4;                 // wave tiles per enc_emit workgroup

// ---------------------------------------------------------------------------
// enc_emit (chunk image): word-aligned tiles, every load of a step in flight.
// ---------------------------------------------------------------------------
// The span's output is cut into 16-byte chunks. A chunk wholly inside one
// record's payload is "pure". Every other chunk holds header bytes; its
// header bytes are assembled in LDS while the wave stages the span, in an
// image that is the span's output with the pure chunks cut out: chunk c of
// record r sits at slot c - NP_r before r's pure run and c - NP_r - np_r
// after it (np_r = r's pure chunks, NP_r = the sum over the records before
// r). The stream loop then does, per chunk, one 16-byte payload load and
// one ds_read_b128 of its image slot, and takes each dword from one or the
// other. The payload load of a chunk that is only partly payload is clamped
// into the payload ([pst, en - 16]) and its dwords rotated into place, so
// nothing outside the payload is read and the staging does no payload loads
// (records with 0 < payload < 16 bytes put their payload in the image).
// No branch separates one chunk's load from the next, so kU chunks per lane
// (kU KiB per wave) are in flight at once.
constexpr int kImgChunks = 248;               // image capacity per span (3968 B: 6 workgroups per CU)
constexpr int kMap2Cap = 512;                 // granules per span (granule = 4 chunks, doubled to fit)
constexpr int kEmitChunkUnroll = 2;           // chunks per lane per step (2 + nontemporal stores: -5 % vs 1)
constexpr int kEmitNT = 2;                    // nontemporal output stores (loads: measured slower)
constexpr uint64_t kFastTileMax = 1ull << 30; // larger tiles go to enc_fixup (int32 offsets here)
// a record's own non-pure chunks: header <= 4 * (7 + 2 * 52) bytes, + the
// chunk it shares with its predecessor, + its tail chunk
static_assert((4 * (7 + 2 * 52) + 15) / 16 + 2 <= kImgChunks / 8, "a span of 8 maximal records must fit");

struct ImgTile {
    uint4 img[kImgChunks];           // assembled non-pure chunks (header bytes; small payloads)
    int4 ent[kEmitRecs + 1];         // {cf, cp0, cp1, NP} (chunks, span-relative); [ns].x = sentinel
    int4 pay[kEmitRecs + 1];         // {pst, en (bytes, span-chunk-relative; pst = en: no stream payload), src lo, hi}
    uint8_t map[kMap2Cap];           // granule -> span record owning its first chunk
};

__device__ __forceinline__ uint32_t sel4(const u32x4_a4& x, uint32_t i) {
    return i == 0 ? x.x : (i == 1 ? x.y : (i == 2 ? x.z : x.w));
}

template <int kU, int kNT>
__device__ __forceinline__ void enc_emit_tile(const EncArgs& a, ImgTile& T, uint64_t tile) {
    const int lane = threadIdx.x & 63;
    const uint64_t r0 = tile * kEmitRecs;
    uint32_t* img32 = reinterpret_cast<uint32_t*>(T.img);
    const int nrec = int(min(uint64_t(kEmitRecs), a.n - r0));
    const uintptr_t payload = reinterpret_cast<uintptr_t>(a.payload_arena);

    const uint64_t T0 = tile_start(a, tile);
    uint64_t len = 0, poff = 0;
    uint32_t hw = 0;
    bool word_aligned = true;
    if (lane < nrec) {
        const onc_msg d = a.msgs[r0 + lane];
        const RecPlan p = plan_record(d, a.unix);   // the same function as enc_len: lengths agree
        len = p.len;
        hw = len ? meta_hw(p.meta) : 0;
        poff = d.payload_off;
        word_aligned = (len & 3) == 0 && (len == 4ull * hw || ((payload + d.payload_off) & 3) == 0);
    }
    const uint64_t incl = wave_incl_scan_u64(len);
    const uint64_t agg = __shfl(incl, 63, 64);
    const uint64_t start = T0 + incl - len;
    const uint64_t en = start + len;
    const uint64_t pst = start + 4ull * hw;
    if (lane < nrec) {
        a.rec_off[r0 + lane] = start;
        if (len != 0 && en > a.out_cap) a.status[r0 + lane] = ONC_ENC_WRITE_ZERO;
    }
    const bool fast = __all(word_aligned) && (T0 & 3) == 0 && agg < kFastTileMax;
    if (lane == 0) {
        a.tile_base[tile] = T0 | (fast ? 0 : kDeferBit);
        if (!fast) {
            const uint64_t slot =
                __hip_atomic_fetch_add(a.ctl + (a.gen & 1), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            a.fix_list[slot] = uint32_t(tile);
        }
        // the next launch's list counter (its enc_fixup has run before this launch)
        if (tile == 0) __hip_atomic_store(a.ctl + ((a.gen + 1) & 1), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!fast) return;

    // Absolute chunk indices: owned chunks [cfa, own_next), pure [p0, p1).
    const int64_t cfa = int64_t((start + 15) >> 4);
    const int64_t p0 = int64_t((pst + 15) >> 4);
    const int64_t p1 = max(p0, int64_t(en >> 4));
    const int64_t np = len ? p1 - p0 : 0;
    const int64_t cfa_next = __shfl_down(cfa, 1, 64);
    const int64_t cfa_end = int64_t((__shfl(en, nrec - 1, 64) + 15) >> 4);
    const int64_t own_next = lane + 1 < nrec ? cfa_next : cfa_end;
    const uint32_t nonpure = lane < nrec && len ? uint32_t(own_next - cfa - np) : 0u;
    const uint64_t wnp = wave_incl_scan_u64(nonpure);
    const uint64_t plen = en - pst;

    const uintptr_t dummy = reinterpret_cast<uintptr_t>(a.msgs);   // >= 64 valid bytes
    int lo_rec = 0;
    while (lo_rec < nrec) {
        // span: records [lo_rec, hi_rec) whose non-pure chunks (+1 for a
        // chunk shared with the record before) fit the image
        const uint64_t wbase = lo_rec ? __shfl(wnp, lo_rec - 1, 64) : 0;
        const uint64_t over = __ballot(lane >= lo_rec && lane < nrec && wnp - wbase + 1 > uint64_t(kImgChunks));
        const int hi_rec = over ? min(nrec, int(__builtin_ctzll(over))) : nrec;
        const int ns = hi_rec - lo_rec;
        const uint64_t S0 = __shfl(start, lo_rec, 64);
        const uint64_t S1 = __shfl(en, hi_rec - 1, 64);
        const int64_t C0 = int64_t(S0 >> 4);
        const uint64_t B0 = uint64_t(C0) << 4;        // byte origin of the span-relative offsets
        if (lo_rec) wave_lds_sync();                   // the previous span's readers are done
        const bool active = lane >= lo_rec && lane < hi_rec;
        const int j = lane - lo_rec;
        const int64_t npx = active ? np : 0;
        const int64_t NP = int64_t(wave_incl_scan_u64(uint64_t(npx))) - npx;   // lanes < lo_rec add 0
        const int32_t NC = int32_t(((S1 + 15) >> 4) - C0);
        uint32_t gsh = 2;                              // granule = 4 chunks, doubled until the span fits
        while ((NC >> gsh) >= kMap2Cap) ++gsh;
        const uint64_t nonempty = __ballot(active && len != 0);
        if (active) {
            const bool small = plen != 0 && plen < 16;    // payload kept in the image
            const uintptr_t sb = payload + poff - pst;    // payload byte at output offset o: sb + o
            T.ent[j] = make_int4(int32_t(cfa - C0), int32_t(p0 - C0), int32_t(p1 - C0), int32_t(NP));
            const int32_t ps = int32_t(pst - B0), pe = int32_t(en - B0);
            T.pay[j] = make_int4(small ? pe : ps, pe, int32_t(uint32_t(sb)), int32_t(uint32_t(sb >> 32)));
            if (len != 0) {
                // header words: image dword of output dword P is P - 4 (C0 + NP)
                const int64_t ib = int64_t(start >> 2) - 4 * (C0 + NP);
                const onc_msg d = a.msgs[r0 + lane];
                const EncSrc src{a.unix, reinterpret_cast<uintptr_t>(a.auth_arena), payload};
                put_header_words(d, uint32_t(len), src, &img32[ib]);
                if (small) {
                    // all of it lies in non-pure chunks (np = 0): right after the header
                    for (uint32_t k = 0; 4 * k < plen; ++k) img32[ib + hw + k] = gload<uint32_t>(sb + pst + 4 * k);
                }
                // granules whose first chunk this record owns (chunk 0 of a
                // span not starting on a chunk: its first non-empty record)
                const int32_t own_lo = (S0 & 15) && lane == __builtin_ctzll(nonempty) ? 0 : int32_t(cfa - C0);
                const int32_t own_hi = int32_t(own_next - C0);    // <= NC
                const int32_t g_hi = min((own_hi + (1 << gsh) - 1) >> gsh, kMap2Cap);
                for (int32_t g = (own_lo + (1 << gsh) - 1) >> gsh; g < g_hi; ++g) T.map[g] = uint8_t(j);
            }
        }
        if (lane == 0) T.ent[ns] = make_int4(0x7FFFFFFF, 0, 0, 0);
        wave_lds_sync();

        const uint64_t E = min(S1, a.out_cap);
        lo_rec = hi_rec;
        if (E <= S0) continue;                         // no bytes (all records failed, or beyond out_cap)
        const int32_t NCe = int32_t(((E + 15) >> 4) - C0);
        for (int32_t step = 0; step < NCe; step += 64 * kU) {
            uintptr_t A[kU];
            int32_t slot[kU];
            uint32_t sel[kU];      // bits 0-3: dword i is payload; bits 4-5: rotation
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int32_t c = min(step + lane + 64 * u, NCe - 1);
                int r = T.map[c >> gsh];
                while (c >= T.ent[r + 1].x) ++r;
                const int4 m = T.ent[r];
                const int4 q = T.pay[r];
                const int32_t s = c - m.w - (c >= m.z ? m.z - m.y : 0);
                slot[u] = s < 0 ? 0 : (s >= kImgChunks ? kImgChunks - 1 : s);
                const int32_t o = c << 4;
                const bool hasp = q.x < q.y && o < q.y && o + 16 > q.x;
                const int32_t x = max(q.x, min(o, q.y - 16));          // clamped window start
                const uint64_t sbase = uint64_t(uint32_t(q.z)) | (uint64_t(uint32_t(q.w)) << 32);
                A[u] = hasp ? sbase + B0 + uint64_t(int64_t(x)) : dummy;
                uint32_t pm = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) pm |= (o + 4 * i >= q.x && o + 4 * i < q.y) ? (1u << i) : 0u;
                sel[u] = (hasp ? pm : 0u) | (uint32_t((o - x) >> 2) & 3u) << 4;
            }
            u32x4_a4 X[kU];
            uint4 L[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                if (kNT & 1) X[u] = __builtin_nontemporal_load(reinterpret_cast<const ONC_GLOBAL u32x4_a4*>(A[u]));
                else X[u] = gload<u32x4_a4>(A[u]);
                L[u] = T.img[slot[u]];
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int32_t c = step + lane + 64 * u;
                if (c >= NCe) break;
                const uint32_t rot = sel[u] >> 4;
                const uint32_t h[4] = {L[u].x, L[u].y, L[u].z, L[u].w};
                uint32_t v[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = (sel[u] >> i) & 1 ? sel4(X[u], (i + rot) & 3) : h[i];
                const uint64_t o = B0 + (uint64_t(c) << 4);
                if ((kNT & 2) && o >= S0 && o + 16 <= E)
                    __builtin_nontemporal_store(u32x4{v[0], v[1], v[2], v[3]}, reinterpret_cast<u32x4*>(a.out + o));
                else
                    store_chunk(a.out, o, max(o, S0), min(o + 16, E), v);
            }
        }
    }
}

// kNT: bit 0 = nontemporal payload loads, bit 1 = nontemporal stores;
// kOcc: workgroups per CU the register allocation must allow (0 = free)
template <int kU, int kNT = 0, int kOcc = 0>
__global__ __launch_bounds__(64 * kFastWaves, kOcc ? kOcc * kFastWaves / 4 : 1) void enc_emit_kernel_t(EncArgs a) {
    __shared__ ImgTile s_tiles[kFastWaves];
    const uint64_t tile = uint64_t(blockIdx.x) * kFastWaves + (threadIdx.x >> 6);
    if (tile < num_emit_tiles(a.n)) enc_emit_tile<kU, kNT>(a, s_tiles[threadIdx.x >> 6], tile);
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
__device__ __forceinline__ void enc_fixup_tile(const EncArgs& a, GenTile& T, uint64_t tile) {
    const int lane = threadIdx.x;
    const uint64_t tb = a.tile_base[tile];
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
    hipLaunchKernelGGL(enc_len_kernel, dim3(uint32_t(num_len_blocks(a.n))), dim3(kLenRecs), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_enc_emit(const EncArgs& a, hipStream_t s) {
    const uint64_t blocks = (num_emit_tiles(a.n) + kFastWaves - 1) / kFastWaves;
    hipLaunchKernelGGL((enc_emit_kernel_t<kEmitChunkUnroll, kEmitNT>), dim3(uint32_t(blocks)), dim3(64 * kFastWaves), 0, s, a);
    return hipGetLastError();
}

constexpr uint32_t kFixupBlocks = 1024;      // persistent: workgroups stride over the flagged tiles

// enc_fixup: one wavefront (= workgroup) per flagged tile, striding over the
// list enc_emit built (counter ctl[gen & 1]; enc_emit clears the other one
// for the next launch).
__global__ __launch_bounds__(64) void enc_fixup_kernel(EncArgs a) {
    __shared__ GenTile T;
    const uint64_t count = __hip_atomic_load(a.ctl + (a.gen & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint64_t i = blockIdx.x; i < count; i += gridDim.x) {
        if (i != blockIdx.x) wave_lds_sync();       // the previous tile's readers are done
        enc_fixup_tile(a, T, a.fix_list[i]);
    }
}

hipError_t launch_enc_fixup(const EncArgs& a, hipStream_t s) {
    const uint32_t blocks = uint32_t(min(uint64_t(kFixupBlocks), num_emit_tiles(a.n)));
    hipLaunchKernelGGL(enc_fixup_kernel, dim3(blocks), dim3(64), 0, s, a);
    return hipGetLastError();
}


}  // namespace onc
