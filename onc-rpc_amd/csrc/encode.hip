// encode.hip — batch RpcMessage::serialise_into for gfx950.
//
// Reference: RpcMessage::serialise_into (src/rpc_message.rs:136-164) and the
// serialise_into/serialised_len chain it calls (call_body.rs:98-119,
// auth/flavor.rs:106-174, auth/unix_params.rs:162-245, opaque.rs:38-63,
// reply/*). The reference is called once per message by the user's loop;
// here one pass encodes a whole batch into one contiguous send buffer.
//
// Pipeline (3 launches on one stream):
//   enc_len    lane per record: plan_record() = serialised_len + validation;
//              per-64-record-tile and per-1024-record-workgroup byte totals.
//   scan       single-workgroup exclusive scan of the workgroup totals.
//   enc_emit   wave per 64-record tile: wavefront __shfl scan places the
//              records; the tile's non-pure 16-byte chunks (those holding
//              header bytes) are assembled in an LDS image; the output is
//              streamed chunk by chunk, 2 KiB contiguous per wave per step
//              (global_store_dwordx4, nontemporal): one 16-byte payload load
//              (clamped into the payload, rotated) + one ds_read_b128 per
//              chunk. Word path for 4-byte-aligned tiles, byte path for the
//              others (unpadded odd-length payloads).
#include "common.h"
#include "kernels.h"

namespace onc {

// Per-record plan + per-tile byte totals: tile = kEmitRecs (64) records =
// one wavefront scan (lane 63 writes the total); a workgroup of kLenRecs =
// 1024 records writes its total for the scan. Each lane plans kLenPer (2)
// records, one of each of its wave's two tiles (stores stay coalesced), with
// both descriptors' loads issued before either is used: 512-thread
// workgroups, half the waves of one record per lane, so the whole grid is
// resident at once (1M records: 7.8k waves on 8k slots) instead of 1.9
// rounds of workgroups.
constexpr int kLenPer = 2;
constexpr int kLenThreads = kLenRecs / kLenPer;
// kRoot: a.root selects the serialised type (onc_encode_body, ONC_ROOT_*);
// otherwise RpcMessage (the product encode, instantiated without the root
// switch).
template <bool kRoot>
__global__ __launch_bounds__(kLenThreads) void enc_len_kernel(EncArgs a) {
    __shared__ uint64_t s_wave[2 * (kLenThreads / 64)];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t rw = uint64_t(blockIdx.x) * kLenRecs + uint64_t(wv) * (64 * kLenPer);
    onc_msg d[kLenPer];
#pragma unroll
    for (int k = 0; k < kLenPer; ++k) {
        const uint64_t r = rw + 64 * k + lane;
        if (r < a.n) d[k] = a.msgs[r];
    }
    uint64_t wsum = 0, psum = 0;
#pragma unroll
    for (int k = 0; k < kLenPer; ++k) {
        const uint64_t r = rw + 64 * k + lane;
        uint64_t len = 0, pay = 0;
        if (r < a.n) {
            RecPlan p;
            if (kRoot) {
                p = plan_root(d[k], a.unix, a.bounds, a.root);
            } else {
                // decl 1 (the plan of an emit): declared AUTH_UNIX lengths as
                // given (no parameter-block load: the emit checks the block);
                // a record failing that form is planned in full for its
                // reference-order status (rare: only failing records).
                // decl 2 (onc_encode_lengths): the same extent, every check
                // up front for the status (include/onc_rpc.h onc_auth)
                if (a.decl) p = plan_record<true>(d[k], a.unix, a.bounds);
                if (a.decl == 2) {
                    const RecPlan f = plan_record<false>(d[k], a.unix, a.bounds);
                    p.status = f.status;
                } else if (!a.decl || p.status != ONC_OK) {
                    p = plan_record<false>(d[k], a.unix, a.bounds);
                }
            }
            len = p.len;
            pay = len - 4ull * meta_hw(p.meta);           // 0 for a record without extent (len = meta = 0)
            a.status[r] = p.status;
            if (a.rec_len) a.rec_len[r] = uint32_t(len);
            if (a.len_out) a.len_out[r] = uint32_t(len);
        }
        const uint64_t incl = wave_incl_scan_u64(len);
        const uint64_t tile = (rw + 64 * k) / kEmitRecs;
        if (lane == 63 && tile * kEmitRecs < a.n) a.tile_sum[tile] = incl;
        wsum += lane_u64(incl, 63);
        if (a.block_pay) psum += lane_u64(wave_incl_scan_u64(pay), 63);
    }
    if (lane == 0) s_wave[wv] = wsum;
    if (lane == 0 && a.block_pay) s_wave[kLenThreads / 64 + wv] = psum;
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint64_t v = threadIdx.x < kLenThreads / 64 ? s_wave[threadIdx.x] : 0;
        const uint64_t t = wave_incl_scan_u64(v);
        if (threadIdx.x == 63) a.block_sum[blockIdx.x] = t;
        if (a.block_pay) {
            const uint64_t q = wave_incl_scan_u64(threadIdx.x < kLenThreads / 64 ? s_wave[kLenThreads / 64 + threadIdx.x] : 0);
            if (threadIdx.x == 63) a.block_pay[blockIdx.x] = q;
        }
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
// + totals of the tiles before it there (lane i loads tile i of the
// workgroup; one wave reduction). The base is the scan kernel's output, or
// (kFused) the sum of the workgroup totals before it, lane l adding
// workgroups l, l + 64, ... Split in two so that the caller can issue its
// own loads between: tile_loads issues every load (no branches, clamped
// indices), tile_reduce consumes them. Wave-uniform result.
template <bool kFused>
struct TileLoads {
    static constexpr int kW = kFused ? int(kFusedBlocks / 64) : 1;
    uint64_t v;
    uint64_t w[kW];
};

// kGiven: the base of the tile's enc_len workgroup is the caller's
// (`given`, the running sum of the wave-specialised kernel's header-heavy
// mode) instead of a load of the scanned bases.
template <bool kFused, bool kGiven = false>
__device__ __forceinline__ TileLoads<kFused> tile_loads(const EncArgs& a, uint64_t tile, uint64_t given = 0) {
    const int lane = threadIdx.x & 63;
    const uint64_t blk = tile / (kLenRecs / kEmitRecs);
    const uint64_t t0 = blk * (kLenRecs / kEmitRecs);
    TileLoads<kFused> t;
    t.v = a.tile_sum[t0 + (lane < kLenRecs / kEmitRecs ? lane : 0)];
    if (kFused) {
        const uint64_t nb = num_len_blocks(a.n);
#pragma unroll
        for (int k = 0; k < TileLoads<kFused>::kW; ++k) t.w[k] = a.block_sum[min(uint64_t(lane) + uint64_t(64 * k), nb - 1)];
    } else {
        t.w[0] = kGiven ? given : a.block_base[blk];
    }
    return t;
}

template <bool kFused>
__device__ __forceinline__ uint64_t tile_reduce(const TileLoads<kFused>& t, uint64_t tile) {
    const int lane = threadIdx.x & 63;
    const uint64_t blk = tile / (kLenRecs / kEmitRecs);
    const uint64_t t0 = blk * (kLenRecs / kEmitRecs);
    uint64_t v = t0 + lane < tile ? t.v : 0;
    if (kFused) {
#pragma unroll
        for (int k = 0; k < TileLoads<kFused>::kW; ++k) v += lane + 64ull * k < blk ? t.w[k] : 0;
        return lane_u64(wave_incl_scan_u64(v), 63);
    }
    return t.w[0] + lane_u64(wave_incl_scan_u64(v), 63);
}

// Bytes the caller's earlier launches already placed before this launch's
// first record (onc_encode of a batch in chunks: the previous chunk's end,
// read from the rec_off it wrote); 0 for a whole batch.
__device__ __forceinline__ uint64_t launch_base(const EncArgs& a) { return a.base_dev ? *a.base_dev : 0ull; }

constexpr int kFastWaves = 4;                 // wave tiles per enc_emit workgroup

// Phase timestamps of a tile (lab builds with -DONC_EMIT_PROF only):
// 0 start, 1 placement known, 2 plan + scan done, 3 span staged in LDS,
// 4 span streamed, 5 tile done (s_memrealtime, 100 MHz).
#ifdef ONC_EMIT_PROF
#define ONC_PROF(k) \
    do { if (a.prof && (threadIdx.x & 63) == 0) a.prof[8 * tile + (k)] = wall_clock64(); } while (0)
#else
#define ONC_PROF(k) do {} while (0)
#endif

// ---------------------------------------------------------------------------
// enc_emit (chunk image): every load of a step in flight.
// ---------------------------------------------------------------------------
// The span's output is cut into 16-byte chunks. A chunk wholly inside one
// record's payload is "pure". Every other chunk holds header bytes; its
// header bytes are assembled in LDS while the wave stages the span, in an
// image that is the span's output with the pure chunks cut out: chunk c of
// record r sits at slot c - NP_r before r's pure run and c - NP_r - np_r
// after it (np_r = r's pure chunks, NP_r = the sum over the records before
// r). The stream loop then does, per chunk, one 16-byte payload load and
// one ds_read_b128 of its image slot, and takes each byte from one or the
// other. The payload load of a chunk that is only partly payload is clamped
// into the payload ([pst, en - 16]) and rotated into place, so nothing
// outside the payload is read and the staging does no payload loads
// (records with 0 < payload < 16 bytes put their payload in the image).
// No branch separates one chunk's load from the next, so kU chunks per lane
// (kU KiB per wave) are in flight at once.
// Two stream loops, chosen per tile (wave-uniform): when every record starts
// and ends on a 4-byte boundary and its payload source is 4-byte aligned
// (XDR payloads are), each output dword is wholly header or payload: one
// 4-aligned dwordx4 load, a dword rotation, a per-dword select. Otherwise
// (unpadded odd-length payloads) the byte path: the header is written into
// the image at its byte alignment (partial dwords with byte stores, the
// neighbours own the other bytes), the payload load is a dwordx4 + dword
// at the 4-aligned address below the window + v_alignbyte, then a byte
// rotation and a byte-masked merge (v_bfi).
// Image capacity per span: 320 chunks (7.7 KiB per wave with the entries and
// the map; 4 workgroups of 4 waves per CU, the VGPR limit, use 123 KiB of
// LDS). A tile of 64 configs[0]-shaped records (AUTH_UNIX with 16 gids,
// ~9 header chunks each: 576) streams in 2 spans instead of 3 at 248:
// enc_emit 126 -> 117 us on c0; c1 (~4 per record) is one span either way.
#ifndef ONC_IMG_CHUNKS
#define ONC_IMG_CHUNKS 320
#endif
constexpr int kImgChunks = ONC_IMG_CHUNKS;
#ifndef ONC_MAP_CAP
#define ONC_MAP_CAP 512
#define ONC_GSH_MIN 2
#endif
constexpr int kMap2Cap = ONC_MAP_CAP;         // granules per span (granule = 4 chunks, doubled to fit; an
                                              // exact 2048-entry chunk map measured no faster)
#ifndef ONC_EMIT_U
#define ONC_EMIT_U 1
#endif
constexpr int kEmitChunkUnroll = ONC_EMIT_U;    // chunks per lane per pipelined step
constexpr int kEmitNT = 2;                    // nontemporal output stores (loads: only for long payloads, launch_enc_emit)
constexpr uint64_t kSpanBytesMax = 1ull << 30;  // a span's offsets fit uint32 (one record may exceed it)
// A record's own non-pure chunks: its header is at most 4 * (7 + 2 * 54)
// = 460 bytes (a Call whose cred and verifier are both AUTH_UNIX at the
// associated-data limit of 200 bytes: 2 + 1 + 1 + 47 + 3 words for a
// 188-byte name and no gids, or 2 + 1 + 1 + 31 + 3 + 16 for a 124-byte name
// and 16 gids), a payload under 16 bytes joins it in the image (<= 475
// bytes), and the header can start and end inside a chunk: <= 31 chunks.
// Spans are cut at run time to what fits the image (the loop below), so the
// only static requirement is that one maximal record always fits on its own.
static_assert((4 * (7 + 2 * 54) + 15 + 15) / 16 + 1 <= kImgChunks, "one maximal record must fit the image");

// pay[].x = pay[].y of a record with no streamed payload (none, or under 16
// bytes and kept in the image): no chunk overlaps [kNoPay, kNoPay)
constexpr uint32_t kNoPay = 0x7FFFFFF0u;

struct ImgTile {
    uint4 img[kImgChunks];           // assembled non-pure chunks (header bytes; small payloads)
    int4 ent[kEmitRecs + 1];         // {cf, NP + pure chunks, cp1, NP} (chunks, span-relative); [ns].x = sentinel
    uint4 pay[kEmitRecs + 1];        // {pst, en (bytes, span-chunk-relative; kNoPay both: no stream payload), src lo, hi}
    uint8_t map[kMap2Cap];           // granule -> span record owning its first chunk
    int32_t bad[kEmitRecs];          // a declared credential's failing deferred check (0: none)
};

// Image slots are swizzled inside aligned groups of 8 (slot s lives at
// s ^ ((s >> 3) & 7)). The header build writes one dword per lane per
// instruction, lane = record, and records of one shape sit a fixed number of
// slots apart: configs[0]'s 128-byte AUTH_UNIX headers are 8 slots = 32
// dwords apart, so without the swizzle all 32 lanes of a ds_or_b32 lane
// group hit one bank (bank = dword mod 32) — 32-way. With it, neighbouring
// records' same word lands on 8 different chunk positions (4-way). The
// swizzle stays inside a group of 8, so the capacity is unchanged.
__device__ __forceinline__ int32_t img_slot(int32_t s) { return s ^ ((s >> 3) & 7); }
__device__ __forceinline__ uint32_t img_dword(uint32_t d) {
    return d ^ (((d >> 5) & 7u) << 2);
}
static_assert(kImgChunks % 8 == 0, "the slot swizzle permutes aligned groups of 8");

// Header words of a record into the image at byte offset b (any alignment).
// The image is zeroed per span and every record ORs its bytes in
// (ds_or_b32): a dword shared with a neighbouring record (b & 3 != 0: the
// first and last of the record) gets each record's own bytes with zeros
// elsewhere, so no byte-granular stores and no ordering between lanes are
// needed. One branch-free sink type, so the header serialiser is
// instantiated once.
struct ImgSink {
    uint32_t* img32;
    uint32_t d;        // image dword being produced (unswizzled)
    uint32_t sh;       // 32 - 8 * (b & 3)
    uint32_t prev;
    __device__ __forceinline__ void operator()(uint32_t w) {
        const uint32_t v = uint32_t(((uint64_t(w) << 32) | prev) >> sh);
        __hip_atomic_fetch_or(img32 + img_dword(d), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        ++d;
        prev = w;
    }
    __device__ __forceinline__ void finish() {
        if (sh != 32)
            __hip_atomic_fetch_or(img32 + img_dword(d), prev >> sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
};

#if defined(ONC_LAB_HDR)
struct XorSink {
    uint32_t acc;
    __device__ __forceinline__ void operator()(uint32_t w) { acc = (acc << 1 | acc >> 31) ^ w; }
};
#endif

// Clear bytes [b, b + n) of the image (the header words of a record that
// failed a deferred check, already ORed in): the neighbours' bytes in the
// two edge dwords stay.
__device__ __forceinline__ void img_clear(uint32_t* img32, uint32_t b, uint32_t n) {
    const uint32_t e = b + n;
    for (uint32_t dw = b >> 2; 4 * dw < e; ++dw) {
        const uint32_t lo = max(b, 4 * dw) - 4 * dw, hi = min(e, 4 * dw + 4) - 4 * dw;   // bytes [lo, hi) of the dword
        const uint32_t m = (hi == 4 ? ~0u : (1u << (8 * hi)) - 1u) & ~((1u << (8 * lo)) - 1u);
        __hip_atomic_fetch_and(img32 + img_dword(dw), ~m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
}

// One chunk of the word path: dword i is payload (sel bit i) taken from the
// rotated load, else the image dword.
// The rotation by `rot` dwords is two select stages on its bits (8 selects)
// rather than a 4-way select per dword.
__device__ __forceinline__ void merge_words(const u32x4_a4& X, const uint4& L, uint32_t sel, uint32_t v[4]) {
    const bool r1 = (sel >> 4) & 1u, r2 = (sel >> 5) & 1u;
    const uint32_t a0 = r1 ? X.y : X.x, a1 = r1 ? X.z : X.y, a2 = r1 ? X.w : X.z, a3 = r1 ? X.x : X.w;
    const uint32_t z0 = r2 ? a2 : a0, z1 = r2 ? a3 : a1, z2 = r2 ? a0 : a2, z3 = r2 ? a1 : a3;
    v[0] = sel & 1u ? z0 : L.x;
    v[1] = sel & 2u ? z1 : L.y;
    v[2] = sel & 4u ? z2 : L.z;
    v[3] = sel & 8u ? z3 : L.w;
}

// One chunk of the byte path: bytes [lo, hi) of the chunk are payload, taken
// from the 16 loaded bytes rotated by r; the rest from the image.
__device__ __forceinline__ void merge_bytes(const uint32_t X[4], const uint4& L, uint32_t r, uint32_t lo,
                                            uint32_t hi, uint32_t v[4]) {
    const uint32_t rd = r >> 2, rb = r & 3u;
    uint32_t Z[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t k = (uint32_t(i) + rd) & 3u;
        Z[i] = k == 0 ? X[0] : (k == 1 ? X[1] : (k == 2 ? X[2] : X[3]));
    }
    const uint32_t h[4] = {L.x, L.y, L.z, L.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t y = funnel(Z[i], Z[(i + 1) & 3], rb);
        const uint32_t a = min(max(lo, 4u * i), 4u * i + 4) - 4u * i;    // payload bytes [a, b) of dword i
        const uint32_t b = min(max(hi, 4u * i), 4u * i + 4) - 4u * i;
        const uint32_t bm = uint32_t(((1ull << (8 * b)) - 1ull) & ~((1ull << (8 * a)) - 1ull));
        v[i] = (y & bm) | (h[i] & ~bm);
    }
}

// Per-chunk plan of the stream loop: payload load address (or a dummy),
// image slot, and the merge selector (word path: bits 0-3 dword i is
// payload, bits 4-5 rotation; byte path: r | lo << 8 | hi << 16).
struct ChunkPlan {
    uintptr_t A;
    int32_t slot;
    uint32_t sel;
    uint32_t plen;           // full-interior spans: the record's streamed payload bytes (sel = o - its start)
};

template <bool kByte>
__device__ __forceinline__ ChunkPlan plan_chunk(const ImgTile& T, uint32_t gsh, uint64_t B0, int32_t c,
                                                uintptr_t dummy) {
    int r = T.map[c >> gsh];
    if (gsh != 0)                                  // exact owner when a granule is one chunk
        while (c >= T.ent[r + 1].x) ++r;
    const int4 m = T.ent[r];
    const uint4 q = T.pay[r];
    const int32_t s = c - (c >= m.z ? m.y : m.w);     // image slot: NP before the pure run, NP + its length after
    ChunkPlan P;
    P.slot = img_slot(s < 0 ? 0 : (s >= kImgChunks ? kImgChunks - 1 : s));
    const uint32_t o = uint32_t(c) << 4;
    const bool hasp = q.x < q.y && o < q.y && o + 16 > q.x;
    const uint32_t x = max(q.x, min(o, q.y - 16));            // clamped window start
    const uint64_t sbase = uint64_t(q.z) | (uint64_t(q.w) << 32);
    P.A = hasp ? sbase + B0 + x : dummy;
    if (kByte) {
        const uint32_t lo = hasp ? (q.x > o ? q.x - o : 0u) : 0u;
        const uint32_t hi = hasp ? min(q.y - o, 16u) : 0u;
        P.sel = ((o - x) & 15u) | (lo << 8) | (hi << 16);
    } else {
        // dwords i with o + 4i in [q.x, q.y) (word path: q.x, q.y, o all 4-aligned)
        const uint32_t lo = min(max(int32_t(q.x - o), 0), 16) >> 2;
        const uint32_t hi = min(max(int32_t(q.y - o), 0), 16) >> 2;
        const uint32_t pm = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
        P.sel = (hasp ? pm : 0u) | (((o - x) >> 2) & 3u) << 4;
    }
    return P;
}

// Word path, interior span (every payload's 16-byte-granular source window
// lies inside the payload arena; the producer checks it per span): the load
// for chunk c is taken at the unclamped source of its own bytes, so the
// loaded dwords are already in place — no rotation, and bytes outside the
// record's payload are other arena bytes, replaced by the image's.
__device__ __forceinline__ ChunkPlan plan_chunk_interior(const ImgTile& T, uint32_t gsh, uint64_t B0, int32_t c,
                                                         uintptr_t dummy) {
    int r = T.map[c >> gsh];
    if (gsh != 0)
        while (c >= T.ent[r + 1].x) ++r;
    const int4 m = T.ent[r];
    const uint4 q = T.pay[r];
    const int32_t s = c - (c >= m.z ? m.y : m.w);     // image slot: NP before the pure run, NP + its length after
    ChunkPlan P;
    P.slot = img_slot(s < 0 ? 0 : (s >= kImgChunks ? kImgChunks - 1 : s));
    const uint32_t o = uint32_t(c) << 4;
    const bool hasp = o < q.y && o + 16 > q.x;          // kNoPay records: never
    const uint64_t sbase = uint64_t(q.z) | (uint64_t(q.w) << 32);
    P.A = hasp ? sbase + B0 + o : dummy;
    const uint32_t lo = min(max(int32_t(q.x - o), 0), 16) >> 2;
    const uint32_t hi = min(max(int32_t(q.y - o), 0), 16) >> 2;
    P.sel = hasp ? ((1u << (hi - lo)) - 1u) << lo : 0u;
    return P;
}

// Word path, full-interior span (additionally every record of the span has
// a streamed payload and the source of each of its chunks, header chunks
// included, lies inside the arena): every chunk loads its own source bytes
// unconditionally and each dword is payload iff its offset from the
// record's payload start is below the payload length.
__device__ __forceinline__ ChunkPlan plan_chunk_full(const ImgTile& T, uint32_t gsh, uint64_t B0, int32_t c) {
    int r = T.map[c >> gsh];
    if (gsh != 0)
        while (c >= T.ent[r + 1].x) ++r;
    const int4 m = T.ent[r];
    const uint4 q = T.pay[r];
    const int32_t s = c - (c >= m.z ? m.y : m.w);
    ChunkPlan P;
    P.slot = img_slot(s < 0 ? 0 : (s >= kImgChunks ? kImgChunks - 1 : s));
    const uint32_t o = uint32_t(c) << 4;
    P.A = (uint64_t(q.z) | (uint64_t(q.w) << 32)) + B0 + o;
    P.sel = o - q.x;
    P.plen = q.y - q.x;
    return P;
}

__device__ __forceinline__ void merge_words_full(const uint32_t X[4], const uint4& L, uint32_t d, uint32_t len,
                                                 uint32_t v[4]) {
    v[0] = d < len ? X[0] : L.x;
    v[1] = d + 4u < len ? X[1] : L.y;
    v[2] = d + 8u < len ? X[2] : L.z;
    v[3] = d + 12u < len ? X[3] : L.w;
}

__device__ __forceinline__ void merge_words_inplace(const uint32_t X[4], const uint4& L, uint32_t sel, uint32_t v[4]) {
    v[0] = sel & 1u ? X[0] : L.x;
    v[1] = sel & 2u ? X[1] : L.y;
    v[2] = sel & 4u ? X[2] : L.z;
    v[3] = sel & 8u ? X[3] : L.w;
}

template <int kNT, bool kByte>
__device__ __forceinline__ void load_chunk(const ChunkPlan& P, uint32_t X[4]) {
    if (kByte) {
        load16_unaligned(P.A, X);
    } else {
        u32x4_a4 w;
        if (kNT & 1) w = __builtin_nontemporal_load(reinterpret_cast<const ONC_GLOBAL u32x4_a4*>(P.A));
        else w = gload<u32x4_a4>(P.A);
        X[0] = w.x; X[1] = w.y; X[2] = w.z; X[3] = w.w;
    }
}

template <bool kByte>
__device__ __forceinline__ void merge_chunk(const ChunkPlan& P, const uint32_t X[4], const uint4& L, uint32_t v[4]) {
    if (kByte) {
        merge_bytes(X, L, P.sel & 15u, (P.sel >> 8) & 0xFFu, P.sel >> 16, v);
    } else {
        const u32x4_a4 w = {X[0], X[1], X[2], X[3]};
        merge_words(w, L, P.sel, v);
    }
}

// The stream loop over the span's full chunks, software-pipelined with two
// register sets: step s + 1's payload loads and image reads are issued
// before step s is merged and stored. gfx950 counts loads and stores on one
// in-order vmcnt, so a load issued after a store cannot be waited for
// without waiting for the store too; issued before it, waiting for the
// loads leaves the previous step's stores in flight. The loop therefore has
// no data-dependent VMEM control flow: every step issues exactly kU loads
// and kU stores (lanes past the last full chunk repeat it — same bytes to
// the same address), and the next step is always issued (the surplus
// after the last step re-reads the last chunk). The one or two partial
// chunks at the span's edges are written with byte stores of only the
// span's bytes (EdgeChunks).
//
// The partial edge chunks of a span (lane 0: chunk 0 when the span starts
// inside it; lane 1: chunk NCe - 1 when the span ends inside another chunk):
// their payload loads are issued before the stream's first step, and they
// are merged and stored once the first two steps are issued. Loaded after
// the stream (as in round 2), the edge could not be waited for without
// waiting for every store of the span (the in-order vmcnt): a full store
// drain per span, on the wave that also starts the next span's staging (or,
// in the wave-specialised kernel, on the consumer every other one then
// waits for at the span's barrier).
template <int kNT, bool kByte>
struct EdgeChunks {
    uint32_t X[4];           // only the loaded dwords stay live across the first steps' issue; the plan
                             // (LDS reads) is taken again at the merge
    __device__ __forceinline__ static bool mine(int32_t cf, int32_t cl, int32_t NCe, int lane) {
        return (lane == 0 && cf == 1) || (lane == 1 && cl == NCe - 1 && (NCe - 1 > 0 || cf == 0));
    }
    __device__ __forceinline__ void issue(const ImgTile& T, uint32_t gsh, uint64_t B0, int32_t cf, int32_t cl,
                                          int32_t NCe, int lane, uintptr_t dummy) {
        if (mine(cf, cl, NCe, lane)) {
            const ChunkPlan P = plan_chunk<kByte>(T, gsh, B0, lane == 0 ? 0 : NCe - 1, dummy);
            load_chunk<kNT, kByte>(P, X);
        }
    }
    __device__ __forceinline__ void finish(const EncArgs& a, const ImgTile& T, uint32_t gsh, uint64_t B0,
                                           uint64_t S0, uint64_t E, int32_t cf, int32_t cl, int32_t NCe, int lane,
                                           uintptr_t dummy) const {
        if (mine(cf, cl, NCe, lane)) {
            const int32_t c = lane == 0 ? 0 : NCe - 1;
            const ChunkPlan P = plan_chunk<kByte>(T, gsh, B0, c, dummy);
            const uint4 L = T.img[P.slot];
            uint32_t v[4];
            merge_chunk<kByte>(P, X, L, v);
            const uint64_t o = B0 + (uint64_t(c) << 4);
            store_chunk(a.out, o, max(o, S0), min(o + 16, E), v);
        }
    }
};

template <int kU, int kNT, bool kByte, bool kEarly = !kByte>
__device__ __forceinline__ void stream_span(const EncArgs& a, const ImgTile& T, uint32_t gsh, uint64_t B0,
                                            uint64_t S0, uint64_t E1, int32_t NCe, uintptr_t dummy) {
    const int lane = threadIdx.x & 63;
    constexpr int32_t S = 64 * kU;
    const int32_t cf = S0 > B0 ? 1 : 0;                 // chunk 0 partial: span starts inside it
    const int32_t cl = (E1 & 15) ? NCe - 1 : NCe;         // full chunks [cf, cl)
    EdgeChunks<kNT, kByte> E;
    if (kEarly) E.issue(T, gsh, B0, cf, cl, NCe, lane, dummy);
    if (cl > cf) {
        ChunkPlan Pa[kU], Pb[kU];
        uint32_t Xa[kU][4], Xb[kU][4];
        uint4 La[kU], Lb[kU];
#define ONC_ISSUE(P, X, L, base)                                                          \
    _Pragma("unroll") for (int u = 0; u < kU; ++u) {                                     \
        P[u] = plan_chunk<kByte>(T, gsh, B0, min((base) + lane + 64 * u, cl - 1), dummy);   \
        load_chunk<kNT, kByte>(P[u], X[u]);                                               \
        L[u] = T.img[P[u].slot];                                                          \
    }
#define ONC_CONSUME(P, X, L, base)                                                        \
    _Pragma("unroll") for (int u = 0; u < kU; ++u) {                                     \
        const int32_t c = min((base) + lane + 64 * u, cl - 1);                            \
        uint32_t v[4];                                                                    \
        merge_chunk<kByte>(P[u], X[u], L[u], v);                                          \
        u32x4* d = reinterpret_cast<u32x4*>(a.out + B0 + (uint64_t(c) << 4));             \
        if (kNT & 2) __builtin_nontemporal_store(u32x4{v[0], v[1], v[2], v[3]}, d);  \
        else *d = u32x4{v[0], v[1], v[2], v[3]};                                          \
    }
        ONC_ISSUE(Pa, Xa, La, cf);
        ONC_ISSUE(Pb, Xb, Lb, cf + S);
        if (kEarly) E.finish(a, T, gsh, B0, S0, E1, cf, cl, NCe, lane, dummy);
        for (int32_t st = cf;; st += 2 * S) {
            ONC_CONSUME(Pa, Xa, La, st);
            if (st + S >= cl) break;
            ONC_ISSUE(Pa, Xa, La, st + 2 * S);
            ONC_CONSUME(Pb, Xb, Lb, st + S);
            if (st + 2 * S >= cl) break;
            ONC_ISSUE(Pb, Xb, Lb, st + 3 * S);
        }
#undef ONC_ISSUE
#undef ONC_CONSUME
    }
    if (!kEarly || cl <= cf) {
        if (!kEarly) E.issue(T, gsh, B0, cf, cl, NCe, lane, dummy);
        E.finish(a, T, gsh, B0, S0, E1, cf, cl, NCe, lane, dummy);
    }
}

// A record whose declared AUTH_UNIX credential failed a deferred block check
// (rare) keeps the extent it was placed with, so that every record after it
// stays where the plan put it; its header bytes in the image become a
// placeholder that keeps the stream framable (include/onc_rpc.h onc_auth,
// ABI 7): the record mark of its extent, (len - 4) | 1 << 31
// (rpc_message.rs:156: a receiver's expected_message_len, :343-367, cuts it
// as one whole record and goes on to the next), then zero bytes up to its
// payload. The header words the serialiser wrote (an empty parameter block
// in place of the failing one) are cleared first. Leaves the sink at the
// header's end.
__device__ __forceinline__ void img_placeholder(uint32_t* img32, ImgSink& w, uint64_t ibb, uint32_t hw, uint64_t len) {
    const uint32_t b = uint32_t(ibb);
    img_clear(img32, b, 4u * hw);
    const uint32_t mark = bswap(uint32_t(len - 4) | 0x80000000u), m = 8u * (b & 3u);
    __hip_atomic_fetch_or(img32 + img_dword(b >> 2), mark << m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    if (m) __hip_atomic_fetch_or(img32 + img_dword((b >> 2) + 1), mark >> (32u - m), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WAVEFRONT);
    w.d = (b >> 2) + hw;
    w.prev = 0u;
}

// The one-launch small batch (codec.hip small_batch: at most kSpWaves tiles,
// so the one workgroup of enc_emit_single_kernel is the whole batch): each
// wave plans its tile, hands the tile's byte total to wave 0 through LDS,
// and wave 0 hands back the exclusive prefix of the totals. All waves of a
// workgroup are resident together, so waiting on a flag another wave of it
// sets always ends; there is no predecessor workgroup and nothing in global
// memory to wait on. (Rounds 5's single-pass lab placed the tiles of larger
// batches by a decoupled look-back across workgroups; measured slower than
// enc_len + enc_emit and removed — DESIGN.md §4, profiles/HISTORY.md.)
template <int kGW>
struct WgPlace {
    uint64_t agg[kGW];
    uint64_t base[kGW];
    uint32_t ready[kGW];            // wave w's total is in agg[w] (w > 0); ready[0]: the bases are set
};
__device__ __forceinline__ uint32_t lds_flag(const uint32_t* f) {
    return __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <int kGW>
__device__ __forceinline__ uint64_t wg_place(WgPlace<kGW>& X, uint64_t tile, uint64_t agg, uint64_t ntiles) {
    const int w = int(tile % kGW);
    const int live = int(min(uint64_t(kGW), ntiles - tile / kGW * kGW));
    // (every lane stores the same wave-uniform values: no lane-0-only
    // regions next to the readfirstlane waits, tools/lookback_diag.hip)
    if (w != 0) {
        X.agg[w] = agg;
        __hip_atomic_store(&X.ready[w], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        while (__builtin_amdgcn_readfirstlane(int(lds_flag(&X.ready[0]))) == 0) __builtin_amdgcn_s_sleep(1);
        return X.base[w];
    }
    uint64_t run = agg;
    for (int v = 1; v < live; ++v) {
        while (__builtin_amdgcn_readfirstlane(int(lds_flag(&X.ready[v]))) == 0) __builtin_amdgcn_s_sleep(1);
        X.base[v] = run;
        run += X.agg[v];
    }
    __hip_atomic_store(&X.ready[0], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    return 0;
}

// kSmall: the tile of a one-workgroup small batch (enc_emit_single_kernel):
// planned here (enc_len's plan, statuses and lengths written) and placed
// through X (wg_place) instead of by enc_len's totals.
template <int kU, int kNT, bool kFused, bool kRoot = false, bool kGiven = false, bool kLen = false,
          bool kSmall = false, int kGW = kFastWaves>
__device__ __forceinline__ void enc_emit_tile(const EncArgs& a, ImgTile& T, uint64_t tile, uint64_t given = 0,
                                              WgPlace<kGW>* X = nullptr) {
    const int lane = threadIdx.x & 63;
    const uint64_t r0 = tile * kEmitRecs;
    uint32_t* img32 = reinterpret_cast<uint32_t*>(T.img);
    const int nrec = int(min(uint64_t(kEmitRecs), a.n - r0));
    const uintptr_t payload = reinterpret_cast<uintptr_t>(a.payload_arena);

    // Prologue: the tile-placement loads and this lane's descriptor issued
    // together, one memory round trip before the planning starts.
    ONC_PROF(0);
    TileLoads<kFused> tl;
    if constexpr (!kSmall) tl = tile_loads<kFused, kGiven>(a, tile, given);
    MsgRegs mr = issue_msg(a.msgs + r0 + min(lane, nrec - 1));
    // kLen: the plan's length of the lane's record, issued with the rest
    uint32_t glen = 0;
    if constexpr (kLen) glen = a.len_in[r0 + min(lane, nrec - 1)];
    if constexpr (kSmall) {
        asm volatile("" : "+v"(mr.q[0]), "+v"(mr.q[1]), "+v"(mr.q[2]), "+v"(mr.q[3]));
    } else if constexpr (kFused) {
        static_assert(TileLoads<kFused>::kW == 16, "pin list below");
        asm volatile("" : "+v"(mr.q[0]), "+v"(mr.q[1]), "+v"(mr.q[2]), "+v"(mr.q[3]), "+v"(tl.v),
                     "+v"(tl.w[0]), "+v"(tl.w[1]), "+v"(tl.w[2]), "+v"(tl.w[3]), "+v"(tl.w[4]), "+v"(tl.w[5]),
                     "+v"(tl.w[6]), "+v"(tl.w[7]), "+v"(tl.w[8]), "+v"(tl.w[9]), "+v"(tl.w[10]), "+v"(tl.w[11]),
                     "+v"(tl.w[12]), "+v"(tl.w[13]), "+v"(tl.w[14]), "+v"(tl.w[15]));
    } else {
        asm volatile("" : "+v"(mr.q[0]), "+v"(mr.q[1]), "+v"(mr.q[2]), "+v"(mr.q[3]), "+v"(tl.v), "+v"(tl.w[0]));
    }
    if constexpr (kLen) asm volatile("" : "+v"(glen));
    const onc_msg dm = as_msg(mr);
    // output coordinates: byte 0 = the 16-aligned chunk base below the
    // caller's `out`, which sits at `origin` (any writer position)
    uint64_t T0 = 0;
    if constexpr (!kSmall) T0 = a.origin + (kGiven ? 0ull : launch_base(a)) + tile_reduce<kFused>(tl, tile);
    ONC_PROF(1);
    uint64_t len = 0, poff = 0;
    uint32_t hw = 0;
    bool word_aligned = true;
    if (lane < nrec) {
        const onc_msg& d = dm;
        if constexpr (kLen) {
            // the plan's length (0: a failing record); the header is what is
            // not payload (RpcMessage bodies: a Call's, an accepted Success's)
            len = glen;
            const bool body = d.msg_type == ONC_MSG_CALL ||
                              (d.msg_type == ONC_MSG_REPLY && d.reply_stat == ONC_REPLY_ACCEPTED &&
                               d.stat == ONC_ACCEPT_SUCCESS);
            hw = len ? uint32_t((len - (body ? uint64_t(d.payload_len) : 0ull)) >> 2) : 0;
        } else if constexpr (kSmall) {
            // enc_len's plan of the record (its decl 1 form) and its outputs
            RecPlan p = plan_record<true>(d, a.unix, a.bounds);
            if (p.status != ONC_OK) p = plan_record<false>(d, a.unix, a.bounds);
            a.status[r0 + lane] = p.status;
            if (a.rec_len) a.rec_len[r0 + lane] = uint32_t(p.len);
            len = p.len;
            hw = len ? meta_hw(p.meta) : 0;
        } else {
            // the same function as enc_len: lengths agree (declared AUTH_UNIX
            // lengths: no parameter-block load here)
            const RecPlan p = kRoot ? plan_root(d, a.unix, a.bounds, a.root) : plan_record<true>(d, a.unix, a.bounds);
            len = p.len;
            hw = len ? meta_hw(p.meta) : 0;
        }
        poff = d.payload_off;
        word_aligned = (len & 3) == 0 && (len == 4ull * hw || ((payload + d.payload_off) & 3) == 0);
    }
    const uint64_t incl = wave_incl_scan_u64(len);
    if constexpr (kSmall) T0 = a.origin + wg_place(*X, tile, lane_u64(incl, 63), num_emit_tiles(a.n));
    const uint64_t start = T0 + incl - len;
    const uint64_t en = start + len;
    const uint64_t pst = start + 4ull * hw;
    if (lane < nrec) {
        // (a chunk's first offset is the base it read: the previous chunk wrote it)
        if (r0 + lane != 0 || !a.base_dev) a.rec_off[r0 + lane] = start - a.origin;
        if (r0 + lane + 1 == a.n) a.rec_off[a.n] = en - a.origin;   // the grand total
        if (len != 0 && en > a.out_cap) a.status[r0 + lane] = ONC_ENC_WRITE_ZERO;
    }
    const bool byte_mode = !(__all(word_aligned) && (T0 & 3) == 0);

    // Absolute chunk indices: owned chunks [cfa, own_next), pure [p0, p1).
    const int64_t cfa = int64_t((start + 15) >> 4);
    const int64_t p0 = int64_t((pst + 15) >> 4);
    const int64_t p1 = max(p0, int64_t(en >> 4));
    const int64_t np = len ? p1 - p0 : 0;
    const int64_t cfa_next = int64_t(next_lane_u64(uint64_t(cfa)));
    const int64_t cfa_end = int64_t((lane_u64(en, nrec - 1) + 15) >> 4);
    const int64_t own_next = lane + 1 < nrec ? cfa_next : cfa_end;
    const uint32_t nonpure = lane < nrec && len ? uint32_t(own_next - cfa - np) : 0u;
    const uint64_t wnp = wave_incl_scan_u64(nonpure);
    const uint64_t plen = en - pst;

    const uintptr_t dummy = reinterpret_cast<uintptr_t>(a.msgs);   // >= 64 valid bytes
    ONC_PROF(2);
    if (!kRoot) T.bad[lane] = ONC_OK;
    int lo_rec = 0;
    while (lo_rec < nrec) {
        // span: records [lo_rec, hi_rec) whose non-pure chunks (+1 for a
        // chunk shared with the record before) fit the image and whose bytes
        // fit kSpanBytesMax (at least one record)
        const uint64_t wbase = lo_rec ? lane_u64(wnp, lo_rec - 1) : 0;
        const uint64_t sbeg = lane_u64(start, lo_rec);
        const uint64_t over = __ballot(lane > lo_rec && lane < nrec &&
                                       (wnp - wbase + 1 > uint64_t(kImgChunks) || en - sbeg > kSpanBytesMax));
        const int hi_rec = over ? min(nrec, int(__builtin_ctzll(over))) : nrec;
        const int ns = hi_rec - lo_rec;
        const uint64_t S0 = sbeg;
        const uint64_t S1 = lane_u64(en, hi_rec - 1);
        const int64_t C0 = int64_t(S0 >> 4);
        const uint64_t B0 = uint64_t(C0) << 4;        // byte origin of the span-relative offsets
        if (lo_rec) wave_lds_sync();                   // the previous span's readers are done
        // records OR into the image: zero the slots this span uses (the
        // cut above bounds them by kImgChunks)
        // (whole groups of 8: the swizzle permutes inside a group)
        const int used = int(min(uint64_t(kImgChunks), uint64_t((lane_u64(wnp, hi_rec - 1) - wbase + 8) & ~7ull)));
        for (int k = lane; k < used; k += 64) T.img[k] = make_uint4(0, 0, 0, 0);
        const bool active = lane >= lo_rec && lane < hi_rec;
        const int j = lane - lo_rec;
        const int64_t npx = active ? np : 0;
        const int64_t NP = int64_t(wave_incl_scan_u64(uint64_t(npx))) - npx;   // lanes < lo_rec add 0
        const int32_t NC = int32_t(((S1 + 15) >> 4) - C0);
        uint32_t gsh = ONC_GSH_MIN;                    // granule = 4 chunks, doubled until the span fits
        while ((NC >> gsh) >= kMap2Cap) ++gsh;
        const uint64_t nonempty = __ballot(active && len != 0);
        if (active) {
            const bool small = plen != 0 && plen < 16;    // payload kept in the image
            const uintptr_t sb = payload + poff - pst;    // payload byte at output offset o: sb + o
            T.ent[j] = make_int4(int32_t(cfa - C0), int32_t(NP + npx), int32_t(p1 - C0), int32_t(NP));
            const uint32_t ps = uint32_t(pst - B0), pe = uint32_t(en - B0);
            const bool nopay = small || ps == pe;
            T.pay[j] = make_uint4(nopay ? kNoPay : ps, nopay ? kNoPay : pe, uint32_t(sb), uint32_t(sb >> 32));
            if (len != 0) {
                // the record's non-pure bytes are contiguous in the image from
                // image byte start - 16 (C0 + NP)
                const uint64_t ibb = start - 16ull * uint64_t(C0 + NP);
                // reloaded (an L2 hit) rather than kept live across the span
                // loop (kept live: 162 VGPRs, 3 waves per SIMD)
                MsgRegs mr2 = issue_msg(a.msgs + r0 + lane);
                asm volatile("" : "+v"(mr2.q[0]), "+v"(mr2.q[1]), "+v"(mr2.q[2]), "+v"(mr2.q[3]));
                const onc_msg d = as_msg(mr2);
                const EncSrc src{a.unix, reinterpret_cast<uintptr_t>(a.auth_arena), payload};
                ImgSink w{img32, uint32_t(ibb >> 2), 32u - 8u * uint32_t(ibb & 3), 0u};
                // a declared AUTH_UNIX credential: the parameter-block checks
                // the plan deferred run on the block words the serialiser
                // loads (or preloaded), which stops there; a failing record
                // keeps its extent, the words written so far cleared
                // (include/onc_rpc.h onc_auth). (Checking the preloaded block
                // before the header build instead: 15 VGPRs spilled.)
                // (the status lands in LDS, read back right after the build:
                // nothing extra live across the header build)
                DeclCheck dc{a.bounds.auth_len, &T.bad[lane]};
#if defined(ONC_LAB_HDR)
                // lab builds only (tools/hdr_lab.sh; wrong output bytes):
                // 1 = no header build at all (the image stays zero),
                // 2 = the header words computed (every load) but not written
                // to the image: what the LDS writes of the build cost,
                // 3 = everything but the credential block's load
                if constexpr (ONC_LAB_HDR == 2) {
                    XorSink xs{0u};
                    if (kRoot) put_root_words(d, uint32_t(len), src, a.root, xs);
                    else put_header_words(d, uint32_t(len), src, xs, nullptr, false, &dc);
                    if (xs.acc == 0x9E3779B9u) img32[0] = xs.acc;       // keeps the words live
                } else if constexpr (ONC_LAB_HDR == 3) {
                    // 3 = the header written with a register-made credential
                    // block (stamp 0, uid 501, gid 20, 16 gids, no name): the
                    // whole build but the block's load
                    UnixRegs fk;
                    fk.q[0] = u32x4{0u, 501u, 20u, 16u};
                    fk.q[1] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
                    for (int k = 2; k < 6; ++k) fk.q[k] = u32x4{uint32_t(k), 7u, 11u, 13u};
                    put_header_words(d, uint32_t(len), src, w, &fk, true, &dc);
                }
#else
                if (kRoot) put_root_words(d, uint32_t(len), src, a.root, w);
                else put_header_words(d, uint32_t(len), src, w, nullptr, false, &dc);
#endif
                if (!kRoot) {
                    const int32_t bad = T.bad[lane];
                    if (bad != ONC_OK) {
                        a.status[r0 + lane] = bad;
                        img_placeholder(img32, w, ibb, hw, len);
                    }
                }
                if (small) {
                    // all of it lies in non-pure chunks (np = 0): right after
                    // the header (bytes past its end read as zero), by a sink
                    // of its own (the header's last bytes flushed first: both
                    // OR into the dword they share)
                    w.finish();
                    const uintptr_t pb = sb + pst;
                    w = ImgSink{img32, uint32_t(ibb >> 2) + hw, w.sh, 0u};
                    for (uint32_t k = 0; 4 * k < plen; ++k) w(load4_masked(pb + 4 * k, pb + plen));
                } else if (kRoot && plen != 0 && pst < (uint64_t(cfa) << 4)) {
                    // a body root's header can be shorter than a chunk
                    // (AcceptedStatus: 4 bytes): payload bytes in the chunk
                    // the record starts in belong to a chunk the record
                    // before owns, whose stream loads only its own payload —
                    // they go into the image (the rest streams from chunk
                    // cfa on). A message header (>= 24 bytes) always ends
                    // past that chunk.
                    const uintptr_t pb = sb + pst;
                    const uint32_t h = uint32_t((uint64_t(cfa) << 4) - pst);
                    for (uint32_t k = 0; 4 * k < h; ++k) w(load4_masked(pb + 4 * k, pb + h));
                }
                w.finish();
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
        if (lo_rec == 0) ONC_PROF(3);

        const uint64_t E = min(S1, a.out_cap);
        lo_rec = hi_rec;
        if (E <= S0) continue;                         // no bytes (all records failed, or beyond out_cap)
        const int32_t NCe = int32_t(((E + 15) >> 4) - C0);
        if (byte_mode) stream_span<1, kNT, true>(a, T, gsh, B0, S0, E, NCe, dummy);
        else stream_span<kU, kNT, false>(a, T, gsh, B0, S0, E, NCe, dummy);
        if (lo_rec == hi_rec && hi_rec == nrec) ONC_PROF(4);
    }
    ONC_PROF(5);
}

// ---------------------------------------------------------------------------
// enc_emit, wave-specialised (ONC_EMIT_WS): a persistent workgroup of 4 waves
// runs a two-slot pipeline over its tiles (tile = blockIdx.x + k * gridDim.x):
// wave 0 (the producer) does everything enc_emit_tile does before the
// stream — placement, plan, scans, the span's LDS image and maps — for the
// next span into one slot while waves 1-3 (the consumers) stream the
// previous span out of the other slot, interleaved by steps of 64 * kU
// chunks (consumer c takes steps c, c + 3, ...; kU = 2, or 1 for payloads
// averaging >= 512 bytes). One workgroup barrier per span. The wave-per-
// tile kernel keeps ~26 % of every tile's life in staging with no memory
// traffic, and its tiles start in lock-step rounds, so those phases
// coincide chip-wide; here the streams never stop for staging. Chosen per
// batch by codec.hip (enc_args); DESIGN.md §4 has the measurements.
struct SpanHdr {
    uint64_t B0, S0, E;
    int32_t NCe;
    uint32_t gsh;
    uint32_t byte_mode;
    uint32_t state;          // 0: nothing to stream, 1: stream, 2: no more spans
    uint32_t interior;       // word path: 1 every payload source window inside the arena (plan_chunk_interior), 2 every chunk source too (plan_chunk_full)
};
struct WsSlot {
    ImgTile T;
    SpanHdr h;
};

// The producer's per-tile state: wave-uniform values in registers, the
// per-record ones (lane = record) in LDS — kept in registers across the
// phase loop they would be live in the consumers' stream too (178 VGPRs).
struct WsTile {
    uint64_t tile, r0;
    int nrec, lo_rec;
    bool byte_mode;
    uint64_t run_blk, run_base;   // enc_len workgroup totals summed so far: [0, run_blk)
};
struct WsLane {
    uint64_t len, poff, start, en, pst, wnp;
    int64_t cfa, p0, p1, own_next;
};

// Tile placement without a scan launch and without the 16 pinned loads of
// the fused wave-per-tile path: a workgroup's tiles ascend, so the producer
// keeps a running sum of the enc_len workgroup totals and adds the ones
// between its previous tile's workgroup and this one's (<= 64: one load
// per lane), then the tile totals before the tile inside its workgroup.
constexpr uint64_t kTilesPerBlk = kLenRecs / kEmitRecs;
// A tile's prologue loads (its workgroup's tile totals, the workgroup totals
// since the producer's previous tile, its descriptors), issued together.
// (Issuing them a phase ahead, in flight across the barrier, measured no
// faster.)
struct WsLoads {
    MsgRegs mr;
    uint64_t tv, bw;
};
__device__ __forceinline__ WsLoads ws_issue(const EncArgs& a, uint64_t run_blk, uint64_t tile) {
    const int lane = threadIdx.x & 63;
    const uint64_t t0 = tile / kTilesPerBlk * kTilesPerBlk;
    const uint64_t r0 = tile * kEmitRecs;
    const int nrec = int(min(uint64_t(kEmitRecs), a.n - r0));
    WsLoads L;
    L.tv = a.tile_sum[t0 + (uint64_t(lane) < kTilesPerBlk ? lane : 0)];
    L.bw = a.block_sum[min(run_blk + lane, num_len_blocks(a.n) - 1)];
    L.mr = issue_msg(a.msgs + r0 + min(lane, nrec - 1));
    return L;
}

// The tile's descriptors as the prologue loaded them, kept in LDS for the
// header builds of its spans ([quarter][lane]: conflict-free b128 accesses)
// instead of a second load from L2 per span (a dependent round trip on the
// producer's path while the consumers hold the memory system busy).
struct WsDesc {
    u32x4 q[4][64];
};
__device__ __forceinline__ void ws_begin_tile(const EncArgs& a, WsTile& S, WsLane* ln, WsDesc& dsc, uint64_t tile,
                                              WsLoads pf) {
    const int lane = threadIdx.x & 63;
    const uintptr_t payload = reinterpret_cast<uintptr_t>(a.payload_arena);
    S.tile = tile;
    S.r0 = tile * kEmitRecs;
    S.nrec = int(min(uint64_t(kEmitRecs), a.n - S.r0));
    S.lo_rec = 0;
    const uint64_t blk = tile / kTilesPerBlk;
    const uint64_t t0 = blk * kTilesPerBlk;
    const uint64_t tv = pf.tv, bw = pf.bw;
    const MsgRegs mr = pf.mr;
#pragma unroll
    for (int k = 0; k < 4; ++k) dsc.q[k][lane] = mr.q[k];
    S.run_base += lane_u64(wave_incl_scan_u64(S.run_blk + lane < blk ? bw : 0), 63);
    S.run_blk = blk;
    const uint64_t T0 = a.origin + S.run_base + lane_u64(wave_incl_scan_u64(t0 + lane < tile ? tv : 0), 63);
    const onc_msg dm = as_msg(mr);
    uint64_t len = 0, poff = 0;
    uint32_t hw = 0;
    bool word_aligned = true;
    if (lane < S.nrec) {
        const RecPlan p = plan_record<true>(dm, a.unix, a.bounds);
        len = p.len;
        hw = len ? meta_hw(p.meta) : 0;
        poff = dm.payload_off;
        word_aligned = (len & 3) == 0 && (len == 4ull * hw || ((payload + dm.payload_off) & 3) == 0);
    }
    const uint64_t incl = wave_incl_scan_u64(len);
    const uint64_t start = T0 + incl - len;
    const uint64_t en = start + len;
    const uint64_t pst = start + 4ull * hw;
    if (lane < S.nrec) {
        // (a chunk's first offset is the base it read: the previous chunk wrote it)
        if (S.r0 + lane != 0 || !a.base_dev) a.rec_off[S.r0 + lane] = start - a.origin;
        if (S.r0 + lane + 1 == a.n) a.rec_off[a.n] = en - a.origin;
        if (len != 0 && en > a.out_cap) a.status[S.r0 + lane] = ONC_ENC_WRITE_ZERO;
    }
    S.byte_mode = !(__all(word_aligned) && (T0 & 3) == 0);
    const int64_t cfa = int64_t((start + 15) >> 4);
    const int64_t p0 = int64_t((pst + 15) >> 4);
    const int64_t p1 = max(p0, int64_t(en >> 4));
    const int64_t np = len ? p1 - p0 : 0;
    const int64_t cfa_next = int64_t(next_lane_u64(uint64_t(cfa)));
    const int64_t cfa_end = int64_t((lane_u64(en, S.nrec - 1) + 15) >> 4);
    const int64_t own_next = lane + 1 < S.nrec ? cfa_next : cfa_end;
    const uint32_t nonpure = lane < S.nrec && len ? uint32_t(own_next - cfa - np) : 0u;
    const uint64_t wnp = wave_incl_scan_u64(nonpure);
    ln[lane] = WsLane{len, poff, start, en, pst, wnp, cfa, p0, p1, own_next};
}

// The next span of the producer's tile into slot W (image, entries, map,
// header); advances S.lo_rec.
__device__ __forceinline__ void ws_stage_span(const EncArgs& a, WsTile& S, const WsLane* ln, const WsDesc& dsc,
                                              WsSlot& W) {
    const int lane = threadIdx.x & 63;
    const WsLane L = ln[lane];
    const uint64_t Slen = L.len, Spoff = L.poff, Sstart = L.start, Sen = L.en, Spst = L.pst, Swnp = L.wnp;
    const int64_t Scfa = L.cfa, Sp0 = L.p0, Sp1 = L.p1, Sown_next = L.own_next;
    const int64_t Snp = Slen ? Sp1 - Sp0 : 0;
    const uint64_t Splen = Sen - Spst;
    const uintptr_t payload = reinterpret_cast<uintptr_t>(a.payload_arena);
    uint32_t* img32 = reinterpret_cast<uint32_t*>(W.T.img);
    const int lo_rec = S.lo_rec, nrec = S.nrec;
    const uint64_t wbase = lo_rec ? lane_u64(Swnp, lo_rec - 1) : 0;
    const uint64_t sbeg = lane_u64(Sstart, lo_rec);
    const uint64_t over = __ballot(lane > lo_rec && lane < nrec &&
                                   (Swnp - wbase + 1 > uint64_t(kImgChunks) || Sen - sbeg > kSpanBytesMax));
    const int hi_rec = over ? min(nrec, int(__builtin_ctzll(over))) : nrec;
    const uint64_t S0 = sbeg;
    const uint64_t S1 = lane_u64(Sen, hi_rec - 1);
    const int64_t C0 = int64_t(S0 >> 4);
    const uint64_t B0 = uint64_t(C0) << 4;
    const int used = int(min(uint64_t(kImgChunks), uint64_t((lane_u64(Swnp, hi_rec - 1) - wbase + 8) & ~7ull)));
    for (int k = lane; k < used; k += 64) W.T.img[k] = make_uint4(0, 0, 0, 0);
    const bool active = lane >= lo_rec && lane < hi_rec;
    const int j = lane - lo_rec;
    const int64_t npx = active ? Snp : 0;
    const int64_t NP = int64_t(wave_incl_scan_u64(uint64_t(npx))) - npx;
    const int32_t NC = int32_t(((S1 + 15) >> 4) - C0);
    uint32_t gsh = ONC_GSH_MIN;
    while ((NC >> gsh) >= kMap2Cap) ++gsh;
    const uint64_t nonempty = __ballot(active && Slen != 0);
    wave_lds_sync();                                   // the zeroed image before the ORs
    if (active) {
        const bool small = Splen != 0 && Splen < 16;
        const uintptr_t sb = payload + Spoff - Spst;
        W.T.ent[j] = make_int4(int32_t(Scfa - C0), int32_t(NP + npx), int32_t(Sp1 - C0), int32_t(NP));
        const uint32_t ps = uint32_t(Spst - B0), pe = uint32_t(Sen - B0);
        const bool nopay = small || ps == pe;
        W.T.pay[j] = make_uint4(nopay ? kNoPay : ps, nopay ? kNoPay : pe, uint32_t(sb), uint32_t(sb >> 32));
        if (Slen != 0) {
            const uint64_t ibb = Sstart - 16ull * uint64_t(C0 + NP);
            MsgRegs mr2;
#pragma unroll
            for (int k = 0; k < 4; ++k) mr2.q[k] = dsc.q[k][lane];
            const onc_msg d = as_msg(mr2);
            const EncSrc src{a.unix, reinterpret_cast<uintptr_t>(a.auth_arena), payload};
            ImgSink w{img32, uint32_t(ibb >> 2), 32u - 8u * uint32_t(ibb & 3), 0u};
            int32_t bad = ONC_OK;
            DeclCheck dc{a.bounds.auth_len, &bad};
            put_header_words(d, uint32_t(Slen), src, w, nullptr, false, &dc);
            if (bad != ONC_OK) {                       // (see enc_emit_tile)
                a.status[S.r0 + lane] = bad;
                img_placeholder(img32, w, ibb, uint32_t((Spst - Sstart) >> 2), (Spst - Sstart) + Splen);   // (Slen: not kept live)
            }
            if (small) {
                const uintptr_t pb = sb + Spst;
                for (uint32_t k = 0; 4 * k < Splen; ++k) w(load4_masked(pb + 4 * k, pb + Splen));
            }
            w.finish();
            const int32_t own_lo = (S0 & 15) && lane == __builtin_ctzll(nonempty) ? 0 : int32_t(Scfa - C0);
            const int32_t own_hi = int32_t(Sown_next - C0);
            const int32_t g_hi = min((own_hi + (1 << gsh) - 1) >> gsh, kMap2Cap);
            for (int32_t g = (own_lo + (1 << gsh) - 1) >> gsh; g < g_hi; ++g) W.T.map[g] = uint8_t(j);
        }
    }
    // interior: the 16-byte-granular source windows of every payload of the
    // span (from its first to its last output chunk) lie inside the arena
    bool inside = true, full = true;
    if (active && Splen >= 16) {
        const uint64_t head = Spst & 15u, tail = (16u - (Sen & 15u)) & 15u;
        inside = Spoff >= head && Spoff + Splen + tail <= a.bounds.payload_len;
        // full: the record's own chunks from its first (cfa) on read inside the arena too
        full = inside && Spoff >= Spst - (uint64_t(Scfa) << 4);
    } else if (active && Slen != 0) {
        full = false;                                  // a record without streamed payload: chunks need `hasp`
    }
    const bool interior = __all(inside);
    const bool interior_full = __all(full);
    const uint64_t E = min(S1, a.out_cap);
    if (lane == 0) {
        W.T.ent[hi_rec - lo_rec] = make_int4(0x7FFFFFFF, 0, 0, 0);
        SpanHdr h;
        h.B0 = B0;
        h.S0 = S0;
        h.E = E;
        h.NCe = E > S0 ? int32_t(((E + 15) >> 4) - C0) : 0;
        h.gsh = gsh;
        h.byte_mode = S.byte_mode ? 1u : 0u;
        h.state = E > S0 ? 1u : 0u;
        h.interior = S.byte_mode || !interior ? 0u : (interior_full ? 2u : 1u);
        W.h = h;
    }
    S.lo_rec = hi_rec;
}

// stream_span for consumer `part` of `nparts`: the span's full chunks in
// steps of 64 * kU chunks, this wave taking steps part, part + nparts, ...
// (same two-register-set pipeline); part nparts - 1, which never has more
// steps than another part, also writes the partial edge chunks.
template <int kU, int kNT, bool kByte, int kInterior = 0>
__device__ __forceinline__ void stream_span_part(const EncArgs& a, const ImgTile& T, const SpanHdr& h, int part,
                                                 int nparts, uintptr_t dummy) {
    const int lane = threadIdx.x & 63;
    constexpr int32_t S = 64 * kU;
    const uint32_t gsh = h.gsh;
    const uint64_t B0 = h.B0, S0 = h.S0, E = h.E;
    const int32_t NCe = h.NCe;
    const int32_t cf = S0 > B0 ? 1 : 0;
    const int32_t cl = (E & 15) ? NCe - 1 : NCe;
    const int32_t nsteps = cl > cf ? (cl - cf + S - 1) / S : 0;
    EdgeChunks<kNT, kByte> Ed;
    const bool edge_part = part == nparts - 1;
    // the edge loads issued before the first steps: 1 KiB steps (configs[3]
    // enc_emit 440 -> 437 us); with 2 KiB steps the extra registers and the
    // peeled loop cost more than the drain (configs[1] 106 -> 108-109 us)
    constexpr bool kEarly = kU == 1;
    if (kEarly && edge_part) Ed.issue(T, gsh, B0, cf, cl, NCe, lane, dummy);
    if (part < nsteps) {
        ChunkPlan Pa[kU], Pb[kU];
        uint32_t Xa[kU][4], Xb[kU][4];
        uint4 La[kU], Lb[kU];
#define ONC_ISSUE(P, X, L, base)                                                          \
    _Pragma("unroll") for (int u = 0; u < kU; ++u) {                                     \
        const int32_t c_ = min((base) + lane + 64 * u, cl - 1);                           \
        P[u] = kInterior == 2 ? plan_chunk_full(T, gsh, B0, c_)                           \
             : kInterior == 1 ? plan_chunk_interior(T, gsh, B0, c_, dummy)                \
                              : plan_chunk<kByte>(T, gsh, B0, c_, dummy);                 \
        load_chunk<kNT, kByte>(P[u], X[u]);                                               \
        L[u] = T.img[P[u].slot];                                                          \
    }
#define ONC_CONSUME(P, X, L, base)                                                        \
    _Pragma("unroll") for (int u = 0; u < kU; ++u) {                                     \
        const int32_t c = min((base) + lane + 64 * u, cl - 1);                            \
        uint32_t v[4];                                                                    \
        if (kInterior == 2) merge_words_full(X[u], L[u], P[u].sel, P[u].plen, v);         \
        else if (kInterior == 1) merge_words_inplace(X[u], L[u], P[u].sel, v);            \
        else merge_chunk<kByte>(P[u], X[u], L[u], v);                                     \
        u32x4* d = reinterpret_cast<u32x4*>(a.out + B0 + (uint64_t(c) << 4));             \
        if (kNT & 2) __builtin_nontemporal_store(u32x4{v[0], v[1], v[2], v[3]}, d);        \
        else *d = u32x4{v[0], v[1], v[2], v[3]};                                          \
    }
        int32_t jj = part;
        if constexpr (kEarly) {
            ONC_ISSUE(Pa, Xa, La, cf + S * jj);
            ONC_ISSUE(Pb, Xb, Lb, cf + S * min(jj + nparts, nsteps - 1));
            if (edge_part) Ed.finish(a, T, gsh, B0, S0, E, cf, cl, NCe, lane, dummy);
            for (;;) {
                ONC_CONSUME(Pa, Xa, La, cf + S * jj);
                jj += nparts;
                if (jj >= nsteps) break;
                ONC_ISSUE(Pa, Xa, La, cf + S * min(jj + nparts, nsteps - 1));
                ONC_CONSUME(Pb, Xb, Lb, cf + S * jj);
                jj += nparts;
                if (jj >= nsteps) break;
                ONC_ISSUE(Pb, Xb, Lb, cf + S * min(jj + nparts, nsteps - 1));
            }
        } else {
            ONC_ISSUE(Pa, Xa, La, cf + S * jj);
            for (;;) {
                ONC_ISSUE(Pb, Xb, Lb, cf + S * min(jj + nparts, nsteps - 1));
                ONC_CONSUME(Pa, Xa, La, cf + S * jj);
                jj += nparts;
                if (jj >= nsteps) break;
                ONC_ISSUE(Pa, Xa, La, cf + S * min(jj + nparts, nsteps - 1));
                ONC_CONSUME(Pb, Xb, Lb, cf + S * jj);
                jj += nparts;
                if (jj >= nsteps) break;
            }
        }
#undef ONC_ISSUE
#undef ONC_CONSUME
    }
    if (edge_part && (!kEarly || part >= nsteps)) {
        if (!kEarly) Ed.issue(T, gsh, B0, cf, cl, NCe, lane, dummy);
        Ed.finish(a, T, gsh, B0, S0, E, cf, cl, NCe, lane, dummy);
    }
}

#ifndef ONC_WS_U
#define ONC_WS_U 2            // consumer chunks per lane per step (c1: 2 -> enc_emit 121 -> 116 us vs 1)
#endif
constexpr int kWsGrid = 1024;   // persistent workgroups (4 per CU on 256 CUs)
static_assert(kWsGrid / kTilesPerBlk <= 64, "a producer adds at most 64 workgroup totals per tile");

// Header-heavy batches (codec.hip picks this kernel from the declared payload
// arena, which overstates the payload when it is a decoded wire: a re-encode
// of configs[0]-shaped records measured enc_emit 99 -> 159 us): every
// workgroup samples the enc_len totals of kWsSample workgroups spread over
// the launch (enc_len's block_pay: streamed payload bytes; block_sum: all
// bytes) and, when the payload is under kWsPayPerHeader times the header
// bytes, its four waves run the wave-per-tile code instead — each wave its
// own tiles (g, g + G, ...; G = the grid's waves), placed by a running sum of
// the enc_len workgroup totals, as the producer does.
constexpr uint64_t kWsPayPerHeader = 4;     // the pipeline when payload >= 4 x header bytes
constexpr uint64_t kWsSample = 64;          // enc_len workgroups sampled, evenly spaced over the launch
union WsShared {
    struct {
        WsSlot slot[2];
        WsLane ln[64];
        WsDesc desc;
    } ws;
    ImgTile wpt[4];
};

// The rule (round 4, tools/mix_lab.py sweep, profiles/lab_r04_mix_sweep.log):
// the pipeline's single producer stages header bytes while three consumers
// stream payload, so the pipeline wins once the payload is about four times
// the header bytes — AUTH_NONE calls (44-byte headers): 128 B payloads 61 us
// wave-per-tile against 67 pipelined, 192 B 93 / 92, 256 B 119 / 106;
// AUTH_UNIX 16-gid calls (128 B): 256 B 152 / 178, 512 B 250 / 245; a quarter
// of configs[0]'s records among configs[1]'s (3.2x) 117 / 122. (Round 3's
// rule, payload >= 128 B per record, sent a half/half mix of the two to the
// pipeline: 130 us against 107.) Sampled across the whole launch, not its
// head (round 3 read the first 64 workgroups only): 64 enc_len workgroups
// spaced evenly, their byte and payload totals, one load of each per lane.
// (Summing all 1024 workgroups of a 1M-record launch in every workgroup's
// prologue cost configs[1]'s enc_emit 3.5 us.)
__device__ __forceinline__ bool ws_header_heavy(const EncArgs& a) {
    if (!a.block_pay || (a.variant & ONC_VARIANT_WS_PIPELINE)) return false;   // the pipeline on every shape (tests)
    const int lane = threadIdx.x & 63;
    const uint64_t nb = num_len_blocks(a.n);
    // every workgroup once when there are fewer than kWsSample (lane * nb /
    // kWsSample would read the head of the launch, some of it twice)
    const uint64_t b = nb >= kWsSample ? uint64_t(lane) * nb / kWsSample : uint64_t(lane);
    const bool use = uint64_t(lane) < kWsSample && (nb >= kWsSample || uint64_t(lane) < nb);
    const uint64_t pay = use ? a.block_pay[b] : 0;
    const uint64_t all = use ? a.block_sum[b] : 0;
    const uint64_t p = lane_u64(wave_incl_scan_u64(pay), 63), t = lane_u64(wave_incl_scan_u64(all), 63);
    return p < kWsPayPerHeader * (t - p);
}

template <int kU, int kNT>
__device__ __forceinline__ void ws_as_wave_per_tile(const EncArgs& a, ImgTile& T) {
    const int lane = threadIdx.x & 63;
    const uint64_t ntiles = num_emit_tiles(a.n), nb = num_len_blocks(a.n);
    const uint64_t G = uint64_t(gridDim.x) * 4;
    uint64_t run_blk = 0, run_base = launch_base(a);
    for (uint64_t tile = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); tile < ntiles; tile += G) {
        // workgroup totals [run_blk, blk): G tiles apart = G / 16 workgroups per step
        const uint64_t blk = tile / kTilesPerBlk;
        uint64_t v = 0;
        for (uint64_t b = run_blk + lane; b < blk; b += 64) v += a.block_sum[min(b, nb - 1)];
        run_base += lane_u64(wave_incl_scan_u64(v), 63);
        run_blk = blk;
        enc_emit_tile<kU, kNT, false, false, true>(a, T, tile, run_base);
    }
}

template <int kU, int kNT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void enc_emit_ws_kernel(EncArgs a) {
    __shared__ WsShared s_sh;
    WsSlot* s_slot = s_sh.ws.slot;
    WsLane* s_ln = s_sh.ws.ln;
    WsDesc& s_desc = s_sh.ws.desc;
    const int wv = threadIdx.x >> 6;
    if (ws_header_heavy(a)) {                       // wave-uniform and grid-uniform
        ws_as_wave_per_tile<1, kNT>(a, s_sh.wpt[wv]);
        return;
    }
    const uint64_t ntiles = num_emit_tiles(a.n);
    const uintptr_t dummy = reinterpret_cast<uintptr_t>(a.msgs);
    WsTile S;
    S.run_blk = 0;
    S.run_base = launch_base(a);
    uint64_t next = blockIdx.x;
    bool have = false;
    // producer: one span into slot W, or "done"
    const auto produce = [&](WsSlot& W) {
        if (!have && next < ntiles) {
            WsLoads pf = ws_issue(a, S.run_blk, next);
            asm volatile("" : "+v"(pf.mr.q[0]), "+v"(pf.mr.q[1]), "+v"(pf.mr.q[2]), "+v"(pf.mr.q[3]), "+v"(pf.tv),
                         "+v"(pf.bw));
            ws_begin_tile(a, S, s_ln, s_desc, next, pf);
            next += gridDim.x;
            have = true;
        }
        if (!have) {
            if ((threadIdx.x & 63) == 0) W.h.state = 2u;
            return;
        }
        ws_stage_span(a, S, s_ln, s_desc, W);
        if (S.lo_rec >= S.nrec) have = false;
    };
#ifdef ONC_EMIT_PROF
    uint64_t pr_t0 = wall_clock64(), pr_busy = 0, pr_phases = 0;
#endif
    if (wv == 0) produce(s_slot[0]);
    __syncthreads();
    int cur = 0;
    for (;;) {
        const uint32_t state = s_slot[cur].h.state;
        if (state == 2u) break;
#ifdef ONC_EMIT_PROF
        const uint64_t pr_a = wall_clock64();
#endif
        if (wv == 0) {
            produce(s_slot[cur ^ 1]);
        } else if (state == 1u) {
            const SpanHdr h = s_slot[cur].h;
            if (h.byte_mode) stream_span_part<1, kNT, true>(a, s_slot[cur].T, h, wv - 1, 3, dummy);
            else if (h.interior == 2 && !(a.variant & ONC_VARIANT_WS_NO_FULL))
                stream_span_part<kU, kNT, false, 2>(a, s_slot[cur].T, h, wv - 1, 3, dummy);
            else if (h.interior && !(a.variant & ONC_VARIANT_WS_NO_INTERIOR))
                stream_span_part<kU, kNT, false, 1>(a, s_slot[cur].T, h, wv - 1, 3, dummy);
            else stream_span_part<kU, kNT, false>(a, s_slot[cur].T, h, wv - 1, 3, dummy);
        }
#ifdef ONC_EMIT_PROF
        if (wv <= 1) {
            __builtin_amdgcn_s_waitcnt(0);             // the wave's own memory operations done
            pr_busy += wall_clock64() - pr_a;
            ++pr_phases;
        }
#endif
        __syncthreads();
        cur ^= 1;
    }
#ifdef ONC_EMIT_PROF
    // per workgroup: [0] lifetime, [1] producer busy, [2] phases, [4] consumer 1 busy
    if (a.prof && (threadIdx.x & 63) == 0 && wv <= 1) {
        if (wv == 0) {
            a.prof[8 * blockIdx.x + 0] = wall_clock64() - pr_t0;
            a.prof[8 * blockIdx.x + 1] = pr_busy;
            a.prof[8 * blockIdx.x + 2] = pr_phases;
        } else {
            a.prof[8 * blockIdx.x + 4] = pr_busy;
        }
    }
#endif
}

// kNT: bit 0 = nontemporal payload loads, bit 1 = nontemporal stores (header
// chunks stored temporally so that the decoder finds them cached made the
// decode slower, 60 -> 69 us on c1: the dirty lines are written back at the
// kernel boundary). The message instances need 106 VGPRs (4 waves per SIMD;
// held there by the attribute); squeezed to 5 waves per SIMD (96 VGPRs) they
// spill. The body-root instances keep what they need (140 VGPRs).
template <int kU, int kNT = 0, bool kFused = false, bool kRoot = false, bool kLen = false>
__global__ __launch_bounds__(64 * kFastWaves) __attribute__((amdgpu_waves_per_eu(kRoot ? 1 : 4))) void enc_emit_kernel_t(EncArgs a) {
    __shared__ ImgTile s_tiles[kFastWaves];
    const uint64_t tile = uint64_t(blockIdx.x) * kFastWaves + (threadIdx.x >> 6);
    if (tile < num_emit_tiles(a.n))
        enc_emit_tile<kU, kNT, kFused, kRoot, false, kLen>(a, s_tiles[threadIdx.x >> 6], tile);
}

// The one-launch small batch (codec.hip small_batch): one workgroup of
// kSpWaves tile waves is the whole batch (8 image tiles: the same 4 waves per
// SIMD as the 4-wave kernel).
__global__ __launch_bounds__(64 * kSpWaves) __attribute__((amdgpu_waves_per_eu(4))) void enc_emit_single_kernel(EncArgs a) {
    __shared__ ImgTile s_tiles[kSpWaves];
    __shared__ WgPlace<kSpWaves> s_place;
    if (threadIdx.x < kSpWaves) s_place.ready[threadIdx.x] = 0u;
    __syncthreads();
    const uint64_t tile = uint64_t(threadIdx.x >> 6);
    if (tile < num_emit_tiles(a.n))
        enc_emit_tile<kEmitChunkUnroll, kEmitNT, false, false, false, false, true, kSpWaves>(
            a, s_tiles[threadIdx.x >> 6], tile, 0, &s_place);
}

hipError_t launch_enc_len(const EncArgs& a, hipStream_t s) {
    if (a.root != ONC_ROOT_RPC_MESSAGE)
        ONC_LAUNCH(enc_len_kernel<true>, dim3(uint32_t(num_len_blocks(a.n))), dim3(kLenThreads), 0, s, a);
    else
        ONC_LAUNCH(enc_len_kernel<false>, dim3(uint32_t(num_len_blocks(a.n))), dim3(kLenThreads), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_enc_emit(const EncArgs& a, hipStream_t s) {
    if (a.ws) {
        const uint64_t tiles = num_emit_tiles(a.n);
        // (a grid trimmed to equal tiles per workgroup, 977 for configs[1],
        // measured slower: concurrency beats the ragged last phase)
        const uint32_t g = uint32_t(min(uint64_t(kWsGrid), tiles));
        // long payloads (>= 512 B on average, configs[3]) also load them
        // nontemporally: the stream does not evict the descriptors and
        // parameter blocks the producer reads (configs[3] enc_emit 442 ->
        // 423 us per 1M chunk; configs[1]-shaped batches measured no gain)
        if (a.ws == 2) ONC_LAUNCH((enc_emit_ws_kernel<1, kEmitNT | 1>), dim3(g), dim3(256), 0, s, a);
        else ONC_LAUNCH((enc_emit_ws_kernel<ONC_WS_U, kEmitNT>), dim3(g), dim3(256), 0, s, a);
        return hipGetLastError();
    }
    const uint64_t blocks = (num_emit_tiles(a.n) + kFastWaves - 1) / kFastWaves;
    if (a.root != ONC_ROOT_RPC_MESSAGE) {
        // body-level roots (onc_encode_body): the wave-per-tile kernel with
        // the root switch (codec.hip never picks the wave-specialised one)
        if (a.fused_base)
            ONC_LAUNCH((enc_emit_kernel_t<kEmitChunkUnroll, kEmitNT, true, true>), dim3(uint32_t(blocks)),
                       dim3(64 * kFastWaves), 0, s, a);
        else
            ONC_LAUNCH((enc_emit_kernel_t<kEmitChunkUnroll, kEmitNT, false, true>), dim3(uint32_t(blocks)),
                       dim3(64 * kFastWaves), 0, s, a);
        return hipGetLastError();
    }
    const dim3 g{uint32_t(blocks)}, b{uint32_t(64 * kFastWaves)};
    if (a.small) {
        if (num_emit_tiles(a.n) > uint64_t(kSpWaves)) return hipErrorInvalidValue;   // one workgroup is the batch
        ONC_LAUNCH(enc_emit_single_kernel, dim3(1), dim3(64 * kSpWaves), 0, s, a);
        return hipGetLastError();
    }
    if (a.len_in) {
        if (a.fused_base) ONC_LAUNCH((enc_emit_kernel_t<kEmitChunkUnroll, kEmitNT, true, false, true>), g, b, 0, s, a);
        else ONC_LAUNCH((enc_emit_kernel_t<kEmitChunkUnroll, kEmitNT, false, false, true>), g, b, 0, s, a);
        return hipGetLastError();
    }
    if (a.fused_base) ONC_LAUNCH((enc_emit_kernel_t<kEmitChunkUnroll, kEmitNT, true>), g, b, 0, s, a);
    else ONC_LAUNCH((enc_emit_kernel_t<kEmitChunkUnroll, kEmitNT, false>), g, b, 0, s, a);
    return hipGetLastError();
}

}  // namespace onc
