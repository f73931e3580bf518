// iov.hip — vectored batch encode for gfx950.
//
// The reference writes every record, payload included, through
// `W: Write` (RpcMessage::serialise_into, src/rpc_message.rs:136-164;
// CallBody's payload write_all, call_body.rs:107) and lists a zero-copy
// writer as future work (README.md:71-75, TODO rpc_message.rs:19). Here
// only the header part of each record (all of it but the raw payload, which
// is always last) is serialised, packed back to back; each record gets an
// iovec entry {header slice, payload slice in place, wire offset}. For the
// configs[1] record that is 44 of 300 bytes.
//
//   iov_len   1024-record workgroups, 2 records per lane (both descriptors'
//             loads issued first): plan_record(); per-64-record tile totals
//             of (wire bytes << 16 | header bytes), per-workgroup totals of
//             each.
//   [scan x2] workgroup bases of wire and of header bytes — only above
//             kFusedBlocks workgroups (1M records); below, iov_emit sums the
//             workgroup totals itself.
//   iov_emit  4 waves per workgroup, wave per 64-record tile: the
//             workgroup's base (its 4 tiles share one iov_len workgroup) is
//             summed by the 4 waves together, issued with each wave's tile
//             totals and descriptors (one round trip); a wavefront scan
//             places the records; header words staged in LDS (padded: one
//             word per 32, so lanes writing 32-word headers hit distinct
//             banks), then written to hdr_out as 16-byte nontemporal stores
//             (the tile's headers are contiguous) with dword edges; one
//             32-byte iovec entry per record, nontemporal.
#include "common.h"
#include "kernels.h"

namespace onc {

constexpr int kIovLenPer = 2;
constexpr int kIovLenThreads = kLenRecs / kIovLenPer;
constexpr uint64_t kIovTilesPerBlk = kLenRecs / kEmitRecs;   // 16

__global__ __launch_bounds__(kIovLenThreads) void iov_len_kernel(IovArgs a) {
    __shared__ uint64_t s_len[kIovLenThreads / 64], s_hdr[kIovLenThreads / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t rw = uint64_t(blockIdx.x) * kLenRecs + uint64_t(wv) * (64 * kIovLenPer);
    MsgRegs mr[kIovLenPer];
#pragma unroll
    for (int k = 0; k < kIovLenPer; ++k) {
        const uint64_t r = rw + 64 * k + lane;
        mr[k] = issue_msg(a.msgs + (r < a.n ? r : a.n - 1));
    }
    asm volatile("" : "+v"(mr[0].q[0]), "+v"(mr[0].q[1]), "+v"(mr[0].q[2]), "+v"(mr[0].q[3]), "+v"(mr[1].q[0]),
                 "+v"(mr[1].q[1]), "+v"(mr[1].q[2]), "+v"(mr[1].q[3]));
    uint64_t wl = 0, wh = 0;
#pragma unroll
    for (int k = 0; k < kIovLenPer; ++k) {
        const uint64_t r = rw + 64 * k + lane;
        uint64_t len = 0, hl = 0;
        if (r < a.n) {
            // the extent onc_encode gives the record (declared AUTH_UNIX
            // lengths) and its header bytes — a record failing only a
            // deferred block check keeps both, its header a placeholder
            // (include/onc_rpc.h onc_auth) — with the status of every check
            const onc_msg d = as_msg(mr[k]);
            const RecPlan p = plan_record<true>(d, a.unix, a.bounds);
            const RecPlan f = plan_record<false>(d, a.unix, a.bounds);
            len = p.status == ONC_OK ? p.len : 0;
            hl = p.status == ONC_OK ? 4ull * meta_hw(p.meta) : 0;
            a.status[r] = f.status;
        }
        // header bytes of 64 records < 2^15, so (len << 16 | hl) scans as one u64
        const uint64_t incl = wave_incl_scan_u64((len << 16) | hl);
        const uint64_t tile = (rw + 64 * k) / kEmitRecs;
        if (lane == 63 && tile * kEmitRecs < a.n) a.tile_sum[tile] = incl;
        const uint64_t t = lane_u64(incl, 63);
        wl += t >> 16;
        wh += t & 0xFFFFu;
    }
    if (lane == 0) {
        s_len[wv] = wl;
        s_hdr[wv] = wh;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint64_t vl = threadIdx.x < kIovLenThreads / 64 ? s_len[threadIdx.x] : 0;
        const uint64_t vh = threadIdx.x < kIovLenThreads / 64 ? s_hdr[threadIdx.x] : 0;
        const uint64_t tl = lane_u64(wave_incl_scan_u64(vl), 63);
        const uint64_t th = lane_u64(wave_incl_scan_u64(vh), 63);
        if (threadIdx.x == 0) {
            a.block_len[blockIdx.x] = tl;
            a.block_hdr[blockIdx.x] = th;
        }
    }
}

constexpr int kIovHdrCap = 2048;                       // header words staged per wave tile
constexpr int kIovHdrPad = kIovHdrCap + kIovHdrCap / 32;
constexpr int kIovWaves = 4;
static_assert(kIovTilesPerBlk % kIovWaves == 0, "a workgroup's tiles share one iov_len workgroup");
static_assert(kFusedBlocks == 16 * 64, "fused bases: 4 waves x 4 loads per lane per array");

__device__ __forceinline__ uint32_t pad_word(uint32_t w) { return w + (w >> 5); }

// Header words into the padded LDS staging buffer.
struct PadSink {
    uint32_t* base;
    uint32_t w;
    __device__ __forceinline__ void operator()(uint32_t x) {
        base[pad_word(w)] = x;
        ++w;
    }
};

template <bool kFused>
__global__ __launch_bounds__(64 * kIovWaves) void iov_emit_kernel(IovArgs a) {
    __shared__ uint32_t s_hdr[kIovWaves][kIovHdrPad];
    __shared__ uint64_t s_base[2][kIovWaves];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const uint64_t tile = uint64_t(blockIdx.x) * kIovWaves + wv;
    const uint64_t r0 = tile * kEmitRecs;
    const bool live = r0 < a.n;
    const uint64_t blk = uint64_t(blockIdx.x) * kIovWaves / kIovTilesPerBlk;
    const uint64_t t0 = blk * kIovTilesPerBlk;
    // One round trip: the workgroup-base share of this wave, the totals of
    // the tiles before this one in its iov_len workgroup, the descriptor.
    uint64_t bl[4], bh[4];
    if constexpr (kFused) {
        const uint64_t nb = (a.n + kLenRecs - 1) / kLenRecs;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t j = uint64_t(lane) + 64ull * (4 * q + wv);
            bl[q] = a.block_len[j < nb ? j : nb - 1];
            bh[q] = a.block_hdr[j < nb ? j : nb - 1];
        }
    } else {
        bl[0] = a.block_len_base[blk];
        bh[0] = a.block_hdr_base[blk];
#pragma unroll
        for (int q = 1; q < 4; ++q) bl[q] = bh[q] = 0;
    }
    uint64_t tsum = a.tile_sum[t0 + (uint64_t(lane) < kIovTilesPerBlk ? lane : 0)];
    const int nrec = live ? int(min(uint64_t(kEmitRecs), a.n - r0)) : 1;
    MsgRegs mr = issue_msg(a.msgs + (live ? r0 + min(lane, nrec - 1) : 0));
    int32_t st0 = a.status[live ? r0 + min(lane, nrec - 1) : 0];      // iov_len's status
    asm volatile("" : "+v"(mr.q[0]), "+v"(mr.q[1]), "+v"(mr.q[2]), "+v"(mr.q[3]), "+v"(bl[0]), "+v"(bl[1]),
                 "+v"(bl[2]), "+v"(bl[3]), "+v"(bh[0]), "+v"(bh[1]), "+v"(bh[2]), "+v"(bh[3]), "+v"(tsum), "+v"(st0));
    if constexpr (kFused) {
        uint64_t vl = 0, vh = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t j = uint64_t(lane) + 64ull * (4 * q + wv);
            vl += j < blk ? bl[q] : 0;
            vh += j < blk ? bh[q] : 0;
        }
        vl = lane_u64(wave_incl_scan_u64(vl), 63);
        vh = lane_u64(wave_incl_scan_u64(vh), 63);
        if (lane == 0) {
            s_base[0][wv] = vl;
            s_base[1][wv] = vh;
        }
    }
    __syncthreads();                                   // every wave reaches it (no early return above)
    if (!live) return;
    uint64_t W0, H0;
    {
        uint64_t bw = 0, bhh = 0;
        if constexpr (kFused) {
#pragma unroll
            for (int k = 0; k < kIovWaves; ++k) {
                bw += s_base[0][k];
                bhh += s_base[1][k];
            }
        } else {
            bw = bl[0];
            bhh = bh[0];
        }
        // the tiles before this one in its iov_len workgroup (lanes < 16)
        const bool before = t0 + lane < tile;
        W0 = bw + lane_u64(wave_incl_scan_u64(before ? tsum >> 16 : 0), 63);
        H0 = bhh + lane_u64(wave_incl_scan_u64(before ? tsum & 0xFFFFu : 0), 63);
    }
    uint32_t* hdr = s_hdr[wv];
    const onc_msg d = as_msg(mr);
    uint64_t len = 0, hl = 0;
    bool rec_ok = false;
    if (lane < nrec) {
        // as iov_len: the extent and header bytes from the declared lengths
        // (a record failing only a deferred block check, iov_len's status
        // != OK, keeps both: its header is the placeholder onc_encode writes)
        const RecPlan p = plan_record<true>(d, a.unix, a.bounds);
        len = p.status == ONC_OK ? p.len : 0;
        rec_ok = len != 0;
        hl = rec_ok ? 4ull * meta_hw(p.meta) : 0;
    }
    const bool hole = rec_ok && st0 != ONC_OK;
    const uint64_t sv = (len << 16) | hl;
    const uint64_t incl = wave_incl_scan_u64(sv);
    const uint64_t excl = incl - sv;
    const uint64_t wire_off = W0 + (excl >> 16);
    const uint64_t hoff = H0 + (excl & 0xFFFFu);        // byte offset in hdr_out
    const uint64_t last = lane_u64(incl, nrec - 1);
    const uint64_t Ht = last & 0xFFFFu;                  // header bytes of the tile
    const bool fits = hoff + hl <= a.hdr_cap;
    if (lane < nrec) {
        const bool ok = rec_ok && fits;
        if (rec_ok && !hole && !fits) a.status[r0 + lane] = ONC_ENC_WRITE_ZERO;
        u32x4* e = reinterpret_cast<u32x4*>(a.iov + r0 + lane);
        const uint64_t po = ok ? d.payload_off : 0;
        const uint32_t pl = ok ? uint32_t(len - hl) : 0u;
        __builtin_nontemporal_store(u32x4{uint32_t(hoff), uint32_t(hoff >> 32), uint32_t(po), uint32_t(po >> 32)}, e);
        __builtin_nontemporal_store(u32x4{uint32_t(wire_off), uint32_t(wire_off >> 32), ok ? uint32_t(hl) : 0u, pl},
                                    e + 1);
    }
    if (lane == nrec - 1 && r0 + nrec == a.n && a.totals) {
        a.totals[0] = H0 + Ht;
        a.totals[1] = W0 + (last >> 16);
    }
    // Header bytes written: the prefix of the tile's headers whose records
    // end within hdr_cap (header ends increase with the record index).
    uint64_t cut = (lane < nrec && fits) ? hoff + hl : 0;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) cut = max(cut, uint64_t(__shfl_xor(cut, o, 64)));
    if (cut <= H0) return;
    const EncSrc src{a.unix, reinterpret_cast<uintptr_t>(a.auth_arena), reinterpret_cast<uintptr_t>(a.payload_arena)};
    uint8_t* ob = a.hdr_out + H0;                      // H0 is a multiple of 4
    if (Ht <= 4ull * kIovHdrCap) {
        if (lane < nrec && hl != 0) {
            PadSink w{hdr, uint32_t((hoff - H0) >> 2)};
            if (hole) put_placeholder_words(uint32_t(len), uint32_t(hl >> 2), w);
            else put_header_words(d, uint32_t(len), src, w);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t nw = uint32_t((cut - H0) >> 2);
        // dwords up to the first 16-byte boundary, 16-byte stores, dwords after
        const uint32_t p0 = min(nw, uint32_t(((16u - (reinterpret_cast<uintptr_t>(ob) & 15u)) & 15u) >> 2));
        const uint32_t nq = (nw - p0) >> 2;
        uint32_t* o32 = reinterpret_cast<uint32_t*>(ob);
        if (uint32_t(lane) < p0) o32[lane] = hdr[pad_word(lane)];
        for (uint32_t q = lane; q < nq; q += 64) {
            const uint32_t k = p0 + 4 * q;
            const u32x4 v{hdr[pad_word(k)], hdr[pad_word(k + 1)], hdr[pad_word(k + 2)], hdr[pad_word(k + 3)]};
            __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(o32 + k));
        }
        const uint32_t kt = p0 + 4 * nq + lane;
        if (kt < nw) o32[kt] = hdr[pad_word(kt)];
    } else if (lane < nrec && hl != 0 && fits) {
        // headers beyond the LDS budget (auth bodies near 200 bytes): each
        // record writes its own words
        WordSink w{reinterpret_cast<uint32_t*>(ob) + ((hoff - H0) >> 2)};
        if (hole) put_placeholder_words(uint32_t(len), uint32_t(hl >> 2), w);
        else put_header_words(d, uint32_t(len), src, w);
    }
}

hipError_t launch_iov_len(const IovArgs& a, hipStream_t s) {
    ONC_LAUNCH(iov_len_kernel, dim3(uint32_t(num_len_blocks(a.n))), dim3(kIovLenThreads), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_iov_emit(const IovArgs& a, hipStream_t s) {
    const uint64_t blocks = (num_emit_tiles(a.n) + kIovWaves - 1) / kIovWaves;
    if (num_len_blocks(a.n) <= kFusedBlocks)
        ONC_LAUNCH(iov_emit_kernel<true>, dim3(uint32_t(blocks)), dim3(64 * kIovWaves), 0, s, a);
    else
        ONC_LAUNCH(iov_emit_kernel<false>, dim3(uint32_t(blocks)), dim3(64 * kIovWaves), 0, s, a);
    return hipGetLastError();
}

}  // namespace onc
