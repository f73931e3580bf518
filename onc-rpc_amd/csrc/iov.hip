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
//   iov_len   lane per record: plan_record(); per-64-record tile totals of
//             (wire bytes << 16 | header bytes), per-256-record totals of
//             each.
//   scan x2   workgroup bases of wire bytes and of header bytes.
//   iov_emit  wave per tile: wavefront scan places the records; header
//             words staged in LDS, then copied to hdr_out with coalesced
//             dword stores (the tile's headers are contiguous); one 32-byte
//             iovec entry per record.
#include "common.h"
#include "kernels.h"

namespace onc {

__global__ __launch_bounds__(kTile) void iov_len_kernel(IovArgs a) {
    __shared__ uint64_t s_len[kTile / 64], s_hdr[kTile / 64];
    const uint64_t r = uint64_t(blockIdx.x) * kTile + threadIdx.x;
    uint64_t len = 0, hl = 0;
    if (r < a.n) {
        const onc_msg d = a.msgs[r];
        const RecPlan p = plan_record(d, a.unix, a.bounds);
        len = p.len;
        hl = p.len ? 4ull * meta_hw(p.meta) : 0;
        a.status[r] = p.status;
    }
    // header bytes of 64 records < 2^15, so (len << 16 | hl) scans as one u64
    const uint64_t incl = wave_incl_scan_u64((len << 16) | hl);
    const uint64_t tile = r / kEmitRecs;
    if ((threadIdx.x & 63) == 63) {
        if (tile * kEmitRecs < a.n) a.tile_sum[tile] = incl;
        s_len[threadIdx.x >> 6] = incl >> 16;
        s_hdr[threadIdx.x >> 6] = incl & 0xFFFFu;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        a.block_len[blockIdx.x] = s_len[0] + s_len[1] + s_len[2] + s_len[3];
        a.block_hdr[blockIdx.x] = s_hdr[0] + s_hdr[1] + s_hdr[2] + s_hdr[3];
    }
}

constexpr int kIovHdrCap = 2048;   // header words staged per wave tile
constexpr int kIovWaves = 4;

__global__ __launch_bounds__(64 * kIovWaves) void iov_emit_kernel(IovArgs a) {
    __shared__ uint32_t s_hdr[kIovWaves][kIovHdrCap];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const uint64_t tile = uint64_t(blockIdx.x) * kIovWaves + wv;
    const uint64_t r0 = tile * kEmitRecs;
    if (r0 >= a.n) return;
    // tile bases: workgroup bases + the totals of the preceding tiles there
    const uint64_t blk = tile / (kTile / kEmitRecs);
    uint64_t W0 = a.block_len_base[blk], H0 = a.block_hdr_base[blk];
    for (uint64_t t = blk * (kTile / kEmitRecs); t < tile; ++t) {
        const uint64_t ts = a.tile_sum[t];
        W0 += ts >> 16;
        H0 += ts & 0xFFFFu;
    }
    const int nrec = int(min(uint64_t(kEmitRecs), a.n - r0));
    uint32_t* hdr = s_hdr[wv];

    onc_msg d;
    uint64_t len = 0, hl = 0;
    if (lane < nrec) {
        d = a.msgs[r0 + lane];
        const RecPlan p = plan_record(d, a.unix, a.bounds);
        len = p.len;
        hl = p.len ? 4ull * meta_hw(p.meta) : 0;
    }
    const uint64_t sv = (len << 16) | hl;
    const uint64_t incl = wave_incl_scan_u64(sv);
    const uint64_t excl = incl - sv;
    const uint64_t wire_off = W0 + (excl >> 16);
    const uint64_t hoff = H0 + (excl & 0xFFFFu);        // byte offset in hdr_out
    const uint64_t last = lane_u64(incl, nrec - 1);
    const uint64_t Ht = last & 0xFFFFu;                  // header bytes of the tile
    const bool fits = hoff + hl <= a.hdr_cap;
    if (lane < nrec) {
        const bool ok = len != 0 && fits;
        if (len != 0 && !fits) a.status[r0 + lane] = ONC_ENC_WRITE_ZERO;
        uint4* e = reinterpret_cast<uint4*>(a.iov + r0 + lane);
        const uint64_t po = ok ? d.payload_off : 0;
        const uint32_t pl = ok ? uint32_t(len - hl) : 0u;
        e[0] = make_uint4(uint32_t(hoff), uint32_t(hoff >> 32), uint32_t(po), uint32_t(po >> 32));
        e[1] = make_uint4(uint32_t(wire_off), uint32_t(wire_off >> 32), ok ? uint32_t(hl) : 0u, pl);
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
    uint32_t* out = reinterpret_cast<uint32_t*>(a.hdr_out + H0);   // H0 is a multiple of 4
    if (Ht <= 4ull * kIovHdrCap) {
        if (lane < nrec && hl != 0) {
            WordSink w{hdr + ((hoff - H0) >> 2)};
            put_header_words(d, uint32_t(len), src, w);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t nw = uint32_t((cut - H0) >> 2);
        for (uint32_t k = lane; k < nw; k += 64) out[k] = hdr[k];
    } else if (lane < nrec && hl != 0 && fits) {
        // headers beyond the LDS budget (auth bodies near 200 bytes): each
        // record writes its own words
        WordSink w{out + ((hoff - H0) >> 2)};
        put_header_words(d, uint32_t(len), src, w);
    }
}

hipError_t launch_iov_len(const IovArgs& a, hipStream_t s) {
    ONC_LAUNCH(iov_len_kernel, dim3(uint32_t(num_tiles(a.n))), dim3(kTile), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_iov_emit(const IovArgs& a, hipStream_t s) {
    const uint64_t blocks = (num_emit_tiles(a.n) + kIovWaves - 1) / kIovWaves;
    ONC_LAUNCH(iov_emit_kernel, dim3(uint32_t(blocks)), dim3(64 * kIovWaves), 0, s, a);
    return hipGetLastError();
}

}  // namespace onc
