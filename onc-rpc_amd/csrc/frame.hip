// frame.hip — record framing of a byte stream on gfx950.
//
// The reference frames one message at a time: the caller runs
// expected_message_len (src/rpc_message.rs:343-367) on the remaining bytes
// and cuts a one-message slice of that length (the contract of every
// TryFrom<&[u8]>, rpc_message.rs:238-242). Record k+1's start depends on
// record k's header: a serial chain. Here it is framed in parallel by
// speculation + verification, with the same result as the serial loop:
//
//   frame_guess   wave per chunk (64 KiB by default; ONC_RPC_FRAME_CHUNK):
//                 guess the first record start in the chunk (the first
//                 position that looks like an ONC-RPC header: last-fragment
//                 bit, length within the buffer, message type 0 with
//                 rpcvers 2 or 1 with reply_stat 0/1) with a coalesced
//                 1 KiB-per-step sweep. Chunk 0 starts at byte 0.
//   frame_chunks  lane per chunk: follow the exact chain from the guess
//                 (header length only, as the reference does) out of the
//                 chunk: exit position and record count, or where and why
//                 the chain stops.
//                 Then (same lane) the check: a guessed chunk is consistent
//                 when its chain lands exactly on the guess of the chunk it
//                 lands in and every chunk it jumps over has no guess.
//                 Because chunk 0 is exact, every guessed chunk before the
//                 first inconsistency is on the true chain (induction).
//   frame_walk    one wave, only when a check failed (payload bytes that
//                 look like headers, or records that do not look like
//                 RPC messages): walks the true chain from the first
//                 failure, re-chasing chunks whose guess was wrong, skipping
//                 verified stretches with 64-wide ballots.
//   counts -> scan (len_tiles/scan_tiles/len_apply) -> frame_write: every
//                 chunk on the chain re-chases its records writing rec_off.
#include "common.h"
#include "kernels.h"

namespace onc {

constexpr uint64_t kNone = ~0ull;
constexpr int32_t kExit = -1;   // st: the chain left the chunk at x (more records follow)
// st >= 0: the chain ends in this chunk: ONC_OK (the buffer ends exactly at
// x), or the expected_message_len error / IncompleteMessage at position x.

__device__ __forceinline__ uint32_t be_at(uintptr_t base, uint64_t p) { return bswap(load4(base + p)); }

struct Chase {
    uint64_t x;
    uint32_t cnt;      // records started before leaving [p, lim)
    int32_t st;
    uint32_t aux0, aux1;
};

// The caller's loop from record start p while p < lim. The first
// kStartsCap record starts go to the sink (kept for frame_write, which then
// copies them instead of chasing again).
constexpr uint32_t kStartsCap = 64;
struct NoStarts {
    __device__ __forceinline__ void operator()(uint32_t, uint64_t) const {}
};
struct GlobalStarts {       // straight to the chunk's slice of a.starts (the walk's re-chase)
    uint64_t* rec;
    __device__ __forceinline__ void operator()(uint32_t i, uint64_t p) const {
        if (rec) rec[i] = p;
    }
};
#ifndef ONC_FRAME_CHUNKS_WG
#define ONC_FRAME_CHUNKS_WG 64   // 512 waves spread over every CU: c2 framing chase 37.0 -> 34.6 us vs 256
#endif
constexpr int kChunksWG = ONC_FRAME_CHUNKS_WG;   // lanes (chunks) per frame_chunks workgroup
struct LdsStarts {          // chunk-relative u32 in an LDS column (stride kChunksWG), copied out after the chase:
    uint32_t* col;          // a global store inside the chase would hold up the next hop's load (one vmcnt)
    uint64_t c0;
    __device__ __forceinline__ void operator()(uint32_t i, uint64_t p) const { col[i * kChunksWG] = uint32_t(p - c0); }
};
template <class Sink>
__device__ __forceinline__ Chase chase(const FrameArgs& a, uint64_t p, uint64_t lim, const Sink& rec) {
    const uintptr_t base = reinterpret_cast<uintptr_t>(a.wire);
    Chase c{p, 0, kExit, 0, 0};
    while (p < lim) {
        if (a.len - p < 4) {                       // expected_message_len: rpc_message.rs:344-346
            c.st = ONC_ERR_INCOMPLETE_HEADER;
            break;
        }
        const uint32_t h = be_at(base, p);
        if ((h & 0x80000000u) == 0) {              // :359-362
            c.st = ONC_ERR_FRAGMENTED;
            break;
        }
        const uint64_t want = uint64_t(h & 0x7FFFFFFFu) + 4;
        if (a.len - p < want) {                    // the one-message slice would be short
            c.st = ONC_ERR_INCOMPLETE_MESSAGE;
            c.aux0 = uint32_t(a.len - p);
            c.aux1 = uint32_t(want);
            break;
        }
        if (c.cnt < kStartsCap) rec(c.cnt, p);
        ++c.cnt;
        p += want;
    }
    if (c.st == kExit && p >= a.len) c.st = ONC_OK;   // the last record ends the buffer
    c.x = p;
    return c;
}

// Full plausibility test of a record start at p (p + 16 <= len).
// Beyond the record mark and message type: a call has rpcvers 2 and a
// credential length <= 200 (flavor.rs:83); a reply has reply_stat 0 with a
// verifier length <= 200, or reply_stat 1 with a rejection kind 0/1. Every
// record the reference's decoder accepts passes; the test only steers the
// guess (a record that fails it is still framed, via the walk).
template <class Be>
__device__ __forceinline__ bool plausible_with(uint64_t len, uint64_t p, const Be& be) {
    const uint32_t h = be(0);
    const uint32_t mt = be(8);
    const uint32_t rv = be(12);
    const uint64_t want = uint64_t(h & 0x7FFFFFFFu) + 4;
    if (!(h & 0x80000000u) || want < 24 || want > len - p) return false;
    if (mt == 0) return rv == 2u && want >= 44 && be(32) <= ONC_MAX_AUTH_LEN;
    if (mt != 1 || rv > 1u) return false;
    const uint32_t w4 = be(16), w5 = be(20);
    return rv == 0 ? (want >= 28 && w5 <= ONC_MAX_AUTH_LEN) : w4 <= 1u;
}

__device__ __forceinline__ bool plausible_at(const FrameArgs& a, uint64_t p) {
    const uintptr_t base = reinterpret_cast<uintptr_t>(a.wire);
    return plausible_with(a.len, p, [&](uint32_t k) { return be_at(base, p + k); });
}

// 16-bit mask of the bytes of a 16-byte block (as four dwords) that could
// start a record: high bit set (last-fragment flag of the record mark) and
// three zero bytes at +8..+10 (message type 0 or 1 as a big-endian u32).
// n = the next 16 bytes (for positions whose +8..+10 cross the block).
__device__ __forceinline__ uint32_t cand_mask16(const u32x4& v, const u32x4& n) {
    const uint32_t w[8] = {v.x, v.y, v.z, v.w, n.x, n.y, n.z, n.w};
    uint32_t hi = 0, zero = 0;                // bit k: byte k has the high bit / is zero (k < 32)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t x = w[i];
        const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);   // 0x80 in each zero byte
        const uint32_t zb = ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
        zero |= zb << (4 * i);
        if (i < 4) {
            const uint32_t h = x & 0x80808080u;
            hi |= (((h >> 7) & 1u) | ((h >> 14) & 2u) | ((h >> 21) & 4u) | ((h >> 28) & 8u)) << (4 * i);
        }
    }
    return hi & (zero >> 8) & (zero >> 9) & (zero >> 10) & 0xFFFFu;
}

// frame_guess: one wave per kGuessSub consecutive chunks (1 by default;
// chunk 0 starts at byte 0): for each, the first position in the chunk that
// looks like a record start. A coalesced sweep (lane = 16 positions, 1 KiB
// of every chunk per step) stages the step's bytes (+ 64 B of lookahead) in
// LDS; the byte-mask filter picks candidates, the full test
// (plausible_with) reads them from LDS, and only candidates that pass it
// test the start their length points to (global loads, every lane at
// once); the lowest passing position wins. A guess only steers the chase:
// correctness never depends on it. Measured on configs[2] (64 KiB chunks):
// 36 µs; the same sweep testing candidates with global loads 39 µs; four
// chunks per wave (one step loop over all four) 68 µs — a wave runs until
// its slowest chunk is found, at 142 VGPRs.
#ifndef ONC_GUESS_SUB
#define ONC_GUESS_SUB 1
#endif
constexpr int kGuessSub = ONC_GUESS_SUB;
constexpr int kGuessWin = 272;            // dwords per staged step: 1 KiB + 64 B
__global__ __launch_bounds__(256) void frame_guess_kernel(FrameArgs a) {
    __shared__ uint32_t s_win[4][kGuessSub][kGuessWin];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    {   // the verification flags of frame_chunks (set there, read by the walk)
        const uint64_t f = uint64_t(blockIdx.x) * 256 + threadIdx.x;
        if (f == 0) {
            *a.first_fail = kNone;
            *a.first_stop = kNone;
            // the call's outputs start cleared (a stream that frames nothing
            // leaves them so): in this launch instead of two fills
#pragma unroll
            for (int k = 0; k < 5; ++k) a.result[k] = 0;
            a.rec_off[0] = 0;
        }
        if (f < ((a.nchunks + 255) >> 8)) a.fail2[f] = a.stop2[f] = 0;
        if (f < ((a.nchunks + 65535) >> 16)) a.fail3[f] = a.stop3[f] = 0;
    }
    const uint64_t t0 = (uint64_t(blockIdx.x) * 4 + wv) * kGuessSub;
    if (t0 >= a.nchunks) return;
    const uintptr_t base = reinterpret_cast<uintptr_t>(a.wire);
    const uint64_t lastblk = (a.len - 1) & ~uint64_t(15);   // last 16-byte block holding a buffer byte
    uint64_t g[kGuessSub];
    uint32_t open = 0;                         // bit j: chunk t0 + j still searching
#pragma unroll
    for (int j = 0; j < kGuessSub; ++j) {
        g[j] = kNone;
        if (t0 + j == 0) g[j] = 0;
        else if (t0 + j < a.nchunks) open |= 1u << j;
    }
    for (uint64_t step = 0; open; ++step) {
        uint64_t blk[kGuessSub];
        u32x4 v[kGuessSub], tv[kGuessSub];
#pragma unroll
        for (int j = 0; j < kGuessSub; ++j) {
            const uint64_t c0 = (t0 + j) * a.chunk, c1 = min(c0 + a.chunk, a.len);
            blk[j] = (c0 & ~uint64_t(15)) + 1024 * step;
            if ((open >> j) & 1) {
                if (blk[j] >= c1) {
                    open &= ~(1u << j);        // no record start in the chunk
                } else {
                    const uint64_t o = blk[j] + 16ull * lane;
                    v[j] = gload<u32x4>(base + (o <= lastblk ? o : lastblk));
                    const uint64_t ot = blk[j] + 1024 + 16ull * (lane & 3);
                    if (lane < 4) tv[j] = gload<u32x4>(base + (ot <= lastblk ? ot : lastblk));
                }
            }
        }
        if (!open) break;
#pragma unroll
        for (int j = 0; j < kGuessSub; ++j) {
            if ((open >> j) & 1) {
                uint32_t* w = s_win[wv][j];
                w[4 * lane + 0] = v[j].x; w[4 * lane + 1] = v[j].y; w[4 * lane + 2] = v[j].z; w[4 * lane + 3] = v[j].w;
                if (lane < 4) {
                    w[256 + 4 * lane + 0] = tv[j].x; w[256 + 4 * lane + 1] = tv[j].y;
                    w[256 + 4 * lane + 2] = tv[j].z; w[256 + 4 * lane + 3] = tv[j].w;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int j = 0; j < kGuessSub; ++j) {
            if (!((open >> j) & 1)) continue;
            const uint32_t* w = s_win[wv][j];
            const uint64_t c0 = (t0 + j) * a.chunk, c1 = min(c0 + a.chunk, a.len);
            const uint64_t hi_pos = min(c1, a.len >= 16 ? a.len - 15 : 0);   // candidates p < hi_pos
            const uint64_t o = blk[j] + 16ull * lane;
            const u32x4 nx = {w[4 * lane + 4], w[4 * lane + 5], w[4 * lane + 6], w[4 * lane + 7]};
            uint32_t cand = cand_mask16(v[j], nx);
            const uint64_t lo = c0 > o ? c0 - o : 0;
            const uint64_t hi = hi_pos > o ? min(uint64_t(16), hi_pos - o) : 0;
            cand &= (hi >= 16 ? 0xFFFFu : ((1u << hi) - 1u)) & (lo >= 16 ? 0u : ~((1u << lo) - 1u));
            uint64_t mine = kNone;
            while (cand) {
                const uint32_t r = 16u * lane + __builtin_ctz(cand);   // window byte offset (< 1024)
                const uint64_t p = blk[j] + r;
                const auto be_lds = [&](uint32_t k) {
                    const uint32_t q = r + k, wi = q >> 2, sh = q & 3u;
                    return bswap(funnel(w[wi], sh ? w[wi + 1] : 0u, sh));
                };
                if (plausible_with(a.len, p, be_lds)) {
                    // and the record it claims is followed by another
                    // plausible start (or the buffer's end): rejects words
                    // inside a record that happen to look like a header
                    const uint64_t q = p + uint64_t(be_lds(0) & 0x7FFFFFFFu) + 4;
                    if (q + 16 > a.len || plausible_at(a, q)) {
                        mine = p;
                        break;
                    }
                }
                cand &= cand - 1;
            }
            const uint64_t m = __ballot(mine != kNone);
            if (m) {
                g[j] = __shfl(mine, __builtin_ctzll(m), 64);
                open &= ~(1u << j);
            }
        }
        __builtin_amdgcn_wave_barrier();       // the next step overwrites the windows
    }
#pragma unroll
    for (int j = 0; j < kGuessSub; ++j)
        if (lane == j && t0 + j < a.nchunks) a.g[t0 + j] = g[j];
}

__device__ __forceinline__ void put_chase(const FrameArgs& a, uint64_t t, const Chase& c) {
    a.x[t] = c.x;
    a.cnt[t] = c.cnt;
    a.st[t] = c.st;
    a.aux[2 * t] = c.aux0;
    a.aux[2 * t + 1] = c.aux1;
}

// frame_chunks: lane per chunk, the exact chain from the guess out of the
// chunk, then the chunk's verification: fail[t] = 1 when guessed chunk t's
// chain does not land on a guess, or jumps over a guessed chunk; stop[t] = 1
// when its chain ends in it. Both also set their per-256-chunk and
// per-65536-chunk summary flags (zeroed by frame_guess) so that the walk
// finds the next set flag in three short ballot scans; first_fail /
// first_stop = the minimum flagged chunk. (The check reads only the guesses,
// final before this launch, and the lane's own chase: one launch fewer than
// a separate verification pass.)
__global__ __launch_bounds__(kChunksWG) void frame_chunks_kernel(FrameArgs a) {
    __shared__ uint32_t s_rec[kStartsCap * kChunksWG];
    const uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= a.nchunks) return;
    const uint64_t c0 = t * a.chunk;
    const uint64_t c1 = min(c0 + a.chunk, a.len);
    const uint64_t g = a.g[t];                 // frame_guess
    uint8_t bad = 0, stop = 0;
    if (g == kNone) {
        put_chase(a, t, Chase{kNone, 0, kExit, 0, 0});
    } else {
        const Chase c = chase(a, g, c1, LdsStarts{&s_rec[threadIdx.x], c0});
        put_chase(a, t, c);
        if (c.st == kExit) {
            const uint64_t j = c.x / a.chunk;
            if (j >= a.nchunks || a.g[j] != c.x) bad = 1;
            for (uint64_t k = t + 1; k < j && !bad; ++k)
                if (a.g[k] != kNone) bad = 1;
        } else {
            stop = 1;
        }
        uint64_t* rec = a.starts + t * kStartsCap;
        for (uint32_t i = 0; i < min(c.cnt, kStartsCap); ++i) rec[i] = c0 + s_rec[i * kChunksWG + threadIdx.x];
    }
    a.fail[t] = bad;
    a.stop[t] = stop;
    if (bad) {
        a.fail2[t >> 8] = 1;
        a.fail3[t >> 16] = 1;
        atomicMin(reinterpret_cast<unsigned long long*>(a.first_fail), static_cast<unsigned long long>(t));
    }
    if (stop) {
        a.stop2[t >> 8] = 1;
        a.stop3[t >> 16] = 1;
        atomicMin(reinterpret_cast<unsigned long long*>(a.first_stop), static_cast<unsigned long long>(t));
    }
}

// First k in [t, lim) with flag[k] != 0, 64 per ballot (all lanes of the
// wave call it with the same arguments); lim if none.
__device__ __forceinline__ uint64_t wave_find(const uint8_t* flag, uint64_t t, uint64_t lim) {
    const int lane = threadIdx.x & 63;
    for (uint64_t b = t; b < lim; b += 64) {
        const uint64_t k = b + lane;
        const uint64_t m = __ballot(k < lim && flag[k] != 0);
        if (m) return b + __ffsll(static_cast<unsigned long long>(m)) - 1;
    }
    return lim;
}

// The same over a three-level flag hierarchy (chunk, 256 chunks, 65536
// chunks): at most a few short scans per level.
__device__ __forceinline__ uint64_t hier_find(const uint8_t* l1, const uint8_t* l2, const uint8_t* l3, uint64_t t,
                                              uint64_t lim) {
    if (t >= lim) return lim;
    const uint64_t e1 = min(lim, (t | 255) + 1);
    uint64_t k = wave_find(l1, t, e1);
    if (k < e1) return k;
    const uint64_t nb = (lim + 255) >> 8;
    const uint64_t b0 = (t >> 8) + 1;
    const uint64_t e2 = min(nb, ((t >> 16) + 1) << 8);
    uint64_t b = wave_find(l2, b0, e2);
    if (b >= e2) {
        const uint64_t ns = (lim + 65535) >> 16;
        const uint64_t sidx = wave_find(l3, (t >> 16) + 1, ns);
        if (sidx >= ns) return lim;
        b = wave_find(l2, sidx << 8, min(nb, (sidx + 1) << 8));
        if (b >= nb) return lim;
    }
    return wave_find(l1, b << 8, min(lim, (b + 1) << 8));
}

// One wave. No-op when every guess was verified, or when the true chain
// ends (first_stop) before the first failure. Otherwise the first failing
// chunk is on the true chain; walk from there. At a chain chunk t with true
// entry E: if g[t] == E and its check passed, the chain is verified up to
// the next failing chunk (which is then on the chain, unless the chain
// stops first); else re-chase t from E and step to the chunk its chain lands
// in, clearing the guesses of chunks the record jumps over.
__global__ __launch_bounds__(64) void frame_walk_kernel(FrameArgs a) {
    const int lane = threadIdx.x;
    const uint64_t f0 = *a.first_fail;
    if (f0 == kNone) return;
    const uint64_t s0 = *a.first_stop;
    if (s0 != kNone && s0 < f0) return;
    const uint64_t P = a.nchunks;
    uint64_t t = f0, E = a.g[f0];
#ifdef ONC_FRAME_DEBUG
    if (lane == 0) printf("frame_walk: P=%lu first_fail=%lu first_stop=%lu g=%lu x=%lu st=%d\n", (unsigned long)P,
                          (unsigned long)f0, (unsigned long)s0, (unsigned long)E, (unsigned long)a.x[f0], a.st[f0]);
    uint64_t iters = 0;
#endif
    for (;;) {
#ifdef ONC_FRAME_DEBUG
        ++iters;
#endif
        const uint64_t g = a.g[t];
        if (g == E && a.fail[t] == 0) {
            const uint64_t f2 = hier_find(a.fail, a.fail2, a.fail3, t + 1, P);
            const uint64_t s2 = hier_find(a.stop, a.stop2, a.stop3, t, f2);
            if (s2 < f2 || f2 >= P) {
                if (lane == 0) *a.first_stop = s2 < f2 ? s2 : kNone;
                break;
            }
            t = f2;
            E = a.g[f2];
            continue;
        }
        Chase c;
        if (g != E) {
            c = chase(a, E, min((t + 1) * a.chunk, a.len),
                      GlobalStarts{lane == 0 ? a.starts + t * kStartsCap : nullptr});   // same in every lane
            if (lane == 0) {
                a.g[t] = E;
                put_chase(a, t, c);
            }
            __threadfence();
        } else {
            c = Chase{a.x[t], a.cnt[t], a.st[t], a.aux[2 * t], a.aux[2 * t + 1]};
        }
        if (c.st != kExit) {
            if (lane == 0) *a.first_stop = t;
            break;
        }
        const uint64_t j = c.x / a.chunk;
        for (uint64_t k = t + 1 + lane; k < j; k += 64) a.g[k] = kNone;
        __threadfence();
        t = j;
        E = c.x;
    }
}

// Records of chunk t that belong to the framed stream, summed per block of
// kCntBlk chunks (one per thread: a 2 GB stream is only 30k chunks, so the
// grid stays wide): the counts kernel and the first level of the count scan
// in one launch. frame_write_slots then sums every chunk's first record
// index itself (the block totals before its block + the counts before it).
constexpr uint64_t kCntBlk = 256;
constexpr uint64_t kCntBlkMax = 2048;   // 512k chunks (32 GiB of stream at 64 KiB); beyond: the 3-launch scan

__device__ __forceinline__ uint32_t cnt_eff_of(const FrameArgs& a, uint64_t t, uint64_t stop) {
    return (t < a.nchunks && a.g[t] != kNone && t <= stop) ? a.cnt[t] : 0u;
}

__global__ __launch_bounds__(256) void frame_cblk_kernel(FrameArgs a, uint64_t* blk_sum) {
    __shared__ uint64_t s_wave[4];
    const uint64_t stop = *a.first_stop;
    const uint64_t t = uint64_t(blockIdx.x) * kCntBlk + threadIdx.x;
    const uint32_t ce = cnt_eff_of(a, t, stop);
    if (t < a.nchunks) a.cnt_eff[t] = ce;
    uint64_t total;
    block_excl_scan_u64<256>(ce, s_wave, &total);
    if (threadIdx.x == 0) blk_sum[blockIdx.x] = total;
}

// Records of chunk t that belong to the framed stream.
__global__ __launch_bounds__(256) void frame_counts_kernel(FrameArgs a) {
    const uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= a.nchunks) return;
    const uint64_t s = *a.first_stop;
    a.cnt_eff[t] = (a.g[t] != kNone && t <= s) ? a.cnt[t] : 0u;
}

__device__ __forceinline__ void put_result(const FrameArgs& a, uint64_t n, uint64_t consumed, int32_t st,
                                           uint32_t aux0, uint32_t aux1) {
    a.rec_off[n] = consumed;
    a.result[0] = n;
    a.result[1] = consumed;
    a.result[2] = uint64_t(int64_t(st));
    a.result[3] = aux0;
    a.result[4] = aux1;
}

// rec_off from the kept starts: a wave per chunk, lane i copies the chunk's
// record i (coalesced 8-byte stores of consecutive records); a chunk with
// more than kStartsCap records is re-chased by its lane 0 (small records).
// The chunk's first record index is the sum of the block totals before its
// block and of the counts before it in its block (frame_cblk's outputs, L2
// hits, one round trip): no separate offsets launch.
__global__ __launch_bounds__(256) void frame_write_slots_kernel(FrameArgs a, const uint64_t* blk_sum) {
    const uint64_t t = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
    const uint32_t i = threadIdx.x & 63;
    if (t >= a.nchunks) return;
    const uint64_t b = t / kCntBlk;
    const uint64_t u0 = b * kCntBlk;
    uint32_t cc[kCntBlk / 64];
#pragma unroll
    for (int q = 0; q < int(kCntBlk / 64); ++q) {
        const uint64_t u = u0 + i + 64ull * q;
        cc[q] = u < t ? a.cnt_eff[u] : 0u;
    }
    const uint32_t ce = a.cnt_eff[t];
    uint64_t s = 0;
    for (uint64_t j = i; j < b; j += 64) s += blk_sum[j];
#pragma unroll
    for (int q = 0; q < int(kCntBlk / 64); ++q) s += cc[q];
    const uint64_t k0 = lane_u64(wave_incl_scan_u64(s), 63);
    if (ce != 0 && k0 <= a.max_records) {
        const uint64_t* rec = a.starts + t * kStartsCap;
        if (ce <= kStartsCap) {
            if (i < ce) {
                const uint64_t k = k0 + i;
                const uint64_t p = rec[i];
                if (k < a.max_records) a.rec_off[k] = p;
                else if (k == a.max_records) put_result(a, k, p, ONC_OK, 0, 0);   // record max_records is not framed
            }
        } else if (i == 0) {
            const uintptr_t base = reinterpret_cast<uintptr_t>(a.wire);
            uint64_t p = a.g[t];
            for (uint32_t j = 0; j < ce; ++j) {
                const uint64_t k = k0 + j;
                if (k == a.max_records) {
                    put_result(a, k, p, ONC_OK, 0, 0);
                    break;
                }
                a.rec_off[k] = p;
                p += uint64_t(be_at(base, p) & 0x7FFFFFFFu) + 4;
            }
        }
    }
    if (i == 0 && t == *a.first_stop) {
        const uint64_t n = k0 + ce;
        // reaching max_records ends the caller's loop before it looks further
        if (n < a.max_records) put_result(a, n, a.x[t], a.st[t], a.aux[2 * t], a.aux[2 * t + 1]);
        else if (n == a.max_records) put_result(a, n, a.x[t], ONC_OK, 0, 0);
    }
}

__global__ __launch_bounds__(256) void frame_write_kernel(FrameArgs a) {
    const uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= a.nchunks) return;
    const uint32_t ce = a.cnt_eff[t];
    const uint64_t k0 = a.cnt_base[t];
    if (ce != 0 && k0 <= a.max_records) {
        const uintptr_t base = reinterpret_cast<uintptr_t>(a.wire);
        const uint64_t* rec = a.starts + t * kStartsCap;
        const bool stored = ce <= kStartsCap;        // the chase kept every start of the chunk
        uint64_t p = a.g[t];
        for (uint32_t i = 0; i < ce; ++i) {
            const uint64_t k = k0 + i;
            if (stored) p = rec[i];
            if (k == a.max_records) {
                // capacity: record max_records is not framed; stop before it
                put_result(a, k, p, ONC_OK, 0, 0);
                break;
            }
            a.rec_off[k] = p;
            if (!stored) p += uint64_t(be_at(base, p) & 0x7FFFFFFFu) + 4;
        }
    }
    if (t == *a.first_stop) {
        const uint64_t n = k0 + ce;
        // reaching max_records ends the caller's loop before it looks further
        if (n < a.max_records) put_result(a, n, a.x[t], a.st[t], a.aux[2 * t], a.aux[2 * t + 1]);
        else if (n == a.max_records) put_result(a, n, a.x[t], ONC_OK, 0, 0);
    }
}

hipError_t launch_frame_guess(const FrameArgs& a, hipStream_t s) {
    const uint64_t waves = (a.nchunks + kGuessSub - 1) / kGuessSub;
    ONC_LAUNCH(frame_guess_kernel, dim3(uint32_t((waves + 3) / 4)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_frame_chunks(const FrameArgs& a, hipStream_t s) {
    const uint32_t blocks = uint32_t((a.nchunks + kChunksWG - 1) / kChunksWG);
    ONC_LAUNCH(frame_chunks_kernel, dim3(blocks), dim3(kChunksWG), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_frame_walk(const FrameArgs& a, hipStream_t s) {
    ONC_LAUNCH(frame_walk_kernel, dim3(1), dim3(64), 0, s, a);
    return hipGetLastError();
}

bool frame_fused_scan_ok(uint64_t nchunks) { return (nchunks + kCntBlk - 1) / kCntBlk <= kCntBlkMax; }

hipError_t launch_frame_cblk(const FrameArgs& a, uint64_t* blk_sum, hipStream_t s) {
    ONC_LAUNCH(frame_cblk_kernel, dim3(uint32_t((a.nchunks + kCntBlk - 1) / kCntBlk)), dim3(256), 0, s, a,
                       blk_sum);
    return hipGetLastError();
}

hipError_t launch_frame_write_slots(const FrameArgs& a, const uint64_t* blk_sum, hipStream_t s) {
    ONC_LAUNCH(frame_write_slots_kernel, dim3(uint32_t((a.nchunks + 3) / 4)), dim3(256), 0, s, a, blk_sum);
    return hipGetLastError();
}

hipError_t launch_frame_counts(const FrameArgs& a, hipStream_t s) {
    const uint32_t blocks = uint32_t((a.nchunks + 255) / 256);
    ONC_LAUNCH(frame_counts_kernel, dim3(blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_frame_write(const FrameArgs& a, hipStream_t s) {
    const uint32_t blocks = uint32_t((a.nchunks + 255) / 256);
    ONC_LAUNCH(frame_write_kernel, dim3(blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace onc
