// kernels.h — host-side launchers of the gfx950 kernels (internal to the
// shared library; the public surface is include/onc_rpc.h).
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/onc_rpc.h"
#include "common.h"

namespace onc {

// Per-kernel timing (onc_codec_enable_timing): codec.hip's run() hands the
// start/stop events to the next launch, which then goes through
// hipExtLaunchKernelGGL — the events take the dispatch packet's own
// timestamps instead of marker packets recorded around it (each marker
// pair serialised the stream: ~7 us per timed launch on gfx950).
struct LaunchEvents {
    hipEvent_t start, stop;
};
extern thread_local LaunchEvents t_launch_events;
inline LaunchEvents take_launch_events() {
    const LaunchEvents e = t_launch_events;
    t_launch_events = LaunchEvents{nullptr, nullptr};
    return e;
}
#define ONC_LAUNCH(K, G, B, L, S, ...)                                                               \
    do {                                                                                             \
        const ::onc::LaunchEvents ev_ = ::onc::take_launch_events();                                 \
        if (ev_.start)                                                                               \
            hipExtLaunchKernelGGL(K, G, B, L, S, ev_.start, ev_.stop, 0, __VA_ARGS__);               \
        else                                                                                         \
            hipLaunchKernelGGL(K, G, B, L, S, __VA_ARGS__);                                          \
    } while (0)

struct EncArgs {
    uint64_t n;
    const onc_msg* msgs;
    const onc_unix_params* unix;
    const uint8_t* auth_arena;
    const uint8_t* payload_arena;
    Bounds bounds;          // arena sizes (onc_batch)
    uint8_t* out;           // 16-byte aligned base of the output chunks
    uint64_t origin;        // byte offset of the caller's `out` from `out` here (0..15)
    uint64_t out_cap;       // origin + the caller's capacity
    uint64_t* rec_off;      // n + 1
    int32_t* status;        // n
    uint32_t* rec_len;      // n, optional
    uint32_t* len_out;      // enc_len: optional codec-owned copy of the lengths (what the emit reads back)
    uint64_t* tile_sum;     // tiles
    uint64_t* block_sum;    // enc_len workgroups (kLenRecs records): byte totals
    uint64_t* block_base;   // exclusive scan of block_sum (unused when fused_base)
    uint64_t* block_pay;    // optional: enc_len workgroups' streamed payload bytes (the wave-specialised
                            // enc_emit's header-heavy test); NULL = not computed
    uint32_t fused_base;    // enc_emit sums block_sum itself (<= kFusedBlocks workgroups; no scan launch)
    uint32_t variant;       // ONC_VARIANT_* bits (onc_codec_options; A/B experiments, tests)
    uint32_t ws;            // enc_emit: the wave-specialised kernel (codec.hip enc_args decides)
    uint32_t root;          // ONC_ROOT_* (onc_encode_body); ONC_ROOT_RPC_MESSAGE for onc_encode
    uint32_t decl;          // enc_len, RpcMessage root: 1 = an emit's plan (declared AUTH_UNIX lengths taken
                            // as given, the emit runs the deferred parameter-block checks); 2 = onc_encode_lengths
                            // (the same extents, every check up front for the statuses); 0 = every check (roots)
    const uint64_t* base_dev;   // optional: output bytes before this launch's first record (chunked encode)
    const uint32_t* len_in;     // optional (wave-per-tile enc_emit): the plan's record lengths, read instead
                                // of re-planning (no dependent AUTH_UNIX parameter load in the prologue)
    uint32_t small;             // the one-launch small batch (enc_emit_single_kernel: one workgroup, the
                                // tiles planned and placed inside it; <= kSpWaves tiles)
#ifdef ONC_EMIT_PROF
    uint64_t* prof;         // lab builds only (tools/emit_prof.hip): per-tile phase timestamps
#endif
};

// Batches of at most this many enc_len workgroups (1M records) skip the
// scan launch: every enc_emit wave sums the block totals before its own
// (16 coalesced u64 loads per lane, issued with its tile-total load).
constexpr uint64_t kFusedBlocks = 1024;

struct IovArgs {
    uint64_t n;
    // (extents follow the declared AUTH_UNIX lengths as onc_encode places them; a record failing only a
    // deferred block check takes its extent with the placeholder header, include/onc_rpc.h onc_auth)
    const onc_msg* msgs;
    const onc_unix_params* unix;
    const uint8_t* auth_arena;
    const uint8_t* payload_arena;
    Bounds bounds;
    uint8_t* hdr_out;
    uint64_t hdr_cap;
    onc_iov_rec* iov;
    int32_t* status;
    uint64_t* totals;          // optional [2]
    uint64_t* tile_sum;        // per 64 records: (wire bytes << 16) | header bytes
    uint64_t* block_len;       // per iov_len workgroup (kLenRecs records)
    uint64_t* block_hdr;
    uint64_t* block_len_base;  // exclusive scans
    uint64_t* block_hdr_base;
};

constexpr uint64_t kFrameChunkDefault = 65536;  // stream bytes per framing lane (FrameArgs::chunk)

struct FrameArgs {
    const uint8_t* wire;
    uint64_t len;
    uint64_t chunk;         // stream bytes per framing lane
    uint64_t nchunks;
    uint64_t max_records;
    uint64_t* rec_off;      // max_records + 1
    uint64_t* starts;       // per chunk: its first record starts (frame.hip kStartsCap)
    uint64_t* result;       // [5] n, consumed, status, aux0, aux1
    // per chunk
    uint64_t* g;            // guessed / verified first record start (~0 = none)
    uint64_t* x;            // exit or stop position of the chain
    uint32_t* cnt;          // records started in the chunk
    int32_t* st;            // -1 = left the chunk, else the stop status
    uint32_t* aux;          // 2 per chunk
    uint8_t* fail;          // chunk's check failed
    uint8_t* stop;          // chunk's chain ends in it
    uint8_t* fail2;         // per 256 chunks
    uint8_t* stop2;
    uint8_t* fail3;         // per 65536 chunks
    uint8_t* stop3;
    uint32_t* cnt_eff;      // records framed from this chunk
    uint64_t* cnt_base;     // exclusive scan of cnt_eff
    uint64_t* first_fail;
    uint64_t* first_stop;
};

struct DecArgs {
    uint64_t n;
    const uint8_t* wire;
    const uint64_t* rec_off;
    onc_decoded out;
    uint32_t variant;       // ONC_VARIANT_* bits (onc_codec_options)
    // onc_decode_lengths: offsets from the lengths inside the decode
    const uint32_t* rec_len;
    const uint64_t* tile_sum;   // per decode workgroup (kDecTile records): byte total
    const uint64_t* blk_sum;    // per 4096 records: byte total (summed in the kernel) ...
    const uint64_t* blk_base;   // ... or their exclusive scan (beyond kDecLenFusedBlocks blocks)
    uint64_t nblk;
    uint64_t base;              // offset of record 0
    uint64_t* rec_off_out;      // optional: the offsets (n + 1)
    // onc_decode_body
    uint32_t body;              // 1: the root kernel (decode_kernel<..., kRoot>)
    uint32_t root;              // ONC_ROOT_*; ONC_ROOT_RPC_MESSAGE = the product decode
    const uint32_t* param;      // per record: expected_len / max_len (or NULL)
    uint32_t* consumed;         // optional: bytes the decoded value occupies
    uint32_t* hint;             // the codec's policy word (mapped host memory; decode.hip kLine) or NULL
    uint32_t line;              // message decode: the line policy (decode.hip kLine)
};
// the line policy when at least this many of a sampled workgroup's 64
// records needed a second first-round window under the standard one
constexpr uint32_t kLine1Min = 24;
constexpr uint64_t kDecLenBlk = 4096;          // records per length block
constexpr uint64_t kDecLenFusedBlocks = 512;   // up to 2M records: block totals summed in the decode

// encode.hip
hipError_t launch_enc_len(const EncArgs& a, hipStream_t s);
hipError_t launch_enc_emit(const EncArgs& a, hipStream_t s);
// iov.hip
hipError_t launch_iov_len(const IovArgs& a, hipStream_t s);
hipError_t launch_iov_emit(const IovArgs& a, hipStream_t s);
// frame.hip
hipError_t launch_frame_walk(const FrameArgs& a, hipStream_t s);
hipError_t launch_frame_counts(const FrameArgs& a, hipStream_t s);
hipError_t launch_frame_guess(const FrameArgs& a, hipStream_t s);
hipError_t launch_frame_chunks(const FrameArgs& a, hipStream_t s);
hipError_t launch_frame_write(const FrameArgs& a, hipStream_t s);
bool frame_fused_scan_ok(uint64_t nchunks);
hipError_t launch_frame_cblk(const FrameArgs& a, uint64_t* blk_sum, hipStream_t s);
hipError_t launch_frame_write_slots(const FrameArgs& a, const uint64_t* blk_sum, hipStream_t s);
// scan.hip
hipError_t launch_scan_tiles(const uint64_t* in, uint64_t* out_excl, uint64_t count, uint64_t base,
                             uint64_t* total_out, hipStream_t s);
hipError_t launch_len_tiles(const uint32_t* len, uint64_t n, uint64_t* tile_sum, hipStream_t s);
hipError_t launch_len_apply(const uint32_t* len, uint64_t n, const uint64_t* tile_base, uint64_t* rec_off,
                            hipStream_t s);
bool scan_lengths_fused_ok(uint64_t n);
hipError_t launch_store_u64(uint64_t* p, uint64_t v, hipStream_t s);
hipError_t launch_lenblk(const uint32_t* len, uint64_t n, uint64_t* blk_sum, hipStream_t s);
hipError_t launch_lenoff(const uint32_t* len, uint64_t n, const uint64_t* blk_sum, uint64_t base, uint64_t* rec_off,
                         hipStream_t s);
// compact.hip
hipError_t launch_compact_lens(const uint64_t* rec_off, const int32_t* status, uint64_t n, uint32_t* lens,
                               uint64_t* first_drop, hipStream_t s);
hipError_t launch_compact_info(const uint64_t* rec_off, const uint64_t* new_off, uint64_t n,
                               const uint64_t* first_drop, uint64_t* info, hipStream_t s);
hipError_t launch_compact_gather(const uint8_t* out, const uint64_t* rec_off, const uint64_t* new_off, uint64_t fb,
                                 uint64_t n, uint64_t base, uint64_t lo, uint8_t* scratch, hipStream_t s);
hipError_t launch_compact_offsets(uint64_t* rec_off, const uint64_t* new_off, uint64_t fb, uint64_t n, uint64_t base,
                                  hipStream_t s);
hipError_t launch_compact_iov_lens(const onc_iov_rec* iov, const int32_t* status, uint64_t n, uint32_t* lens,
                                   hipStream_t s);
hipError_t launch_compact_iov_apply(onc_iov_rec* iov, const int32_t* status, uint64_t n, const uint64_t* new_off,
                                    uint64_t* totals, hipStream_t s);
// decode.hip
hipError_t launch_decode(const DecArgs& a, int mode, hipStream_t s);
hipError_t launch_dlen_tiles(const uint32_t* rec_len, uint64_t n, uint64_t* tile_sum, uint64_t* blk_sum, hipStream_t s);

__host__ __device__ inline uint64_t num_tiles(uint64_t n) { return (n + 255) / 256; }
__host__ __device__ inline uint64_t num_len_blocks(uint64_t n) { return (n + kLenRecs - 1) / kLenRecs; }
__host__ __device__ inline uint64_t num_emit_tiles(uint64_t n) { return (n + kEmitRecs - 1) / kEmitRecs; }
// enc_emit_single_kernel: tiles (waves) of its one workgroup — the largest
// one-launch small-batch encode is kSpWaves * kEmitRecs records
#ifndef ONC_SP_WAVES
#define ONC_SP_WAVES 8
#endif
constexpr int kSpWaves = ONC_SP_WAVES;

}  // namespace onc
