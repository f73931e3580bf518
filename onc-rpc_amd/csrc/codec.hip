// codec.hip — the C ABI (include/onc_rpc.h) over the gfx950 kernels.
//
// A codec handle = one device + one HIP stream + scan scratch. Every call
// only enqueues work on the handle's stream; no host<->device copies and no
// synchronisation happen inside encode/decode (the caller syncs).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <map>
#include <string>
#include <vector>

#include "kernels.h"

struct onc_codec {
    int device = 0;
    hipStream_t stream = nullptr;
    // scratch (u64 words): [tile_sum | tile_base | block_sum | block_base]
    uint64_t* scratch = nullptr;
    uint64_t scratch_tiles = 0;
    uint8_t* frame_scratch = nullptr;   // onc_frame_stream per-chunk state
    // decode first-round policy (decode.hip kLine): a sampled workgroup's
    // count of records that needed a second round, written by the decode
    // into mapped host memory and read here at the next launch
    uint32_t* dec_hint_host = nullptr;
    uint32_t* dec_hint_dev = nullptr;
    uint64_t frame_chunks = 0;
    // onc_codec_options (onc_codec_create_ex); nothing is read from the environment
    uint64_t frame_chunk = onc::kFrameChunkDefault;   // bytes per framing chunk (>= 64)
    uint64_t enc_chunk = 0;    // records per plan + emit chunk (multiple of 1024; 0 = kEncChunk)
    bool force_scan = false;   // ONC_OPT_FORCE_SCAN: always launch the block scan (tests)
    uint32_t variant = 0;      // ONC_VARIANT_* bits (A/B measurements, tests)
    int decode_policy = ONC_DECODE_POLICY_AUTO;
    // the batch whose plan (onc_encode_plan) the scratch holds, and the
    // status array that plan filled; every other call that writes the
    // scratch discards it (forget_plan)
    const onc_msg* planned_msgs = nullptr;
    uint64_t planned_n = ~0ull;
    const int32_t* planned_status = nullptr;
    // record lengths the plan wrote for the emit (the caller's rec_len or
    // `lens`): set when the emit reads them (enc_args use_lens), else NULL
    const uint32_t* planned_lens = nullptr;
    uint32_t* lens = nullptr;      // codec-owned record lengths (per plan chunk)
    uint64_t lens_cap = 0;
    // onc_compact / onc_compact_iov: the new offsets (+ the first dropped
    // record's index in the word after them) and the moved bytes
    uint64_t* cmp_off = nullptr;
    uint64_t cmp_off_cap = 0;     // records
    uint8_t* cmp_bytes = nullptr;
    uint64_t cmp_bytes_cap = 0;
    uint32_t timing = 0;   // bitmask of ONC_K_* ids whose launches are bracketed
    struct Pending {
        int kernel;
        hipEvent_t start, stop;
    };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> spare;
    double ms[ONC_K_COUNT] = {};
    uint64_t launches[ONC_K_COUNT] = {};
    std::string last_error;
};

namespace onc {
thread_local LaunchEvents t_launch_events{nullptr, nullptr};
}
constexpr uint64_t kWsMaxTiles = 32768;   // 2M records

namespace {

int fail(onc_codec* c, hipError_t e, const char* what) {
    if (c) {
        c->last_error = std::string(what) + ": " + hipGetErrorString(e);
    }
    return ONC_RC_EHIP;
}

hipEvent_t take_event(onc_codec* c) {
    if (!c->spare.empty()) {
        hipEvent_t e = c->spare.back();
        c->spare.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

// The handle's stream is being captured into a hipGraph: nothing may
// allocate, synchronise or time launches with events on it then.
bool capturing(const onc_codec* c) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(c->stream, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}

// Launch one kernel, bracketed by events when timing is on (never inside a
// capture).
template <class F>
int run(onc_codec* c, int kernel, const char* what, F&& launch) {
    hipEvent_t a = nullptr, b = nullptr;
    const bool timed = ((c->timing >> kernel) & 1u) && !capturing(c);
    if (timed) {
        a = take_event(c);
        b = take_event(c);
        if (a && b) ::onc::t_launch_events = ::onc::LaunchEvents{a, b};   // taken by the launch (kernels.h)
    }
    const hipError_t e = launch();
    if (timed && a && b) {
        if (::onc::t_launch_events.start) {   // nothing was launched (empty batch): time the gap
            ::onc::t_launch_events = ::onc::LaunchEvents{nullptr, nullptr};
            (void)hipEventRecord(a, c->stream);
            (void)hipEventRecord(b, c->stream);
        }
        c->pending.push_back({kernel, a, b});
    }
    if (e != hipSuccess) return fail(c, e, what);
    return ONC_RC_OK;
}

// A call that writes the scratch words a plan lives in (tile / workgroup
// totals) makes a pending onc_encode_plan unusable: onc_encode_emit refuses
// it instead of placing records by another call's totals.
void forget_plan(onc_codec* c) {
    c->planned_n = ~0ull;
    c->planned_msgs = nullptr;
    c->planned_status = nullptr;
    c->planned_lens = nullptr;
}

int refuse_in_capture(onc_codec* c) {
    c->last_error = "scratch would grow during a stream capture: call onc_codec_reserve first";
    return ONC_RC_ECAPTURE;
}

int ensure_lens(onc_codec* c, uint64_t n) {
    if (n <= c->lens_cap) return ONC_RC_OK;
    if (capturing(c)) return refuse_in_capture(c);
    uint64_t want = c->lens_cap ? c->lens_cap : 65536;
    while (want < n) want *= 2;
    if (c->lens) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipFree(c->lens);
        c->lens = nullptr;
        c->lens_cap = 0;
    }
    if (hipMalloc(&c->lens, want * sizeof(uint32_t)) != hipSuccess) return ONC_RC_ENOMEM;
    c->lens_cap = want;
    forget_plan(c);
    return ONC_RC_OK;
}

// Grows a codec-owned device buffer (outside a capture), keeping nothing.
template <class T>
int ensure_buf(onc_codec* c, T*& p, uint64_t& cap, uint64_t want_elems, const char* what) {
    if (want_elems <= cap) return ONC_RC_OK;
    if (capturing(c)) return refuse_in_capture(c);
    uint64_t want = cap ? cap : 65536;
    while (want < want_elems) want *= 2;
    if (p) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    const hipError_t e = hipMalloc(&p, want * sizeof(T));
    if (e != hipSuccess) {
        fail(c, e, what);
        return ONC_RC_ENOMEM;
    }
    cap = want;
    return ONC_RC_OK;
}

// scratch (u64 words): [tile_sum T | spare 2T | block_sum B | block_base B | 16]
uint64_t scratch_words(uint64_t T) { return 3 * T + 2 * (T / 4 + 1) + 16; }

int ensure_scratch(onc_codec* c, uint64_t tiles) {
    if (tiles <= c->scratch_tiles) return ONC_RC_OK;
    if (capturing(c)) return refuse_in_capture(c);
    uint64_t want = c->scratch_tiles ? c->scratch_tiles : 1024;
    while (want < tiles) want *= 2;
    if (c->scratch) {
        // The stream may still be using the old scratch.
        (void)hipStreamSynchronize(c->stream);
        (void)hipFree(c->scratch);
        c->scratch = nullptr;
        c->scratch_tiles = 0;
    }
    hipError_t e = hipMalloc(&c->scratch, scratch_words(want) * sizeof(uint64_t));
    if (e != hipSuccess) {
        fail(c, e, "hipMalloc(scratch)");
        return ONC_RC_ENOMEM;
    }
    c->scratch_tiles = want;
    forget_plan(c);             // a plan in the old scratch is gone
    return ONC_RC_OK;
}

// Points the encoder's per-call state into the codec scratch.
void bind_scratch(onc_codec* c, onc::EncArgs& a) {
    const uint64_t T = c->scratch_tiles;
    const uint64_t B = T / 4 + 1;
    a.tile_sum = c->scratch;
    a.block_sum = c->scratch + 3 * T;
    a.block_base = c->scratch + 3 * T + B;
}

int set_device(onc_codec* c) {
    const hipError_t e = hipSetDevice(c->device);
    if (e != hipSuccess) return fail(c, e, "hipSetDevice");
    return ONC_RC_OK;
}

// The message decode's first-round policy: pinned (ONC_DECODE_POLICY_LINE /
// _STANDARD), or (AUTO) from the previous launch's sample — a plain read of
// mapped host memory: no synchronisation, at worst one launch stale. A
// capture records the kernel instance of the policy in force.
void decode_policy(onc_codec* c, onc::DecArgs& a) {
    a.hint = c->dec_hint_dev;
    if (c->decode_policy == ONC_DECODE_POLICY_AUTO) {
        const uint32_t seen = *reinterpret_cast<volatile uint32_t*>(c->dec_hint_host);
        a.line = seen >= onc::kLine1Min ? 1u : 0u;
    } else {
        a.line = c->decode_policy == ONC_DECODE_POLICY_LINE ? 1u : 0u;
    }
}

}  // namespace

extern "C" {

int onc_abi_version(void) { return ONC_RPC_ABI_VERSION; }

int onc_codec_create(onc_codec** out, int device, void* hip_stream) {
    return onc_codec_create_ex(out, device, hip_stream, nullptr);
}

int onc_codec_create_ex(onc_codec** out, int device, void* hip_stream, const onc_codec_options* o) {
    if (!out) return ONC_RC_EINVAL;
    *out = nullptr;
    if (o && o->size != 0 && o->size < sizeof(onc_codec_options)) return ONC_RC_EINVAL;
    if (o && (o->decode_policy < ONC_DECODE_POLICY_AUTO || o->decode_policy > ONC_DECODE_POLICY_LINE ||
              (o->frame_chunk != 0 && o->frame_chunk < 64) || (o->flags & ~ONC_OPT_FORCE_SCAN) != 0))
        return ONC_RC_EINVAL;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return ONC_RC_EINVAL;
    onc_codec* c = new onc_codec();
    c->device = device;
    c->stream = static_cast<hipStream_t>(hip_stream);
    if (o) {
        c->force_scan = (o->flags & ONC_OPT_FORCE_SCAN) != 0;
        c->variant = o->variant;
        c->decode_policy = o->decode_policy;
        c->enc_chunk = o->enc_chunk / onc::kLenRecs * onc::kLenRecs;
        if (o->frame_chunk) c->frame_chunk = o->frame_chunk;
    }
    if (set_device(c) != ONC_RC_OK) {
        delete c;
        return ONC_RC_EHIP;
    }
    if (hipHostMalloc(reinterpret_cast<void**>(&c->dec_hint_host), 256, hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void**>(&c->dec_hint_dev), c->dec_hint_host, 0) != hipSuccess) {
        if (c->dec_hint_host) (void)hipHostFree(c->dec_hint_host);
        delete c;
        return ONC_RC_ENOMEM;
    }
    *c->dec_hint_host = 0;
    *out = c;
    return ONC_RC_OK;
}

int onc_codec_destroy(onc_codec* c) {
    if (!c) return ONC_RC_EINVAL;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (auto& p : c->pending) {
        (void)hipEventDestroy(p.start);
        (void)hipEventDestroy(p.stop);
    }
    for (auto e : c->spare) (void)hipEventDestroy(e);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->frame_scratch) (void)hipFree(c->frame_scratch);
    if (c->lens) (void)hipFree(c->lens);
    if (c->cmp_off) (void)hipFree(c->cmp_off);
    if (c->cmp_bytes) (void)hipFree(c->cmp_bytes);
    if (c->dec_hint_host) (void)hipHostFree(c->dec_hint_host);
    delete c;
    return ONC_RC_OK;
}

int onc_codec_set_stream(onc_codec* c, void* hip_stream) {
    if (!c) return ONC_RC_EINVAL;
    c->stream = static_cast<hipStream_t>(hip_stream);
    return ONC_RC_OK;
}

int onc_codec_set_decode_policy(onc_codec* c, int policy) {
    if (!c || policy < ONC_DECODE_POLICY_AUTO || policy > ONC_DECODE_POLICY_LINE) return ONC_RC_EINVAL;
    c->decode_policy = policy;
    return ONC_RC_OK;
}

int onc_codec_sync(onc_codec* c) {
    if (!c) return ONC_RC_EINVAL;
    if (set_device(c) != ONC_RC_OK) return ONC_RC_EHIP;
    const hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return fail(c, e, "hipStreamSynchronize");
    return ONC_RC_OK;
}

int onc_codec_reserve(onc_codec* c, uint64_t max_records) {
    if (!c) return ONC_RC_EINVAL;
    if (set_device(c) != ONC_RC_OK) return ONC_RC_EHIP;
    const int rc = ensure_scratch(c, onc::num_emit_tiles(max_records));
    if (rc != ONC_RC_OK) return rc;
    // the plan's record lengths: onc_encode plans a chunk at a time, but
    // onc_encode_plan plans the whole batch at once (4 bytes per record)
    return ensure_lens(c, max_records);
}

// Host ranges onc_host_register pinned, process-wide (a pinned range belongs
// to no codec: hipHostRegister is per process): start -> {length, count}.
// A register of an address inside one of them maps it and counts it once
// more; each unregister of an address inside it counts down, the last one
// unpins. Memory pinned by its owner (hipHostMalloc, torch pin_memory) is
// mapped and never recorded, so unregistering it does nothing.
struct HostPin {
    uint64_t len;
    uint64_t count;
};
static std::mutex g_host_mu;
static std::map<uintptr_t, HostPin> g_host_pinned;

// the recorded range holding [p, p + len) (len 0: holding p), or end()
static std::map<uintptr_t, HostPin>::iterator pinned_range(uintptr_t p, uint64_t len) {
    auto it = g_host_pinned.upper_bound(p);
    if (it == g_host_pinned.begin()) return g_host_pinned.end();
    --it;
    const uint64_t end = it->first + it->second.len;
    return p < end && p + len <= end ? it : g_host_pinned.end();
}

int onc_host_register(onc_codec* c, void* host, uint64_t len, void** dev_ptr) {
    if (!c || !host || !len || !dev_ptr) return ONC_RC_EINVAL;
    *dev_ptr = nullptr;
    if (set_device(c) != ONC_RC_OK) return ONC_RC_EHIP;
    std::lock_guard<std::mutex> lk(g_host_mu);
    const uintptr_t p = reinterpret_cast<uintptr_t>(host);
    auto mine = g_host_pinned.end();
    hipPointerAttribute_t attr{};
    bool pinned = false;
    if (hipPointerGetAttributes(&attr, host) == hipSuccess) pinned = attr.type == hipMemoryTypeHost;
    else (void)hipGetLastError();                 // an ordinary host pointer
    if (pinned) {
        // inside a range this library pinned: counted once more; inside
        // memory its owner pinned: the whole [host, host + len) must lie in
        // that allocation (else a kernel would fault past its end)
        mine = pinned_range(p, len);
        if (mine == g_host_pinned.end()) {
            // (a range inside one registered here but running past it is
            // refused the same way: it is not one pinned allocation)
            if (pinned_range(p, 0) != g_host_pinned.end()) {
                c->last_error = "onc_host_register: range runs past the pinned range holding its start";
                return ONC_RC_EINVAL;
            }
            void* base = nullptr;
            size_t size = 0;
            if (hipMemGetAddressRange(reinterpret_cast<hipDeviceptr_t*>(&base), &size, host) == hipSuccess) {
                const uintptr_t b = reinterpret_cast<uintptr_t>(base);
                if (p < b || p + len > b + size) {
                    c->last_error = "onc_host_register: range runs past its pinned allocation";
                    return ONC_RC_EINVAL;
                }
            } else {
                (void)hipGetLastError();             // no range known: mapped as the runtime reports it
            }
        }
    } else {
        const hipError_t r = hipHostRegister(host, size_t(len), hipHostRegisterMapped | hipHostRegisterPortable);
        if (r == hipSuccess) {
            mine = g_host_pinned.emplace(p, HostPin{len, 0}).first;
        } else if (r == hipErrorHostMemoryAlreadyRegistered) {
            (void)hipGetLastError();                 // pinned by its owner: only mapped
        } else {
            (void)hipGetLastError();
            return fail(c, r, "hipHostRegister");
        }
    }
    const hipError_t e = hipHostGetDevicePointer(dev_ptr, host, 0);
    if (e != hipSuccess) {
        if (mine != g_host_pinned.end() && mine->second.count == 0) {
            (void)hipHostUnregister(reinterpret_cast<void*>(mine->first));
            g_host_pinned.erase(mine);
        }
        *dev_ptr = nullptr;
        return fail(c, e, "hipHostGetDevicePointer");
    }
    if (mine != g_host_pinned.end()) ++mine->second.count;
    return ONC_RC_OK;
}

int onc_host_unregister(onc_codec* c, void* host) {
    if (!host) return ONC_RC_EINVAL;
    std::lock_guard<std::mutex> lk(g_host_mu);
    const auto it = pinned_range(reinterpret_cast<uintptr_t>(host), 0);
    if (it == g_host_pinned.end()) return ONC_RC_OK;      // not pinned here: nothing to undo
    if (--it->second.count != 0) return ONC_RC_OK;        // still mapped by another registration
    void* start = reinterpret_cast<void*>(it->first);
    g_host_pinned.erase(it);
    const hipError_t e = hipHostUnregister(start);
    return e == hipSuccess ? ONC_RC_OK : fail(c, e, "hipHostUnregister");
}

const char* onc_codec_last_error(const onc_codec* c) { return c ? c->last_error.c_str() : "null codec"; }

const char* onc_status_str(int32_t s) {
    switch (s) {
        case ONC_OK: return "ok";
        case ONC_ERR_INCOMPLETE_MESSAGE: return "incomplete rpc message";
        case ONC_ERR_INCOMPLETE_HEADER: return "incomplete fragment header";
        case ONC_ERR_FRAGMENTED: return "RPC message is fragmented";
        case ONC_ERR_INVALID_MESSAGE_TYPE: return "invalid rpc message type";
        case ONC_ERR_INVALID_REPLY_TYPE: return "invalid rpc reply type";
        case ONC_ERR_INVALID_REPLY_STATUS: return "invalid rpc reply status";
        case ONC_ERR_INVALID_AUTH_DATA: return "invalid rpc auth data";
        case ONC_ERR_INVALID_AUTH_ERROR: return "invalid rpc auth error status";
        case ONC_ERR_INVALID_REJECTED_REPLY_TYPE: return "invalid rpc rejected reply type";
        case ONC_ERR_INVALID_LENGTH: return "invalid length in rpc message";
        case ONC_ERR_INVALID_RPC_VERSION: return "invalid rpc version";
        case ONC_ERR_INVALID_MACHINE_NAME: return "invalid machine name";
        case ONC_ERR_IO_UNEXPECTED_EOF: return "i/o error (UnexpectedEof): failed to fill whole buffer";
        case ONC_ENC_TOO_LONG: return "message length exceeds maximum";
        case ONC_ENC_AUTH_GT_200: return "auth associated data exceeds 200 bytes";
        case ONC_ENC_NAME_GT_255: return "machine name exceeds 255 bytes";
        case ONC_ENC_GIDS_GT_16: return "more than 16 gids";
        case ONC_ENC_BAD_DESCRIPTOR: return "invalid message descriptor";
        case ONC_ENC_WRITE_ZERO: return "failed to write whole buffer";
        default: return "unknown status";
    }
}

const char* onc_kernel_name(int k) {
    switch (k) {
        case ONC_K_ENC_LEN: return "enc_len_kernel";
        case ONC_K_SCAN_TILES: return "scan_tiles_kernel";
        case ONC_K_ENC_EMIT: return "enc_emit_kernel";
        case ONC_K_DEC_PARSE: return "decode_kernel";
        case ONC_K_LEN_TILES: return "len_tiles_kernel";
        case ONC_K_LEN_APPLY: return "len_apply_kernel";
        case ONC_K_IOV_LEN: return "iov_len_kernel";
        case ONC_K_IOV_EMIT: return "iov_emit_kernel";
        case ONC_K_FRAME: return "frame_chunks_kernel";
        case ONC_K_FRAME_WRITE: return "frame_write_kernel";
        case ONC_K_FRAME_WALK: return "frame_walk_kernel";
        case ONC_K_FRAME_COUNTS: return "frame_counts_kernel";
        case ONC_K_FRAME_GUESS: return "frame_guess_kernel";
        case ONC_K_COMPACT: return "compact_kernels";
        default: return "?";
    }
}

int onc_codec_enable_timing(onc_codec* c, int enable) {
    if (!c) return ONC_RC_EINVAL;
    c->timing = uint32_t(enable) & ((1u << ONC_K_COUNT) - 1u);
    return ONC_RC_OK;
}

int onc_codec_kernel_stats(onc_codec* c, double* ms_total, uint64_t* launches) {
    if (!c) return ONC_RC_EINVAL;
    if (set_device(c) != ONC_RC_OK) return ONC_RC_EHIP;
    const hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return fail(c, e, "hipStreamSynchronize");
    for (auto& p : c->pending) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.start, p.stop) == hipSuccess) {
            c->ms[p.kernel] += ms;
            c->launches[p.kernel] += 1;
        }
        c->spare.push_back(p.start);
        c->spare.push_back(p.stop);
    }
    c->pending.clear();
    for (int k = 0; k < ONC_K_COUNT; ++k) {
        if (ms_total) ms_total[k] = c->ms[k];
        if (launches) launches[k] = c->launches[k];
    }
    return ONC_RC_OK;
}

int onc_codec_reset_stats(onc_codec* c) {
    if (!c) return ONC_RC_EINVAL;
    double tmp[ONC_K_COUNT];
    uint64_t tl[ONC_K_COUNT];
    const int rc = onc_codec_kernel_stats(c, tmp, tl);
    for (int k = 0; k < ONC_K_COUNT; ++k) {
        c->ms[k] = 0;
        c->launches[k] = 0;
    }
    return rc;
}

static int check_batch(const onc_batch* b) {
    if (!b) return ONC_RC_EINVAL;
    if (b->n && !b->msgs) return ONC_RC_EINVAL;
    // a non-empty arena needs a pointer
    if ((b->unix_count && !b->unix_params) || (b->auth_len && !b->auth_arena) ||
        (b->payload_len && !b->payload_arena))
        return ONC_RC_EINVAL;
    return ONC_RC_OK;
}

static onc::Bounds bounds_of(const onc_batch* b) { return onc::Bounds{b->unix_count, b->auth_len, b->payload_len}; }

int onc_encode_lengths(onc_codec* c, const onc_batch* batch, uint32_t* rec_len, int32_t* status) {
    if (!c || check_batch(batch) != ONC_RC_OK || (batch->n && (!rec_len || !status))) return ONC_RC_EINVAL;
    if (batch->n == 0) return ONC_RC_OK;
    if (set_device(c) != ONC_RC_OK) return ONC_RC_EHIP;
    const uint64_t tiles = onc::num_emit_tiles(batch->n);
    int rc = ensure_scratch(c, tiles);
    if (rc != ONC_RC_OK) return rc;
    onc::EncArgs a{};
    a.n = batch->n;
    a.msgs = batch->msgs;
    a.unix = batch->unix_params;
    a.auth_arena = batch->auth_arena;
    a.payload_arena = batch->payload_arena;
    a.bounds = bounds_of(batch);
    a.status = status;
    a.rec_len = rec_len;
    a.decl = 2;        // the extents onc_encode places, every check up front (onc_auth)
    bind_scratch(c, a);
    forget_plan(c);
    return run(c, ONC_K_ENC_LEN, "enc_len", [&] { return onc::launch_enc_len(a, c->stream); });
}

namespace {

// Encoder arguments common to the plan and emit phases.
int enc_args(onc_codec* c, const onc_batch* batch, int32_t* status, uint32_t* rec_len, onc::EncArgs& a,
             uint32_t root = ONC_ROOT_RPC_MESSAGE, uint64_t n_whole = 0) {
    const uint64_t tiles = onc::num_emit_tiles(batch->n);
    const int rc = ensure_scratch(c, tiles);
    if (rc != ONC_RC_OK) return rc;
    a = onc::EncArgs{};
    a.n = batch->n;
    a.msgs = batch->msgs;
    a.unix = batch->unix_params;
    a.auth_arena = batch->auth_arena;
    a.payload_arena = batch->payload_arena;
    a.bounds = bounds_of(batch);
    a.status = status;
    a.rec_len = rec_len;
    bind_scratch(c, a);
    // Up to kFusedBlocks enc_len workgroups (1M records), enc_emit sums the
    // workgroup totals itself and the scan launch is skipped.
    a.variant = c->variant;
    // enc_emit kernel choice: the wave-specialised kernel
    // (a producer wave stages spans while three stream the previous one) for
    // batches of <= 2M records whose payloads average >= 128 bytes (or of
    // any size when they average >= 512 bytes: configs[3], 4M x 1 KiB,
    // enc_emit 1808 -> 1765 us) — there
    // it removes the lock-step staging rounds of the wave-per-tile kernel
    // (configs[1]: enc_emit 123 -> 116 us); header-heavy records make its
    // single producer the bottleneck (configs[0]-shaped: 117 -> 141 us) and
    // at 8M records the wave-per-tile kernel's rounds are amortised (903 vs
    // 945 us). Variant bits force it (0x200) or the wave-per-tile kernel
    // (0x400). It places tiles from the workgroup totals itself at any size.
    const uint64_t n = batch->n;
    // the arena's bytes per record are those of the whole batch (a chunk of
    // a chunked encode shares its arenas)
    const uint64_t nw = n_whole ? n_whole : n;
    // a.ws: 0 wave-per-tile; 1 wave-specialised, 2 KiB consumer steps; 2 the
    // same with 1 KiB steps (long payloads: configs[3] 1770 vs 1815 us)
    const bool big = batch->payload_len >= 512 * nw;
    const bool ws_shape = batch->payload_len >= 128 * nw && (onc::num_emit_tiles(n) <= kWsMaxTiles || big);
    a.ws = ((c->variant & ONC_VARIANT_EMIT_WS) || (!(c->variant & ONC_VARIANT_EMIT_TILE) && n && ws_shape)) ? (big ? 2u : 1u) : 0u;
    a.root = root;
    if (root != ONC_ROOT_RPC_MESSAGE) a.ws = 0;   // body roots: the wave-per-tile kernel
    // the wave-specialised kernel checks the real payload volume itself
    // (encode.hip ws_header_heavy): enc_len writes per-workgroup payload
    // totals into the scratch's spare words
    if (a.ws) a.block_pay = c->scratch + c->scratch_tiles;
    a.fused_base = (onc::num_len_blocks(n) <= onc::kFusedBlocks && !c->force_scan) || a.ws;
    return ONC_RC_OK;
}

// The wave-per-tile enc_emit reads the plan's record lengths instead of
// planning again when the batch can hold AUTH_UNIX auths: its own plan would
// load each credential's parameter block (ngids, name_len) one dependent
// round trip after the descriptor (configs[0]-shaped batches). Variant bit
// 0x20000 keeps the re-planning emit.
bool use_lens(const onc_codec* c, const onc_batch* batch, const onc::EncArgs& a) {
    return !a.ws && a.root == ONC_ROOT_RPC_MESSAGE && batch->unix_count != 0 && !(c->variant & ONC_VARIANT_EMIT_REPLAN);
}

// enc_len: plans + per-tile and per-workgroup byte totals into the scratch.
int enc_plan(onc_codec* c, const onc_batch* batch, int32_t* status, uint32_t* rec_len,
             uint32_t root = ONC_ROOT_RPC_MESSAGE, uint64_t n_whole = 0) {
    onc::EncArgs a;
    int rc = enc_args(c, batch, status, rec_len, a, root, n_whole);
    if (rc != ONC_RC_OK) return rc;
    forget_plan(c);
    // the lengths the emit reads back live in codec-owned memory (the
    // caller's rec_len, when given, receives a copy): nothing the caller
    // does between plan and emit can make the emit's placement disagree
    // with the plan's totals
    // declared AUTH_UNIX lengths planned as given; the emit checks the blocks
    a.decl = root == ONC_ROOT_RPC_MESSAGE ? 1u : 0u;
    const bool lens = use_lens(c, batch, a);
    if (lens) {
        rc = ensure_lens(c, batch->n);
        if (rc != ONC_RC_OK) return rc;
        a.len_out = c->lens;
    }
    rc = run(c, ONC_K_ENC_LEN, "enc_len", [&] { return onc::launch_enc_len(a, c->stream); });
    if (rc != ONC_RC_OK) return rc;
    if (root == ONC_ROOT_RPC_MESSAGE) {
        c->planned_msgs = batch->msgs;
        c->planned_n = batch->n;
        c->planned_status = status;
        c->planned_lens = lens ? c->lens : nullptr;
    }
    return ONC_RC_OK;
}

// [scan of the workgroup totals, with the grand total into rec_off[n]] +
// enc_emit: the bytes, placed by the plan in the scratch.
int enc_emit(onc_codec* c, const onc_batch* batch, uint8_t* out, uint64_t out_cap, uint64_t* rec_off,
             int32_t* status, uint32_t* rec_len, uint32_t root = ONC_ROOT_RPC_MESSAGE, uint64_t n_whole = 0,
             const uint64_t* base_dev = nullptr) {
    onc::EncArgs a;
    int rc = enc_args(c, batch, status, rec_len, a, root, n_whole);
    if (rc != ONC_RC_OK) return rc;
    // any writer position: the kernels work on 16-byte chunks from the
    // aligned address below `out`, whose first `origin` bytes are never written
    a.origin = reinterpret_cast<uintptr_t>(out) & 15;
    a.out = out - a.origin;
    a.out_cap = out ? a.origin + out_cap : 0;
    a.rec_off = rec_off;
    a.rec_len = nullptr;   // written by the plan
    a.base_dev = base_dev;
    if (use_lens(c, batch, a)) a.len_in = c->planned_lens;
    if (!a.fused_base) {
        const uint64_t nblk = onc::num_len_blocks(batch->n);
        rc = run(c, ONC_K_SCAN_TILES, "scan", [&] {
            // (no total out: the emit's last record writes rec_off[n], and in a
            // chunked encode rec_off[n] is the next chunk's base)
            return onc::launch_scan_tiles(a.block_sum, a.block_base, nblk, 0, nullptr, c->stream);
        });
        if (rc != ONC_RC_OK) return rc;
    }
    return run(c, ONC_K_ENC_EMIT, "enc_emit", [&] { return onc::launch_enc_emit(a, c->stream); });
}

// plan + emit of a whole batch. Beyond kEncChunk records the batch is
// encoded as consecutive chunks of kEncChunk records, each planned right
// before it is emitted: enc_emit then reads the descriptors enc_len has just
// read (64 MB per chunk: held by the 256 MB Infinity Cache) instead of
// descriptors a whole-batch enc_len read hundreds of MB earlier, and every
// chunk places its tiles by summing its own workgroup totals (no scan
// launch). Chunk k + 1 starts where chunk k ended: its kernels read that
// offset from rec_off[k's end], which chunk k's emit wrote.
constexpr uint64_t kEncChunk = onc::kFusedBlocks * onc::kLenRecs;   // 1M records

// Small batches (at most one enc_emit_single_kernel workgroup: kSpWaves
// tiles, 512 records): one launch, no length pass. The workgroup's waves plan
// their tiles and hand the totals to wave 0 through LDS (encode.hip
// wg_place); nothing outside the workgroup is read or waited on. The per-message loop of a drop-in caller
// (the C++ mirror's serialise_into) pays one kernel launch instead of two.
// Variant bits that force an emit kernel keep the two-pass path (tests).
constexpr uint64_t kSmallRecs = uint64_t(onc::kEmitRecs) * onc::kSpWaves;
constexpr uint32_t kForcedEmit = ONC_VARIANT_EMIT_WS | ONC_VARIANT_EMIT_TILE | ONC_VARIANT_EMIT_REPLAN;
int small_batch(onc_codec* c, const onc_batch* batch, uint8_t* out, uint64_t out_cap, uint64_t* rec_off,
                int32_t* status, uint32_t* rec_len) {
    onc::EncArgs a;
    int rc = enc_args(c, batch, status, rec_len, a);
    if (rc != ONC_RC_OK) return rc;
    forget_plan(c);
    a.ws = 0;
    a.block_pay = nullptr;
    a.small = 1;
    a.origin = reinterpret_cast<uintptr_t>(out) & 15;
    a.out = out - a.origin;
    a.out_cap = out ? a.origin + out_cap : 0;
    a.rec_off = rec_off;
    a.rec_len = rec_len;
    return run(c, ONC_K_ENC_EMIT, "enc_emit", [&] { return onc::launch_enc_emit(a, c->stream); });
}

int encode_batch(onc_codec* c, const onc_batch* batch, uint8_t* out, uint64_t out_cap, uint64_t* rec_off,
                 int32_t* status, uint32_t* rec_len, uint32_t root) {
    const uint64_t n = batch->n;
    const uint64_t chunk = c->enc_chunk ? c->enc_chunk : kEncChunk;
    if (root == ONC_ROOT_RPC_MESSAGE && n <= kSmallRecs && n <= chunk && !(c->variant & kForcedEmit))
        return small_batch(c, batch, out, out_cap, rec_off, status, rec_len);
    if (n <= chunk || (c->variant & ONC_VARIANT_WHOLE_PLAN)) {     // whole-batch plan (lab)
        const int rc = enc_plan(c, batch, status, rec_len, root);
        if (rc != ONC_RC_OK) return rc;
        return enc_emit(c, batch, out, out_cap, rec_off, status, nullptr, root);
    }
    for (uint64_t c0 = 0; c0 < n; c0 += chunk) {
        onc_batch sub = *batch;
        sub.n = std::min(chunk, n - c0);
        sub.msgs = batch->msgs + c0;
        int rc = enc_plan(c, &sub, status + c0, rec_len ? rec_len + c0 : nullptr, root, n);
        if (rc != ONC_RC_OK) return rc;
        rc = enc_emit(c, &sub, out, out_cap, rec_off + c0, status + c0, nullptr, root, n,
                      c0 ? rec_off + c0 : nullptr);
        if (rc != ONC_RC_OK) return rc;
    }
    forget_plan(c);
    return ONC_RC_OK;
}

}  // namespace

int onc_encode(onc_codec* c, const onc_batch* batch, uint8_t* out, uint64_t out_cap, uint64_t* rec_off,
               int32_t* status, uint32_t* rec_len) {
    if (!c || check_batch(batch) != ONC_RC_OK || !rec_off) return ONC_RC_EINVAL;
    if (batch->n && (!status || (!out && out_cap))) return ONC_RC_EINVAL;
    if (set_device(c) != ONC_RC_OK) return ONC_RC_EHIP;
    if (batch->n == 0) {
        const hipError_t e = hipMemsetAsync(rec_off, 0, sizeof(uint64_t), c->stream);
        return e == hipSuccess ? ONC_RC_OK : fail(c, e, "hipMemsetAsync");
    }
    return encode_batch(c, batch, out, out_cap, rec_off, status, rec_len, ONC_ROOT_RPC_MESSAGE);
}

int onc_encode_plan(onc_codec* c, const onc_batch* batch, int32_t* status, uint32_t* rec_len) {
    if (!c || check_batch(batch) != ONC_RC_OK) return ONC_RC_EINVAL;
    if (batch->n && !status) return ONC_RC_EINVAL;
    if (set_device(c) != ONC_RC_OK) return ONC_RC_EHIP;
    if (batch->n == 0) {
        c->planned_msgs = batch->msgs;
        c->planned_n = 0;
        c->planned_status = status;
        return ONC_RC_OK;
    }
    return enc_plan(c, batch, status, rec_len);
}

int onc_encode_emit(onc_codec* c, const onc_batch* batch, uint8_t* out, uint64_t out_cap, uint64_t* rec_off,
                    int32_t* status) {
    if (!c || check_batch(batch) != ONC_RC_OK || !rec_off) return ONC_RC_EINVAL;
    if (batch->n && (!status || (!out && out_cap))) return ONC_RC_EINVAL;
    // the plan in this handle's scratch must be of this batch, with its statuses
    if (c->planned_n != batch->n || c->planned_msgs != batch->msgs) return ONC_RC_EINVAL;
    if (batch->n && c->planned_status != status) return ONC_RC_EINVAL;
    if (set_device(c) != ONC_RC_OK) return ONC_RC_EHIP;
    if (batch->n == 0) {
        const hipError_t e = hipMemsetAsync(rec_off, 0, sizeof(uint64_t), c->stream);
        return e == hipSuccess ? ONC_RC_OK : fail(c, e, "hipMemsetAsync");
    }
    return enc_emit(c, batch, out, out_cap, rec_off, status, nullptr);
}

int onc_encode_iov(onc_codec* c, const onc_batch* batch, uint8_t* hdr_out, uint64_t hdr_cap, onc_iov_rec* iov,
                   int32_t* status, uint64_t* totals) {
    if (!c || check_batch(batch) != ONC_RC_OK) return ONC_RC_EINVAL;
    if (batch->n && (!iov || !status || (!hdr_out && hdr_cap))) return ONC_RC_EINVAL;
    if ((reinterpret_cast<uintptr_t>(hdr_out) & 3) != 0) return ONC_RC_EALIGN;
    if (set_device(c) != ONC_RC_OK) return ONC_RC_EHIP;
    if (batch->n == 0) {
        if (!totals) return ONC_RC_OK;
        const hipError_t e = hipMemsetAsync(totals, 0, 2 * sizeof(uint64_t), c->stream);
        return e == hipSuccess ? ONC_RC_OK : fail(c, e, "hipMemsetAsync");
    }
    const uint64_t tiles = onc::num_emit_tiles(batch->n);
    int rc = ensure_scratch(c, tiles);
    if (rc != ONC_RC_OK) return rc;
    const uint64_t T = c->scratch_tiles;
    const uint64_t B = T / 4 + 1;
    forget_plan(c);
    onc::IovArgs a{};
    a.n = batch->n;
    a.msgs = batch->msgs;
    a.unix = batch->unix_params;
    a.auth_arena = batch->auth_arena;
    a.payload_arena = batch->payload_arena;
    a.bounds = bounds_of(batch);
    a.hdr_out = hdr_out;
    a.hdr_cap = hdr_out ? hdr_cap : 0;
    a.iov = iov;
    a.status = status;
    a.totals = totals;
    a.tile_sum = c->scratch;
    a.block_len = c->scratch + 3 * T;
    a.block_len_base = c->scratch + 3 * T + B;
    a.block_hdr = c->scratch + 2 * T;
    a.block_hdr_base = c->scratch + 2 * T + B;
    // iov_len workgroup totals (kLenRecs records each); up to kFusedBlocks of
    // them iov_emit sums itself, beyond that two scan launches place them
    const uint64_t nblk = onc::num_len_blocks(batch->n);
    rc = run(c, ONC_K_IOV_LEN, "iov_len", [&] { return onc::launch_iov_len(a, c->stream); });
    if (rc != ONC_RC_OK) return rc;
    if (nblk > onc::kFusedBlocks) {
        rc = run(c, ONC_K_SCAN_TILES, "scan", [&] {
            return onc::launch_scan_tiles(a.block_len, a.block_len_base, nblk, 0, nullptr, c->stream);
        });
        if (rc != ONC_RC_OK) return rc;
        rc = run(c, ONC_K_SCAN_TILES, "scan", [&] {
            return onc::launch_scan_tiles(a.block_hdr, a.block_hdr_base, nblk, 0, nullptr, c->stream);
        });
        if (rc != ONC_RC_OK) return rc;
    }
    return run(c, ONC_K_IOV_EMIT, "iov_emit", [&] { return onc::launch_iov_emit(a, c->stream); });
}

// Per-chunk framing state: 56 bytes per chunk + summary flags + the count
// scan's tile sums.
static size_t frame_bytes(uint64_t P) { return P * (56 + 8 * 64) + 2 * (P / 256 + 2) + 2 * (P / 65536 + 2) + (onc::num_tiles(P) + 1) * 16 + 128; }

int onc_frame_stream(onc_codec* c, const uint8_t* wire, uint64_t len, uint64_t* rec_off, uint64_t max_records,
                     uint64_t* result) {
    if (!c || !rec_off || !result || (len && !wire)) return ONC_RC_EINVAL;
    if (set_device(c) != ONC_RC_OK) return ONC_RC_EHIP;
    hipError_t e;
    if (len == 0 || max_records == 0) {                   // nothing framed, nothing consumed
        e = hipMemsetAsync(result, 0, 5 * sizeof(uint64_t), c->stream);
        if (e == hipSuccess) e = hipMemsetAsync(rec_off, 0, sizeof(uint64_t), c->stream);
        if (e != hipSuccess) return fail(c, e, "hipMemsetAsync");
        return ONC_RC_OK;
    }
    // (otherwise frame_guess clears result and rec_off[0] as it starts)
    const uint64_t chunk = c->frame_chunk;
    const uint64_t P = (len + chunk - 1) / chunk;
    if (P > c->frame_chunks) {
        // (in a capture: frame a stream of this size once before capturing)
        if (capturing(c)) return refuse_in_capture(c);
        uint64_t want = c->frame_chunks ? c->frame_chunks : 4096;
        while (want < P) want *= 2;
        if (c->frame_scratch) {
            (void)hipStreamSynchronize(c->stream);
            (void)hipFree(c->frame_scratch);
            c->frame_scratch = nullptr;
            c->frame_chunks = 0;
        }
        e = hipMalloc(&c->frame_scratch, frame_bytes(want));
        if (e != hipSuccess) return fail(c, e, "hipMalloc(frame scratch)");
        c->frame_chunks = want;
    }
    const uint64_t Q = c->frame_chunks;
    uint8_t* f = c->frame_scratch;
    onc::FrameArgs a{};
    a.wire = wire;
    a.len = len;
    a.chunk = chunk;
    a.nchunks = P;
    a.max_records = max_records;
    a.rec_off = rec_off;
    a.result = result;
    a.g = reinterpret_cast<uint64_t*>(f);
    a.x = reinterpret_cast<uint64_t*>(f + 8 * Q);
    a.cnt_base = reinterpret_cast<uint64_t*>(f + 16 * Q);
    a.aux = reinterpret_cast<uint32_t*>(f + 24 * Q);
    a.cnt = reinterpret_cast<uint32_t*>(f + 32 * Q);
    a.st = reinterpret_cast<int32_t*>(f + 36 * Q);
    a.cnt_eff = reinterpret_cast<uint32_t*>(f + 40 * Q);
    a.fail = f + 44 * Q;
    a.stop = f + 45 * Q;
    uint8_t* flags = f + 46 * Q;   // 10 bytes per chunk remain in the 56-byte budget
    a.fail2 = flags;
    a.stop2 = flags + (Q / 256 + 2);
    a.fail3 = flags + 2 * (Q / 256 + 2);
    a.stop3 = a.fail3 + (Q / 65536 + 2);
    a.starts = reinterpret_cast<uint64_t*>(f + 56 * Q);    // 64 starts per chunk
    uint64_t* tail = reinterpret_cast<uint64_t*>(f + (56 + 8 * 64) * Q);
    const uint64_t nt = onc::num_tiles(P);
    uint64_t* tile_sum = tail;
    uint64_t* tile_base = tail + nt + 1;
    a.first_fail = tail + 2 * (nt + 1);
    a.first_stop = a.first_fail + 1;
    int rc = run(c, ONC_K_FRAME_GUESS, "frame_guess", [&] { return onc::launch_frame_guess(a, c->stream); });
    if (rc != ONC_RC_OK) return rc;
    rc = run(c, ONC_K_FRAME, "frame_chunks", [&] { return onc::launch_frame_chunks(a, c->stream); });
    if (rc != ONC_RC_OK) return rc;
    rc = run(c, ONC_K_FRAME_WALK, "frame_walk", [&] { return onc::launch_frame_walk(a, c->stream); });
    if (rc != ONC_RC_OK) return rc;
    if (onc::frame_fused_scan_ok(P) && !c->force_scan) {
        // counts + block totals, then a wave per chunk summing its first
        // record index and copying its kept record starts
        rc = run(c, ONC_K_FRAME_COUNTS, "frame_cblk", [&] { return onc::launch_frame_cblk(a, tile_sum, c->stream); });
        if (rc != ONC_RC_OK) return rc;
        return run(c, ONC_K_FRAME_WRITE, "frame_write",
                   [&] { return onc::launch_frame_write_slots(a, tile_sum, c->stream); });
    }
    rc = run(c, ONC_K_FRAME_COUNTS, "frame_counts", [&] { return onc::launch_frame_counts(a, c->stream); });
    if (rc != ONC_RC_OK) return rc;
    rc = run(c, ONC_K_LEN_TILES, "len_tiles", [&] { return onc::launch_len_tiles(a.cnt_eff, P, tile_sum, c->stream); });
    if (rc != ONC_RC_OK) return rc;
    rc = run(c, ONC_K_SCAN_TILES, "scan_tiles",
             [&] { return onc::launch_scan_tiles(tile_sum, tile_base, nt, 0, nullptr, c->stream); });
    if (rc != ONC_RC_OK) return rc;
    rc = run(c, ONC_K_LEN_APPLY, "len_apply",
             [&] { return onc::launch_len_apply(a.cnt_eff, P, tile_base, a.cnt_base, c->stream); });
    if (rc != ONC_RC_OK) return rc;
    return run(c, ONC_K_FRAME_WRITE, "frame_write", [&] { return onc::launch_frame_write(a, c->stream); });
}

int onc_decode(onc_codec* c, const uint8_t* wire, const uint64_t* rec_off, uint64_t n, int mode,
               const onc_decoded* out) {
    if (!c || !out || (mode != ONC_DECODE_SLICE && mode != ONC_DECODE_BYTES)) return ONC_RC_EINVAL;
    if (n == 0) return ONC_RC_OK;
    if (!rec_off || !out->msgs || !out->unix_params || !out->status || !out->aux0 || !out->aux1)
        return ONC_RC_EINVAL;
    if (set_device(c) != ONC_RC_OK) return ONC_RC_EHIP;
    onc::DecArgs a{};
    a.n = n;
    a.wire = wire;
    a.rec_off = rec_off;
    a.out = *out;
    a.variant = c->variant;
    decode_policy(c, a);
    return run(c, ONC_K_DEC_PARSE, "decode", [&] { return onc::launch_decode(a, mode, c->stream); });
}

int onc_decode_lengths(onc_codec* c, const uint8_t* wire, const uint32_t* rec_len, uint64_t n, uint64_t base,
                       int mode, uint64_t* rec_off, const onc_decoded* out) {
    if (!c || !out || (mode != ONC_DECODE_SLICE && mode != ONC_DECODE_BYTES)) return ONC_RC_EINVAL;
    if (n == 0) return ONC_RC_OK;
    if (!rec_len || !out->msgs || !out->unix_params || !out->status || !out->aux0 || !out->aux1)
        return ONC_RC_EINVAL;
    if (set_device(c) != ONC_RC_OK) return ONC_RC_EHIP;
    // scratch: 64-record workgroup totals (n / 64 words, within the 3T words
    // before the block area), 4096-record block totals and their scan
    const uint64_t wgs = (n + 63) / 64, nblk = (n + onc::kDecLenBlk - 1) / onc::kDecLenBlk;
    int rc = ensure_scratch(c, std::max<uint64_t>(onc::num_tiles(n), wgs / 3 + 1));
    if (rc != ONC_RC_OK) return rc;
    const uint64_t T = c->scratch_tiles;
    forget_plan(c);
    onc::DecArgs a{};
    a.n = n;
    a.wire = wire;
    a.out = *out;
    a.variant = c->variant;
    decode_policy(c, a);
    a.rec_len = rec_len;
    a.tile_sum = c->scratch;
    a.blk_sum = c->scratch + 3 * T;
    a.nblk = nblk;
    a.base = base;
    a.rec_off_out = rec_off;
    uint64_t* blk_sum = c->scratch + 3 * T;
    // one decode workgroup (n <= 64): its offsets are its own wave scan of
    // the lengths from `base` — the totals of earlier workgroups and blocks
    // it would read are masked to 0 (decode.hip kFromLen), so no dlen_tiles
    // launch (a single message's try_from pays one launch)
    if (wgs > 1 || c->force_scan) {
        rc = run(c, ONC_K_LEN_TILES, "dlen_tiles", [&] {
            return onc::launch_dlen_tiles(rec_len, n, c->scratch, blk_sum, c->stream);
        });
        if (rc != ONC_RC_OK) return rc;
    }
    if (nblk > onc::kDecLenFusedBlocks || c->force_scan) {
        uint64_t* blk_base = blk_sum + (T / 4 + 1);
        rc = run(c, ONC_K_SCAN_TILES, "scan_tiles",
                 [&] { return onc::launch_scan_tiles(blk_sum, blk_base, nblk, 0, nullptr, c->stream); });
        if (rc != ONC_RC_OK) return rc;
        a.blk_base = blk_base;
    }
    return run(c, ONC_K_DEC_PARSE, "decode", [&] { return onc::launch_decode(a, mode, c->stream); });
}

int onc_scan_lengths(onc_codec* c, const uint32_t* rec_len, uint64_t n, uint64_t base, uint64_t* rec_off) {
    if (!c || !rec_off || (n && !rec_len)) return ONC_RC_EINVAL;
    if (set_device(c) != ONC_RC_OK) return ONC_RC_EHIP;
    if (n == 0) {
        const hipError_t e = onc::launch_store_u64(rec_off, base, c->stream);
        return e == hipSuccess ? ONC_RC_OK : fail(c, e, "store_u64");
    }
    const uint64_t tiles = onc::num_tiles(n);
    int rc = ensure_scratch(c, tiles);
    if (rc != ONC_RC_OK) return rc;
    uint64_t* tile_sum = c->scratch;
    uint64_t* tile_base = c->scratch + c->scratch_tiles;
    forget_plan(c);
    if (onc::scan_lengths_fused_ok(n) && !c->force_scan) {
        // two launches: 4096-record block totals, then every block sums the
        // totals before it and scans its own lengths
        rc = run(c, ONC_K_LEN_TILES, "lenblk", [&] { return onc::launch_lenblk(rec_len, n, tile_sum, c->stream); });
        if (rc != ONC_RC_OK) return rc;
        return run(c, ONC_K_LEN_APPLY, "lenoff",
                   [&] { return onc::launch_lenoff(rec_len, n, tile_sum, base, rec_off, c->stream); });
    }
    rc = run(c, ONC_K_LEN_TILES, "len_tiles", [&] { return onc::launch_len_tiles(rec_len, n, tile_sum, c->stream); });
    if (rc != ONC_RC_OK) return rc;
    rc = run(c, ONC_K_SCAN_TILES, "scan_tiles",
             [&] { return onc::launch_scan_tiles(tile_sum, tile_base, tiles, base, rec_off + n, c->stream); });
    if (rc != ONC_RC_OK) return rc;
    return run(c, ONC_K_LEN_APPLY, "len_apply",
               [&] { return onc::launch_len_apply(rec_len, n, tile_base, rec_off, c->stream); });
}

int onc_decode_body(onc_codec* c, int root, const uint8_t* wire, const uint64_t* rec_off, uint64_t n, int mode,
                    const uint32_t* param, const onc_decoded* out, uint32_t* consumed) {
    if (!c || !out || (mode != ONC_DECODE_SLICE && mode != ONC_DECODE_BYTES)) return ONC_RC_EINVAL;
    if (root < 0 || root >= ONC_ROOT_COUNT) return ONC_RC_EINVAL;
    if (n == 0) return ONC_RC_OK;
    if (!rec_off || !out->msgs || !out->unix_params || !out->status || !out->aux0 || !out->aux1)
        return ONC_RC_EINVAL;
    // the roots whose reference decoder takes a length argument
    if (!param && (root == ONC_ROOT_OPAQUE || (root == ONC_ROOT_AUTH_UNIX_PARAMS && mode == ONC_DECODE_SLICE)))
        return ONC_RC_EINVAL;
    if (set_device(c) != ONC_RC_OK) return ONC_RC_EHIP;
    onc::DecArgs a{};
    a.n = n;
    a.wire = wire;
    a.rec_off = rec_off;
    a.out = *out;
    a.variant = c->variant;
    a.root = uint32_t(root);
    a.param = param;
    a.consumed = consumed;
    a.body = 1;
    return run(c, ONC_K_DEC_PARSE, "decode", [&] { return onc::launch_decode(a, mode, c->stream); });
}

int onc_encode_body_lengths(onc_codec* c, int root, const onc_batch* batch, uint32_t* rec_len, int32_t* status) {
    if (!c || root < 0 || root >= ONC_ROOT_COUNT || check_batch(batch) != ONC_RC_OK || (batch->n && (!rec_len || !status)))
        return ONC_RC_EINVAL;
    if (batch->n == 0) return ONC_RC_OK;
    if (set_device(c) != ONC_RC_OK) return ONC_RC_EHIP;
    onc::EncArgs a;
    const int rc = enc_args(c, batch, status, rec_len, a, uint32_t(root));
    if (rc != ONC_RC_OK) return rc;
    forget_plan(c);
    return run(c, ONC_K_ENC_LEN, "enc_len", [&] { return onc::launch_enc_len(a, c->stream); });
}

int onc_encode_body(onc_codec* c, int root, const onc_batch* batch, uint8_t* out, uint64_t out_cap, uint64_t* rec_off,
                    int32_t* status, uint32_t* rec_len) {
    if (!c || root < 0 || root >= ONC_ROOT_COUNT || check_batch(batch) != ONC_RC_OK || !rec_off) return ONC_RC_EINVAL;
    if (batch->n && (!status || (!out && out_cap))) return ONC_RC_EINVAL;
    if (set_device(c) != ONC_RC_OK) return ONC_RC_EHIP;
    if (batch->n == 0) {
        const hipError_t e = hipMemsetAsync(rec_off, 0, sizeof(uint64_t), c->stream);
        return e == hipSuccess ? ONC_RC_OK : fail(c, e, "hipMemsetAsync");
    }
    return encode_batch(c, batch, out, out_cap, rec_off, status, rec_len, uint32_t(root));
}

int onc_compact(onc_codec* c, uint8_t* out, uint64_t* rec_off, const int32_t* status, uint64_t n, uint64_t* total) {
    if (!c || !rec_off || (n && (!status || !out))) return ONC_RC_EINVAL;
    if (set_device(c) != ONC_RC_OK) return ONC_RC_EHIP;
    if (capturing(c)) return refuse_in_capture(c);    // synchronous: sizes its scratch from the batch
    hipError_t e;
    if (n == 0) {
        if (total) {
            e = hipMemcpyAsync(total, rec_off, sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
            if (e != hipSuccess) return fail(c, e, "hipMemcpyAsync");
        }
        return ONC_RC_OK;
    }
    int rc = ensure_lens(c, n);
    if (rc == ONC_RC_OK) rc = ensure_buf(c, c->cmp_off, c->cmp_off_cap, n + 2, "hipMalloc(compact offsets)");
    if (rc != ONC_RC_OK) return rc;
    forget_plan(c);
    uint64_t* first_drop = c->cmp_off + n + 1;
    uint64_t* info_dev = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(c->dec_hint_dev) + 64);
    volatile uint64_t* info = reinterpret_cast<volatile uint64_t*>(reinterpret_cast<uint8_t*>(c->dec_hint_host) + 64);
    e = hipMemsetAsync(first_drop, 0xFF, sizeof(uint64_t), c->stream);
    if (e != hipSuccess) return fail(c, e, "hipMemsetAsync");
    rc = run(c, ONC_K_COMPACT, "compact_lens",
             [&] { return onc::launch_compact_lens(rec_off, status, n, c->lens, first_drop, c->stream); });
    if (rc == ONC_RC_OK) rc = onc_scan_lengths(c, c->lens, n, 0, c->cmp_off);
    if (rc == ONC_RC_OK)
        rc = run(c, ONC_K_COMPACT, "compact_info",
                 [&] { return onc::launch_compact_info(rec_off, c->cmp_off, n, first_drop, info_dev, c->stream); });
    if (rc != ONC_RC_OK) return rc;
    e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return fail(c, e, "hipStreamSynchronize");
    const uint64_t fb = info[0], base = info[1], lo = info[2], new_end = info[4];
    if (total) *total = fb < n ? new_end : info[3];
    if (fb >= n) return ONC_RC_OK;                       // no extent to drop: nothing moves
    const uint64_t moved = new_end - lo;
    if (moved) {
        rc = ensure_buf(c, c->cmp_bytes, c->cmp_bytes_cap, moved + 16, "hipMalloc(compact bytes)");
        if (rc != ONC_RC_OK) return rc;
        rc = run(c, ONC_K_COMPACT, "compact_gather", [&] {
            return onc::launch_compact_gather(out, rec_off, c->cmp_off, fb, n, base, lo, c->cmp_bytes, c->stream);
        });
        if (rc != ONC_RC_OK) return rc;
        e = hipMemcpyAsync(out + lo, c->cmp_bytes, moved, hipMemcpyDefault, c->stream);   // (out may be mapped host memory)
        if (e != hipSuccess) return fail(c, e, "hipMemcpyAsync");
    }
    rc = run(c, ONC_K_COMPACT, "compact_offsets",
             [&] { return onc::launch_compact_offsets(rec_off, c->cmp_off, fb, n, base, c->stream); });
    if (rc != ONC_RC_OK) return rc;
    e = hipStreamSynchronize(c->stream);             // synchronous: the buffer is final on return
    return e == hipSuccess ? ONC_RC_OK : fail(c, e, "hipStreamSynchronize");
}

int onc_compact_iov(onc_codec* c, onc_iov_rec* iov, const int32_t* status, uint64_t n, uint64_t* totals) {
    if (!c || (n && (!iov || !status))) return ONC_RC_EINVAL;
    if (set_device(c) != ONC_RC_OK) return ONC_RC_EHIP;
    hipError_t e;
    if (totals) {
        e = hipMemsetAsync(totals, 0, 2 * sizeof(uint64_t), c->stream);
        if (e != hipSuccess) return fail(c, e, "hipMemsetAsync");
    }
    if (n == 0) return ONC_RC_OK;
    int rc = ensure_lens(c, n);
    if (rc == ONC_RC_OK) rc = ensure_buf(c, c->cmp_off, c->cmp_off_cap, n + 2, "hipMalloc(compact offsets)");
    if (rc != ONC_RC_OK) return rc;
    forget_plan(c);
    rc = run(c, ONC_K_COMPACT, "compact_iov_lens",
             [&] { return onc::launch_compact_iov_lens(iov, status, n, c->lens, c->stream); });
    if (rc == ONC_RC_OK) rc = onc_scan_lengths(c, c->lens, n, 0, c->cmp_off);
    if (rc != ONC_RC_OK) return rc;
    return run(c, ONC_K_COMPACT, "compact_iov_apply",
               [&] { return onc::launch_compact_iov_apply(iov, status, n, c->cmp_off, totals, c->stream); });
}

int32_t onc_expected_message_len(const uint8_t* data, uint64_t len, uint32_t* out) {
    if (out) *out = 0;
    if (!data || len < 4) return ONC_ERR_INCOMPLETE_HEADER;          // rpc_message.rs:344-346
    const uint32_t header = (uint32_t(data[0]) << 24) | (uint32_t(data[1]) << 16) |
                            (uint32_t(data[2]) << 8) | uint32_t(data[3]);
    if ((header & 0x80000000u) == 0) return ONC_ERR_FRAGMENTED;       // :359-362
    if (out) *out = (header & 0x7FFFFFFFu) + 4;                       // :365
    return ONC_OK;
}


}  // extern "C"
