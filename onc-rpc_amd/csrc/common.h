// common.h — device-side building blocks shared by the gfx950 codec kernels.
//
// Everything here is integer/byte work on 64-wide wavefronts. The wire is a
// byte stream of big-endian u32 words and raw payload bytes; registers hold
// stream bytes in little-endian order (stream byte b of a word = register
// byte b), so a header field value v is stored as __builtin_bswap32(v).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/onc_rpc.h"

namespace onc {

constexpr int kTile = 256;        // records per tile (= threads per block)
constexpr int kScanThreads = 1024;
constexpr int kEmitRecs = 64;    // records per encode tile = one wavefront (enc_len totals, enc_emit)
#ifndef ONC_LEN_RECS
#define ONC_LEN_RECS 1024
#endif
constexpr int kLenRecs = ONC_LEN_RECS;   // records per enc_len workgroup (= per scanned total)

__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

// Bytes [sh, sh+4) of the 8-byte little-endian concatenation lo|hi
// (v_alignbyte_b32).
__device__ __forceinline__ uint32_t funnel(uint32_t lo, uint32_t hi, uint32_t sh) {
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// pad_length — reference src/opaque.rs:115-121
__host__ __device__ __forceinline__ uint32_t pad4(uint32_t l) { return (4u - (l & 3u)) & 3u; }
__host__ __device__ __forceinline__ uint32_t words4(uint32_t l) { return (l + 3u) >> 2; }

// Loads through address_space(1) pointers: plain integer addresses would
// otherwise lower to flat_load (which also waits on lgkmcnt).
#define ONC_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ T gload(uintptr_t a) {
    return *(const ONC_GLOBAL T*)a;
}
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// A whole 64-byte descriptor as four dwordx4 loads. Callers issue these
// with the other loads of their prologue and pin the registers
// (pin_msg) before the first use, so all of them cost one memory round
// trip: left alone, the compiler narrows the load to the fields each branch
// of the planner reads and sinks each piece into its branch, one dependent
// round trip per field.
struct MsgRegs {
    u32x4 q[4];
};
__device__ __forceinline__ MsgRegs issue_msg(const onc_msg* p) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    MsgRegs r;
#pragma unroll
    for (int k = 0; k < 4; ++k) r.q[k] = gload<u32x4>(a + 16 * k);
    return r;
}
__device__ __forceinline__ onc_msg as_msg(const MsgRegs& r) {
    onc_msg m;
    __builtin_memcpy(&m, &r, sizeof(m));
    return m;
}

// Four stream bytes at absolute byte address `addr`, bytes at or beyond
// `lim` read as zero. Precondition: addr < lim. Only aligned dwords that
// contain at least one byte < lim are touched, so the read never leaves
// the valid range's pages. Branch-free (both loads always issue).
__device__ __forceinline__ uint32_t load4_masked(uintptr_t addr, uintptr_t lim) {
    const uintptr_t al = addr & ~uintptr_t(3);
    const uint32_t sh = uint32_t(addr & 3);
    const bool second = sh != 0 && al + 4 < lim;
    const uint32_t w0 = gload<uint32_t>(al);
    const uint32_t w1 = gload<uint32_t>(al + (second ? 4 : 0));
    uint32_t v = funnel(w0, second ? w1 : 0u, sh);
    const uintptr_t n = lim - addr;
    if (n < 4) v &= (1u << (8u * uint32_t(n))) - 1u;
    return v;
}

// Same without the tail mask: all four bytes are known to be valid.
__device__ __forceinline__ uint32_t load4(uintptr_t addr) {
    const uintptr_t al = addr & ~uintptr_t(3);
    const uint32_t sh = uint32_t(addr & 3);
    const uint32_t w0 = gload<uint32_t>(al);
    const uint32_t w1 = gload<uint32_t>(al + (sh ? 4 : 0));
    return funnel(w0, sh ? w1 : 0u, sh);
}

// 16 bytes at an arbitrary byte address, all valid: one dwordx4 load at the
// 4-aligned address below it, one more dword, v_alignbyte.
__device__ __forceinline__ void load16_unaligned(uintptr_t addr, uint32_t v[4]) {
    const uintptr_t al = addr & ~uintptr_t(3);
    const uint32_t sh = uint32_t(addr & 3);
    const u32x4_a4 w = gload<u32x4_a4>(al);
    const uint32_t w4 = gload<uint32_t>(al + (sh ? 16 : 12));
    v[0] = funnel(w.x, w.y, sh);
    v[1] = funnel(w.y, w.z, sh);
    v[2] = funnel(w.z, w.w, sh);
    v[3] = funnel(w.w, sh ? w4 : 0u, sh);
}

// ---------------------------------------------------------------------------
// Encode planning: serialised_len + validation of one descriptor
// ---------------------------------------------------------------------------
//
// Word counts of the header part of a record (everything before the raw
// payload). XDR pads every item to 4 bytes, so the header is a whole number
// of words relative to the record start; only the payload is unpadded and it
// always comes last (call_body.rs:107, accepted_reply.rs:199).

struct AuthPlan {
    uint32_t words;    // serialised_len / 4  (flavor.rs:154-174)
    uint32_t assoc;    // associated_data_len  (flavor.rs:142-150)
    int32_t status;    // construction-time panics
};

// Sizes of the arenas a batch's descriptors point into (onc_batch): every
// reference is checked against them before it is dereferenced.
struct Bounds {
    uint64_t n_unix;
    uint64_t auth_len;
    uint64_t payload_len;
};

// [off, off + len) lies inside an arena of `size` bytes (no overflow).
__device__ __forceinline__ bool in_arena(uint64_t off, uint64_t len, uint64_t size) {
    return off <= size && len <= size - off;
}

// AuthUnixParams::serialised_len (unix_params.rs:219-230) of a name length and gid count
__host__ __device__ __forceinline__ uint32_t unix_body_len(uint32_t nl, uint32_t ng) { return 20u + 4u * words4(nl) + 4u * ng; }
// A declared AUTH_UNIX length (onc_auth.len, ABI 6) that some parameter block can have: a multiple of 4
// between the empty block (20) and a 255-byte name with 16 gids.
__host__ __device__ __forceinline__ bool unix_len_plausible(uint32_t l) {
    return l >= 20u && (l & 3u) == 0 && l <= unix_body_len(ONC_MAX_MACHINE_NAME_LEN, ONC_MAX_GIDS);
}

// kDecl: an AUTH_UNIX auth that declares its length (onc_auth.len != 0) is
// planned from the descriptor alone — no parameter-block load; the block's
// checks (the name / gid panics, the name's arena bounds, declared ==
// serialised length) are deferred to the emit (check_declared_unix). The
// encoder's length pass runs this form first and the full one only for a
// record it fails (include/onc_rpc.h onc_auth).
template <bool kDecl = false>
__device__ __forceinline__ AuthPlan plan_auth(const onc_auth& a, const onc_unix_params* unix, const Bounds& bd) {
    AuthPlan p;
    const uint32_t kind = a.kind_len >> 24;
    const uint32_t len = a.kind_len & 0xFFFFFFu;
    p.status = ONC_OK;
    if (kind == ONC_KIND_UNIX) {
        if (a.ref >= bd.n_unix) { p.status = ONC_ENC_BAD_DESCRIPTOR; p.words = 0; p.assoc = 0; return p; }
        if (kDecl && len != 0) {
            if (!unix_len_plausible(len)) { p.status = ONC_ENC_BAD_DESCRIPTOR; p.words = 0; p.assoc = 0; return p; }
            p.words = 2 + len / 4;
            // associated_data_len = len - 8 - pad(name) in [len - 11, len - 8]: with len a multiple
            // of 4, len - 8 > 200 exactly when the true value is
            p.assoc = len - 8;
            return p;
        }
        const onc_unix_params* u = unix + a.ref;
        const uint32_t nl = u->name_len, ng = u->ngids;
        // AuthUnixParams::new panics (unix_params.rs:149), then Gids (:47)
        if (nl > ONC_MAX_MACHINE_NAME_LEN) { p.status = ONC_ENC_NAME_GT_255; p.words = 0; p.assoc = 0; return p; }
        if (ng > ONC_MAX_GIDS) { p.status = ONC_ENC_GIDS_GT_16; p.words = 0; p.assoc = 0; return p; }
        if (nl != 0 && !in_arena(u->name_off, nl, bd.auth_len)) {
            p.status = ONC_ENC_BAD_DESCRIPTOR; p.words = 0; p.assoc = 0; return p;
        }
        // a declared length must be the block's
        if (len != 0 && len != unix_body_len(nl, ng)) { p.status = ONC_ENC_BAD_DESCRIPTOR; p.words = 0; p.assoc = 0; return p; }
        // id + len + stamp + opaque(name) + uid + gid + ngids + gids
        p.words = 2 + 1 + 1 + words4(nl) + 3 + ng;
        p.assoc = 12 + nl + 4 * ng;               // unix_params.rs:234-245
    } else if (kind <= ONC_KIND_UNKNOWN) {
        if (len != 0 && !in_arena(a.ref, len, bd.auth_len)) {
            p.status = ONC_ENC_BAD_DESCRIPTOR; p.words = 0; p.assoc = 0; return p;
        }
        p.words = 2 + words4(len);                // id + opaque
        p.assoc = len;
    } else {
        p.status = ONC_ENC_BAD_DESCRIPTOR; p.words = 0; p.assoc = 0;
    }
    return p;
}

// meta word: cred words | verf words << 8 | header words << 16
struct RecPlan {
    uint64_t len;     // serialised_len (0 if status != OK)
    uint32_t meta;
    int32_t status;
};

__device__ __forceinline__ uint32_t meta_cw(uint32_t m) { return m & 0xFFu; }
__device__ __forceinline__ uint32_t meta_vw(uint32_t m) { return (m >> 8) & 0xFFu; }
__device__ __forceinline__ uint32_t meta_hw(uint32_t m) { return m >> 16; }

// RpcMessage::serialised_len (rpc_message.rs:201-204) plus the checks of
// serialise_into in reference order: descriptor / construction panics
// (cred, then verf), oversize (rpc_message.rs:146-151), then the
// associated-data assert (flavor.rs:110, cred before verf).
// kDecl: a Call credential's declared AUTH_UNIX length is taken as given
// (plan_auth); a record that fails this form fails the full one too, with
// the full one's status.
template <bool kDecl = false>
__device__ __forceinline__ RecPlan plan_record(const onc_msg& d, const onc_unix_params* unix, const Bounds& bd) {
    RecPlan r;
    r.len = 0;
    r.meta = 0;
    r.status = ONC_OK;
    uint32_t cw = 0, vw = 0, hw;
    uint64_t body = 0;
    uint32_t assoc_c = 0, assoc_v = 0;
    if (d.msg_type == ONC_MSG_CALL) {
        // (only a Call's credential is planned from its declared length: a
        // verifier's block is checked here — AUTH_UNIX verifiers are rare)
        AuthPlan c = plan_auth<kDecl>(d.cred, unix, bd);
        if (c.status) { r.status = c.status; return r; }
        AuthPlan v = plan_auth<false>(d.verf, unix, bd);
        if (v.status) { r.status = v.status; return r; }
        cw = c.words; vw = v.words;
        assoc_c = c.assoc; assoc_v = v.assoc;
        hw = 7 + cw + vw;   // mark, xid, mtype, rpcvers, prog, vers, proc
        body = d.payload_len;
    } else if (d.msg_type == ONC_MSG_REPLY) {
        if (d.reply_stat == ONC_REPLY_ACCEPTED) {
            if (d.stat > ONC_ACCEPT_SYSTEM_ERR) { r.status = ONC_ENC_BAD_DESCRIPTOR; return r; }
            AuthPlan v = plan_auth<false>(d.verf, unix, bd);
            if (v.status) { r.status = v.status; return r; }
            vw = v.words; assoc_v = v.assoc;
            // mark, xid, mtype, reply_stat, verf, accept_stat [, low, high]
            hw = 4 + vw + 1 + (d.stat == ONC_ACCEPT_PROG_MISMATCH ? 2 : 0);
            body = d.stat == ONC_ACCEPT_SUCCESS ? d.payload_len : 0;
        } else if (d.reply_stat == ONC_REPLY_DENIED) {
            if (d.stat > ONC_REJECT_AUTH_ERROR) { r.status = ONC_ENC_BAD_DESCRIPTOR; return r; }
            if (d.stat == ONC_REJECT_AUTH_ERROR && d.auth_stat > ONC_AUTH_STAT_MAX) {
                r.status = ONC_ENC_BAD_DESCRIPTOR; return r;
            }
            hw = 5 + (d.stat == ONC_REJECT_RPC_MISMATCH ? 2 : 1);
        } else {
            r.status = ONC_ENC_BAD_DESCRIPTOR; return r;
        }
    } else {
        r.status = ONC_ENC_BAD_DESCRIPTOR; return r;
    }
    // payload reference inside the payload arena (onc_batch bounds)
    if (body != 0 && !in_arena(d.payload_off, body, bd.payload_len)) { r.status = ONC_ENC_BAD_DESCRIPTOR; return r; }
    const uint64_t total = 4ull * hw + body;
    if (total & 0xFFFFFFFF80000000ull) { r.status = ONC_ENC_TOO_LONG; return r; }
    if (assoc_c > ONC_MAX_AUTH_LEN || assoc_v > ONC_MAX_AUTH_LEN) { r.status = ONC_ENC_AUTH_GT_200; return r; }
    r.len = total;
    r.meta = cw | (vw << 8) | (hw << 16);
    return r;
}

// The checks plan_auth<true> deferred, in plan_auth's order, on the first 32
// bytes of the auth's parameter block (q0 = stamp, uid, gid, ngids; q1 =
// name_off, name_len, reserved).
__device__ __forceinline__ int32_t check_declared_unix(const u32x4& q0, const u32x4& q1, uint32_t declared,
                                                       uint64_t auth_len) {
    const uint32_t ng = q0.w, nl = q1.z;
    const uint64_t noff = uint64_t(q1.x) | (uint64_t(q1.y) << 32);
    if (nl > ONC_MAX_MACHINE_NAME_LEN) return ONC_ENC_NAME_GT_255;
    if (ng > ONC_MAX_GIDS) return ONC_ENC_GIDS_GT_16;
    if (nl != 0 && !in_arena(noff, nl, auth_len)) return ONC_ENC_BAD_DESCRIPTOR;
    if (unix_body_len(nl, ng) != declared) return ONC_ENC_BAD_DESCRIPTOR;
    return ONC_OK;
}

// The emit's side of plan_record<true>: the deferred checks of a Call's
// declared AUTH_UNIX credential, run by put_unix_words on the block words it
// loads anyway (emits that did not preload the block).
struct DeclCheck {
    uint64_t auth_len;   // the auth arena's size (the machine name's bounds)
    int32_t* st;         // receives the failing check's status (left alone when the block passes)
};

struct EncSrc {
    const onc_unix_params* unix;
    uintptr_t auth_arena;
    uintptr_t payload_arena;
};

// Sequential serialiser of the header words of one planned record (the
// serialise_into call chain in write order), used to stage headers in LDS.
// Emits meta_hw(meta) words, in order, into a sink.

// Sink: plain word stream.
struct WordSink {
    uint32_t* dst;
    __device__ __forceinline__ void operator()(uint32_t w) { *dst++ = w; }
};

// Sink: the same stream re-aligned to output dwords for a record starting at
// byte offset m = start & 3 (m != 0): output dword j = stream bytes
// [4j - m, 4j - m + 4), with bytes outside the header zero. Writes hw + 1
// words (finish() writes the last one).
struct ShiftSink {
    uint32_t* dst;
    uint32_t prev;
    uint32_t sh;       // 4 - m
    __device__ __forceinline__ void operator()(uint32_t w) {
        *dst++ = funnel(prev, w, sh);
        prev = w;
    }
    __device__ __forceinline__ void finish() { *dst = funnel(prev, 0u, sh); }
};

// The whole 96-byte parameter block of unix-table entry `ref` in six dwordx4
// loads issued together (one memory round trip; field by field, each gid was
// a dependent load between two sink writes).
struct UnixRegs {
    u32x4 q[6];
};
__device__ __forceinline__ UnixRegs issue_unix(const onc_unix_params* unix, uint64_t ref) {
    static_assert(sizeof(onc_unix_params) == 96 && offsetof(onc_unix_params, ngids) == 12 &&
                      offsetof(onc_unix_params, name_off) == 16 && offsetof(onc_unix_params, name_len) == 24 &&
                      offsetof(onc_unix_params, gids) == 32,
                  "parameter block layout read by put_unix_words");
    const uintptr_t ua = reinterpret_cast<uintptr_t>(unix + ref);
    UnixRegs u;
#pragma unroll
    for (int k = 0; k < 6; ++k) u.q[k] = gload<u32x4>(ua + 16 * k);
    return u;
}

// AuthUnixParams::serialise_into (unix_params.rs:162-176) of a loaded
// parameter block, preceded (kLen) by its serialised_len — the opaque length
// AuthFlavor::serialise_into writes before it (flavor.rs:123-126).
template <bool kLen, class Sink>
__device__ __forceinline__ void put_unix_words(const UnixRegs& u, const EncSrc& s, Sink& out,
                                               DeclCheck* dc = nullptr, uint32_t declared = 0) {
    const u32x4* q = u.q;
    uint32_t ng = q[0].w, nl = q[1].z;
    if (dc && declared != 0) {
        // a block that fails is serialised as an empty one (no name read, no
        // gids: 20 bytes, never past the declared extent, which is >= 20);
        // its status goes to *dc->st and the caller clears what the record
        // wrote
        const int32_t st = check_declared_unix(q[0], q[1], declared, dc->auth_len);
        if (st != ONC_OK) {
            *dc->st = st;
            ng = nl = 0;
        }
    }
    const uint32_t stamp = q[0].x, uid = q[0].y, gid = q[0].z;
    const uint64_t name_off = uint64_t(q[1].x) | (uint64_t(q[1].y) << 32);
    const uint32_t gids[ONC_MAX_GIDS] = {q[2].x, q[2].y, q[2].z, q[2].w, q[3].x, q[3].y, q[3].z, q[3].w,
                                         q[4].x, q[4].y, q[4].z, q[4].w, q[5].x, q[5].y, q[5].z, q[5].w};
    if (kLen) out(bswap(20u + 4u * words4(nl) + 4u * ng));
    out(bswap(stamp));
    out(bswap(nl));
    const uintptr_t b = s.auth_arena + name_off;
    for (uint32_t j = 0; 4 * j < nl; ++j) out(load4_masked(b + 4ull * j, b + nl));
    out(bswap(uid));
    out(bswap(gid));
    out(bswap(ng));
#pragma unroll
    for (uint32_t j = 0; j < ONC_MAX_GIDS; ++j)
        if (j < ng) out(bswap(gids[j]));
}

// ... of unix-table entry `ref`
template <bool kLen, class Sink>
__device__ __forceinline__ void put_unix_words(uint64_t ref, const EncSrc& s, Sink& out, DeclCheck* dc = nullptr,
                                               uint32_t declared = 0) {
    put_unix_words<kLen>(issue_unix(s.unix, ref), s, out, dc, declared);
}

// Opaque::serialise_into (opaque.rs:38-56) of an auth body: length, body
// words, the last one zero padded.
template <class Sink>
__device__ __forceinline__ void put_opaque_words(const onc_auth& a, const EncSrc& s, Sink& out) {
    const uint32_t len = a.kind_len & 0xFFFFFFu;
    out(bswap(len));
    const uintptr_t b = s.auth_arena + a.ref;
    for (uint32_t j = 0; 4 * j < len; ++j) out(load4_masked(b + 4ull * j, b + len));
}

// AuthFlavor::serialise_into (flavor.rs:106-129).
// (pre: the auth's parameter block, already loaded — an AUTH_UNIX credential
// whose block the caller issued with its other loads)
template <class Sink>
__device__ __forceinline__ void put_auth_words(const onc_auth& a, const EncSrc& s, Sink& out,
                                               const UnixRegs* pre = nullptr, bool use_pre = false,
                                               DeclCheck* dc = nullptr) {
    const uint32_t kind = a.kind_len >> 24;
    out(bswap(kind == ONC_KIND_UNKNOWN ? a.id : kind));
    if (kind != ONC_KIND_UNIX) {
        put_opaque_words(a, s, out);
        return;
    }
    const uint32_t declared = a.kind_len & 0xFFFFFFu;
    if (use_pre) put_unix_words<true>(*pre, s, out, dc, declared);
    else put_unix_words<true>(a.ref, s, out, dc, declared);
}

// CallBody::serialise_into (call_body.rs:98-108) up to the raw payload.
template <class Sink>
__device__ __forceinline__ void put_call_words(const onc_msg& d, const EncSrc& s, Sink& out,
                                               const UnixRegs* cred_pre = nullptr, bool use_pre = false,
                                               DeclCheck* dc = nullptr) {
    out(bswap(2u));                           // RPC_VERSION call_body.rs:10
    out(bswap(d.u.call.program));
    out(bswap(d.u.call.program_version));
    out(bswap(d.u.call.procedure));
    put_auth_words(d.cred, s, out, cred_pre, use_pre, dc);
    put_auth_words(d.verf, s, out);
}

// AcceptedStatus::serialise_into (accepted_reply.rs:195-211) up to a
// Success payload.
template <class Sink>
__device__ __forceinline__ void put_accepted_status_words(const onc_msg& d, Sink& out) {
    out(bswap(uint32_t(d.stat)));
    if (d.stat == ONC_ACCEPT_PROG_MISMATCH) {
        out(bswap(d.u.mismatch.low));
        out(bswap(d.u.mismatch.high));
    }
}

// RejectedReply::serialise_into (rejected_reply.rs:61-73; AuthError :194-207).
template <class Sink>
__device__ __forceinline__ void put_rejected_words(const onc_msg& d, Sink& out) {
    out(bswap(uint32_t(d.stat)));
    if (d.stat == ONC_REJECT_RPC_MISMATCH) {
        out(bswap(d.u.mismatch.low));
        out(bswap(d.u.mismatch.high));
    } else {
        out(bswap(uint32_t(d.auth_stat)));
    }
}

// ReplyBody::serialise_into (reply_body.rs:45-56; AcceptedReply
// accepted_reply.rs:58-61) up to a Success payload.
template <class Sink>
__device__ __forceinline__ void put_reply_words(const onc_msg& d, const EncSrc& s, Sink& out) {
    out(bswap(uint32_t(d.reply_stat)));
    if (d.reply_stat == ONC_REPLY_ACCEPTED) {
        put_auth_words(d.verf, s, out);
        put_accepted_status_words(d, out);
        return;
    }
    put_rejected_words(d, out);
}

// RpcMessage::serialise_into (rpc_message.rs:136-164; MessageType :55-68)
// up to the raw payload.
// (cred_pre, when use_pre: the Call's AUTH_UNIX credential block, already loaded)
// (dc: run the deferred checks of a declared AUTH_UNIX credential, plan_record<true>)
template <class Sink>
__device__ __forceinline__ void put_header_words(const onc_msg& d, uint32_t len, const EncSrc& s, Sink& out,
                                                 const UnixRegs* cred_pre = nullptr, bool use_pre = false,
                                                 DeclCheck* dc = nullptr) {
    out(bswap((len - 4u) | 0x80000000u));        // record mark, rpc_message.rs:156
    out(bswap(d.xid));
    out(bswap(uint32_t(d.msg_type)));
    if (d.msg_type == ONC_MSG_CALL) put_call_words(d, s, out, cred_pre, use_pre, dc);
    else put_reply_words(d, s, out);
}

__device__ __forceinline__ void put_header_words(const onc_msg& d, uint32_t len, const EncSrc& s, uint32_t* dst) {
    WordSink w{dst};
    put_header_words(d, len, s, w);
}

// The header of a record whose declared AUTH_UNIX credential failed a
// deferred block check (include/onc_rpc.h onc_auth, ABI 7): the record mark
// of its extent (rpc_message.rs:156), so that a receiver's
// expected_message_len (:343-367) still frames it, then hw - 1 zero words.
template <class Sink>
__device__ __forceinline__ void put_placeholder_words(uint32_t len, uint32_t hw, Sink& out) {
    out(bswap((len - 4u) | 0x80000000u));
    for (uint32_t k = 1; k < hw; ++k) out(0u);
}

// ---------------------------------------------------------------------------
// Body-level roots (ONC_ROOT_*, include/onc_rpc.h): the serialised_len and
// serialise_into of one type of the message tree instead of RpcMessage.
// The header words of a root are a sub-sequence of the message's, written by
// the same pieces above; a Call / Success payload still comes last.
// ---------------------------------------------------------------------------

// Does the descriptor have the shape of `root`'s value?
__device__ __forceinline__ bool root_shape_ok(const onc_msg& d, uint32_t root) {
    const bool call = d.msg_type == ONC_MSG_CALL, reply = d.msg_type == ONC_MSG_REPLY;
    const bool acc = reply && d.reply_stat == ONC_REPLY_ACCEPTED, den = reply && d.reply_stat == ONC_REPLY_DENIED;
    switch (root) {
        case ONC_ROOT_MESSAGE_TYPE: return call || reply;
        case ONC_ROOT_CALL_BODY:
        case ONC_ROOT_AUTH_FLAVOR: return call;
        case ONC_ROOT_AUTH_UNIX_PARAMS: return call && (d.cred.kind_len >> 24) == ONC_KIND_UNIX;
        case ONC_ROOT_OPAQUE:
            return call && (d.cred.kind_len >> 24) != ONC_KIND_UNIX && (d.cred.kind_len >> 24) <= ONC_KIND_UNKNOWN &&
                   (d.cred.kind_len & 0xFFFFFFu) <= ONC_OPAQUE_ENCODE_MAX;
        case ONC_ROOT_REPLY_BODY: return reply;
        case ONC_ROOT_ACCEPTED_REPLY:
        case ONC_ROOT_ACCEPTED_STATUS: return acc;
        case ONC_ROOT_REJECTED_REPLY: return den;
        case ONC_ROOT_AUTH_ERROR: return den && d.stat == ONC_REJECT_AUTH_ERROR;
        default: return false;
    }
}

// serialised_len of `root` + its serialise_into checks (see onc_encode_body_lengths):
// shape, then the descriptor checks of plan_record for the parts the root
// serialises, the 2^31 limit, and the assoc assert for roots that
// serialise an AuthFlavor. meta: cw / vw as plan_record, hw = the root's
// header words (everything before the payload).
__device__ __forceinline__ RecPlan plan_root(const onc_msg& d, const onc_unix_params* unix, const Bounds& bd,
                                             uint32_t root) {
    if (root == ONC_ROOT_RPC_MESSAGE) return plan_record(d, unix, bd);
    RecPlan r;
    r.len = 0;
    r.meta = 0;
    r.status = ONC_OK;
    if (!root_shape_ok(d, root)) { r.status = ONC_ENC_BAD_DESCRIPTOR; return r; }
    uint32_t cw = 0, vw = 0, hw = 0;
    uint64_t body = 0;
    uint32_t assoc_c = 0, assoc_v = 0;
    if (root == ONC_ROOT_AUTH_FLAVOR || root == ONC_ROOT_AUTH_UNIX_PARAMS || root == ONC_ROOT_OPAQUE) {
        const AuthPlan c = plan_auth(d.cred, unix, bd);
        if (c.status) { r.status = c.status; return r; }
        cw = c.words;
        // AuthFlavor: id + body; AuthUnixParams: without id and length;
        // Opaque: without the id
        hw = root == ONC_ROOT_AUTH_FLAVOR ? cw : (root == ONC_ROOT_AUTH_UNIX_PARAMS ? cw - 2 : cw - 1);
        if (root == ONC_ROOT_AUTH_FLAVOR) assoc_c = c.assoc;
    } else if (d.msg_type == ONC_MSG_CALL) {         // MESSAGE_TYPE, CALL_BODY
        const AuthPlan c = plan_auth(d.cred, unix, bd);
        if (c.status) { r.status = c.status; return r; }
        const AuthPlan v = plan_auth(d.verf, unix, bd);
        if (v.status) { r.status = v.status; return r; }
        cw = c.words; vw = v.words;
        assoc_c = c.assoc; assoc_v = v.assoc;
        hw = (root == ONC_ROOT_MESSAGE_TYPE ? 1 : 0) + 4 + cw + vw;
        body = d.payload_len;
    } else if (d.reply_stat == ONC_REPLY_ACCEPTED) {  // MESSAGE_TYPE .. ACCEPTED_STATUS
        if (d.stat > ONC_ACCEPT_SYSTEM_ERR) { r.status = ONC_ENC_BAD_DESCRIPTOR; return r; }
        if (root != ONC_ROOT_ACCEPTED_STATUS) {
            const AuthPlan v = plan_auth(d.verf, unix, bd);
            if (v.status) { r.status = v.status; return r; }
            vw = v.words; assoc_v = v.assoc;
        }
        hw = (root == ONC_ROOT_MESSAGE_TYPE ? 2 : (root == ONC_ROOT_REPLY_BODY ? 1 : 0)) + vw + 1 +
             (d.stat == ONC_ACCEPT_PROG_MISMATCH ? 2 : 0);
        body = d.stat == ONC_ACCEPT_SUCCESS ? d.payload_len : 0;
    } else if (d.reply_stat == ONC_REPLY_DENIED) {    // MESSAGE_TYPE, REPLY_BODY, REJECTED_REPLY, AUTH_ERROR
        if (d.stat > ONC_REJECT_AUTH_ERROR) { r.status = ONC_ENC_BAD_DESCRIPTOR; return r; }
        if (d.stat == ONC_REJECT_AUTH_ERROR && d.auth_stat > ONC_AUTH_STAT_MAX) {
            r.status = ONC_ENC_BAD_DESCRIPTOR; return r;
        }
        hw = root == ONC_ROOT_AUTH_ERROR ? 1
                                         : (root == ONC_ROOT_MESSAGE_TYPE ? 2 : (root == ONC_ROOT_REPLY_BODY ? 1 : 0)) + 1 +
                                               (d.stat == ONC_REJECT_RPC_MISMATCH ? 2 : 1);
    } else {
        r.status = ONC_ENC_BAD_DESCRIPTOR; return r;
    }
    if (body != 0 && !in_arena(d.payload_off, body, bd.payload_len)) { r.status = ONC_ENC_BAD_DESCRIPTOR; return r; }
    const uint64_t total = 4ull * hw + body;
    if (total & 0xFFFFFFFF80000000ull) { r.status = ONC_ENC_TOO_LONG; return r; }
    if (assoc_c > ONC_MAX_AUTH_LEN || assoc_v > ONC_MAX_AUTH_LEN) { r.status = ONC_ENC_AUTH_GT_200; return r; }
    r.len = total;
    r.meta = cw | (vw << 8) | (hw << 16);
    return r;
}

// The header words of `root` (a descriptor plan_root accepted), in write order.
template <class Sink>
__device__ __forceinline__ void put_root_words(const onc_msg& d, uint32_t len, const EncSrc& s, uint32_t root,
                                               Sink& out) {
    switch (root) {
        case ONC_ROOT_RPC_MESSAGE: put_header_words(d, len, s, out); return;
        case ONC_ROOT_MESSAGE_TYPE:
            out(bswap(uint32_t(d.msg_type)));
            if (d.msg_type == ONC_MSG_CALL) put_call_words(d, s, out);
            else put_reply_words(d, s, out);
            return;
        case ONC_ROOT_CALL_BODY: put_call_words(d, s, out); return;
        case ONC_ROOT_REPLY_BODY: put_reply_words(d, s, out); return;
        case ONC_ROOT_ACCEPTED_REPLY:
            put_auth_words(d.verf, s, out);
            put_accepted_status_words(d, out);
            return;
        case ONC_ROOT_ACCEPTED_STATUS: put_accepted_status_words(d, out); return;
        case ONC_ROOT_REJECTED_REPLY: put_rejected_words(d, out); return;
        case ONC_ROOT_AUTH_ERROR: out(bswap(uint32_t(d.auth_stat))); return;
        case ONC_ROOT_AUTH_FLAVOR: put_auth_words(d.cred, s, out); return;
        case ONC_ROOT_AUTH_UNIX_PARAMS: put_unix_words<false>(d.cred.ref, s, out); return;
        default: put_opaque_words(d.cred, s, out); return;    // ONC_ROOT_OPAQUE
    }
}

// ---------------------------------------------------------------------------
// Cross-lane primitives on DPP / readlane (no LDS round trip)
// ---------------------------------------------------------------------------
// DPP controls (GFX9 encoding): row_shr:n = 0x110 + n, wave_shl:1 = 0x130,
// row_bcast:15 = 0x142, row_bcast:31 = 0x143. Lanes whose source is out of
// range, or outside row_mask, read 0.
template <int kCtrl, int kRowMask = 0xF>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_update_dpp(0u, uint32_t(v), kCtrl, kRowMask, 0xF, true);
    const uint32_t hi = __builtin_amdgcn_update_dpp(0u, uint32_t(v >> 32), kCtrl, kRowMask, 0xF, true);
    return uint64_t(lo) | (uint64_t(hi) << 32);
}

// Inclusive prefix sum over the 64 lanes: Kogge-Stone within each row of 16
// (row_shr 1, 2, 4, 8), then the row totals carried by row_bcast:15 (rows 1,
// 3) and row_bcast:31 (rows 2, 3). Six DPP steps on VALU instead of six
// ds_bpermute round trips. Every lane must be active.
__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v) {
    v += dpp_u64<0x111>(v);
    v += dpp_u64<0x112>(v);
    v += dpp_u64<0x114>(v);
    v += dpp_u64<0x118>(v);
    v += dpp_u64<0x142, 0xA>(v);
    v += dpp_u64<0x143, 0xC>(v);
    return v;
}

// Value of lane l (wave-uniform l) in every lane: v_readlane into SGPRs.
__device__ __forceinline__ uint64_t lane_u64(uint64_t v, int l) {
    return uint64_t(uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v)), l))) |
           (uint64_t(uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v >> 32)), l))) << 32);
}

// Lane i receives lane i + 1's value (lane 63 receives 0): DPP wave_shl:1.
__device__ __forceinline__ uint64_t next_lane_u64(uint64_t v) { return dpp_u64<0x130>(v); }

// ---------------------------------------------------------------------------
// Block-wide exclusive scan of u64 over 256 threads (4 waves)
// ---------------------------------------------------------------------------

// Returns the exclusive prefix of v within the block; *total = block sum.
template <int NT>
__device__ __forceinline__ uint64_t block_excl_scan_u64(uint64_t v, uint64_t* s_wave, uint64_t* total) {
    constexpr int NW = NT / 64;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t incl = wave_incl_scan_u64(v);
    if (lane == 63) s_wave[wave] = incl;
    __syncthreads();
    uint64_t wave_base = 0, sum = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        const uint64_t t = s_wave[w];
        if (w < wave) wave_base += t;
        sum += t;
    }
    *total = sum;
    __syncthreads();   // s_wave may be reused by the caller
    return wave_base + incl - v;
}

}  // namespace onc
