// decode.hip — batch RpcMessage::try_from for gfx950.
//
// Reference decoders, one message per buffer:
//   slice mode  RpcMessage::try_from(&[u8])  src/rpc_message.rs:235-271
//   Bytes mode  RpcMessage::try_from(Bytes)  src/rpc_message.rs:273-314
// with the reader chains of call_body.rs:37-69 / :181-209,
// auth/flavor.rs:52-94 / :190-222, auth/unix_params.rs:90-129 / :252-276,
// opaque.rs:72-98, bytes_ext.rs:17-42 and reply/*.
//
// One lane per record runs the reference's recursive descent as a flat
// state machine over the record's bytes [rec_off[i], rec_off[i+1]). The
// decode is zero-copy like the reference: opaque bodies and payloads are
// returned as (wire offset, length), never moved. The first error wins, in
// the reference's check order, per mode; the two modes differ only where
// the reference does (short reads: IOError vs InvalidLength; AUTH_UNIX is
// parsed inside its length-bounded slice in Bytes mode).
#include "common.h"
#include "kernels.h"

namespace onc {

// Each record's 16-byte-aligned window is pulled into LDS in two rounds of
// dwordx4 loads (one memory latency per round instead of one per field):
// first up to kWin1 chunks (64 B: the whole header of an AUTH_NONE call),
// then, only for records whose header reaches further (the credential length
// read from the first round), up to kWinChunks chunks (160 B: an AUTH_UNIX
// call with 16 gids and a 16-byte machine name). The wave loads its records'
// chunks cooperatively — lanes over a record's granules, handed over through
// LDS (load_round1, load_round2_coop) — and each lane stages its own record.
// The window is laid out [word][lane] so that lanes parsing the same field
// hit distinct banks. Reads past what was loaded fall back to global loads.
#ifndef ONC_DEC_WIN
#define ONC_DEC_WIN 10
#endif
#ifndef ONC_DEC_COOP
#define ONC_DEC_COOP 1      // round 1 loaded cooperatively (load_round1)
#endif
#ifndef ONC_DEC_COOP2
#define ONC_DEC_COOP2 1     // round 2 too, under the standard policy (load_round2_coop)
#endif
constexpr uint32_t kWin1 = 4;                 // round-1 chunks (standard policy)
constexpr uint32_t kWin1L = 8;                // round-1 chunks at most (line policy, decode_kernel)
constexpr uint32_t kWinChunks = ONC_DEC_WIN;
static_assert(kWinChunks >= kWin1L, "round 1 stays inside the window");
constexpr uint32_t kWinWords = 4 * kWinChunks;
#ifndef ONC_DEC_TILE
#define ONC_DEC_TILE 64     // c1 decode 54.7 -> 50.2 us, c2 81 -> 78.6, c3 447 -> 468 vs 256 (profiles/lab_r02_dec_tile.log)
#endif
constexpr int kDecTile = ONC_DEC_TILE;
constexpr uint32_t kSlotPass = 96;       // AUTH_UNIX slots staged per pass (9 KiB of the window)

// The window column holds the record's words aligned to the record: column
// word k = record bytes [4k, 4k + 4), whatever the record's byte offset in
// its first 16-byte granule (the loaded granules are stored shifted by that
// offset, each column word funnelled from two loaded words once, at staging)
// — every field read is one LDS read at a fixed offset. (Funnelling at each
// read instead cost the configs[2] decode 70 -> 55 us against a lab build
// that assumed aligned records.)
struct Rd {
    uintptr_t base;          // absolute address of record byte 0
    uint32_t lim;            // record bytes held by the window
    const uint32_t* col;     // this lane's window column (stride kDecTile words)

    // Big-endian u32 at record-relative position pos (pos % 4 == 0; all 4 bytes valid).
    __device__ __forceinline__ uint32_t be32(uint32_t pos) const {
        if (pos + 4u <= lim) return bswap(col[(pos >> 2) * kDecTile]);
        return bswap(load4(base + pos));
    }

    // n (<= 16) consecutive words from record position pos into out[0..n),
    // zeros after: straight from the window (16 LDS reads at fixed offsets)
    // when all of them lie in it, else word by word.
    __device__ __forceinline__ void words16(uint32_t pos, uint32_t n, uint32_t out[ONC_MAX_GIDS]) const {
        if (pos + 4u * n <= lim) {
            const uint32_t* p = col + (pos >> 2) * kDecTile;
#pragma unroll
            for (uint32_t g = 0; g < ONC_MAX_GIDS; ++g) out[g] = g < n ? bswap(p[g * kDecTile]) : 0u;
        } else {
#pragma unroll
            for (uint32_t g = 0; g < ONC_MAX_GIDS; ++g) out[g] = g < n ? be32(pos + 4u * g) : 0u;
        }
    }
};

#define ONC_RD(var)                                   \
    do {                                              \
        if (pos + 4u > end) return kShort;            \
        var = R.be32(pos);                            \
        pos += 4u;                                    \
    } while (0)

template <int MODE>
struct Rules {
    // Short read: Cursor::read_exact -> IOError(UnexpectedEof) (errors.rs:99-103)
    // vs BytesReaderExt::try_u32 -> InvalidLength (bytes_ext.rs:18-20).
    static constexpr int32_t kShort = MODE == ONC_DECODE_BYTES ? ONC_ERR_INVALID_LENGTH : ONC_ERR_IO_UNEXPECTED_EOF;
};

// Output stores: the decoded descriptors (staged through LDS, 4 KiB
// contiguous per workgroup), the AUTH_UNIX slots (compacted per workgroup,
// staged) and the status / aux arrays fill whole lines and are stored
// nontemporally — the decoder never reads them back, and plain stores leave
// dirty lines for the next kernel to write back (measured: c1 step +2-3 %,
// c3 +2 %; tools/store_lab.hip for the mechanism).
// AUTH_UNIX parameters of a record's credential (k = 0) and verifier
// (k = 1), held in registers until the record is parsed, then written out
// (see the end of decode_kernel): 24 words per slot in onc_unix_params order.
struct UnixSlots {
    uint32_t w[2][24];
    uint32_t mask;      // bit k: slot k holds parameters
};
__device__ __forceinline__ void put_unix(UnixSlots& us, uint64_t slot, uint32_t stamp, uint32_t uid, uint32_t gid,
                                         uint32_t ng, uint64_t name_off, uint32_t nl, const uint32_t* gids) {
    const int k = int(slot & 1);
    us.w[k][0] = stamp;
    us.w[k][1] = uid;
    us.w[k][2] = gid;
    us.w[k][3] = ng;
    us.w[k][4] = uint32_t(name_off);
    us.w[k][5] = uint32_t(name_off >> 32);
    us.w[k][6] = nl;
    us.w[k][7] = 0u;
#pragma unroll
    for (int g = 0; g < 16; ++g) us.w[k][8 + g] = gids[g];
    us.mask |= 1u << k;
}

// Slice mode AuthFlavor::from_cursor (flavor.rs:52-94) with
// AuthUnixParams::from_cursor (unix_params.rs:90-129) and
// Opaque::from_wire (opaque.rs:72-98; bound = the whole message, `end`).
template <class RdT>
__device__ __forceinline__ int32_t auth_slice(const RdT& R, uint32_t& pos, uint32_t end, uint64_t rec_off,
                                              uint64_t slot, onc_auth& a, UnixSlots& us) {
    constexpr int32_t kShort = Rules<ONC_DECODE_SLICE>::kShort;
    uint32_t fl;
    ONC_RD(fl);
    a.id = fl;
    if (fl == ONC_AUTH_UNIX) {
        uint32_t n;
        ONC_RD(n);
        if (n > ONC_MAX_AUTH_LEN) return ONC_ERR_INVALID_LENGTH;           // flavor.rs:83-85
        const uint32_t start = pos;
        uint32_t stamp, nl, uid, gid, ng;
        ONC_RD(stamp);
        ONC_RD(nl);
        if (nl > ONC_MAX_MACHINE_NAME_LEN) return ONC_ERR_INVALID_LENGTH;   // opaque.rs:77-79
        if (uint64_t(pos) + nl + pad4(nl) > end) return ONC_ERR_INVALID_LENGTH;  // opaque.rs:87-90
        const uint32_t name_pos = pos;
        pos += nl + pad4(nl);
        ONC_RD(uid);
        ONC_RD(gid);
        ONC_RD(ng);
        if (ng > ONC_MAX_GIDS) return ONC_ERR_INVALID_AUTH_DATA;          // unix_params.rs:112
        // the gids: every short read among them is the same error, so one
        // bounds check stands for the reference's per-gid reads
        if (uint64_t(pos) + 4ull * ng > end) return kShort;
        uint32_t gids[ONC_MAX_GIDS];
        R.words16(pos, ng, gids);
        pos += 4u * ng;
        if (pos - start != n) return ONC_ERR_INVALID_AUTH_DATA;          // unix_params.rs:117-119
        put_unix(us, slot, stamp, uid, gid, ng, rec_off + name_pos, nl, gids);
        a.kind_len = ONC_AUTH_PACK(ONC_KIND_UNIX, n);     // ABI 6: the declared length (= serialised_len)
        a.ref = slot;
        return ONC_OK;
    }
    uint32_t n;
    ONC_RD(n);
    if (n > ONC_MAX_AUTH_LEN) return ONC_ERR_INVALID_LENGTH;
    if (uint64_t(pos) + n + pad4(n) > end) return ONC_ERR_INVALID_LENGTH;
    const uint32_t kind = fl == ONC_AUTH_NONE ? ONC_KIND_NONE : (fl == ONC_AUTH_SHORT ? ONC_KIND_SHORT : ONC_KIND_UNKNOWN);
    a.kind_len = ONC_AUTH_PACK(kind, n);
    a.ref = rec_off + pos;
    pos += n + pad4(n);
    return ONC_OK;
}

// Bytes mode AuthFlavor::try_from(Bytes) (flavor.rs:190-222): the body is
// first cut with try_array(200) (bytes_ext.rs:25-42); AUTH_UNIX is parsed
// inside that slice (unix_params.rs:252-276) and must fill it exactly.
template <class RdT>
__device__ __forceinline__ int32_t auth_bytes(const RdT& R, uint32_t& pos, uint32_t end, uint64_t rec_off,
                                              uint64_t slot, onc_auth& a, UnixSlots& us) {
    constexpr int32_t kShort = Rules<ONC_DECODE_BYTES>::kShort;
    uint32_t fl, n;
    ONC_RD(fl);
    ONC_RD(n);
    if (n > ONC_MAX_AUTH_LEN) return ONC_ERR_INVALID_LENGTH;
    if (uint64_t(n) + pad4(n) > end - pos) return ONC_ERR_INVALID_LENGTH;
    const uint32_t bstart = pos, bend = pos + n;
    pos += n + pad4(n);
    a.id = fl;
    if (fl == ONC_AUTH_UNIX) {
        uint32_t q = bstart;
        uint32_t stamp, nl, uid, gid, ng;
#define ONC_RDQ(var)                                           \
    do {                                                       \
        if (q + 4u > bend) return ONC_ERR_INVALID_LENGTH;      \
        var = R.be32(q);                                       \
        q += 4u;                                               \
    } while (0)
        ONC_RDQ(stamp);
        ONC_RDQ(nl);
        if (nl > ONC_MAX_MACHINE_NAME_LEN) return ONC_ERR_INVALID_LENGTH;
        if (uint64_t(nl) + pad4(nl) > bend - q) return ONC_ERR_INVALID_LENGTH;
        const uint32_t name_pos = q;
        q += nl + pad4(nl);
        ONC_RDQ(uid);
        ONC_RDQ(gid);
        ONC_RDQ(ng);
        if (ng > ONC_MAX_GIDS) return ONC_ERR_INVALID_AUTH_DATA;
        if (uint64_t(q) + 4ull * ng > bend) return ONC_ERR_INVALID_LENGTH;   // every gid's try_u32 fails alike
        uint32_t gids[ONC_MAX_GIDS];
        R.words16(q, ng, gids);
        q += 4u * ng;
#undef ONC_RDQ
        // params.serialised_len() != auth_data.len() -> InvalidAuthData (flavor.rs:204-208)
        if (20u + nl + pad4(nl) + 4u * ng != n) return ONC_ERR_INVALID_AUTH_DATA;
        put_unix(us, slot, stamp, uid, gid, ng, rec_off + name_pos, nl, gids);
        a.kind_len = ONC_AUTH_PACK(ONC_KIND_UNIX, n);     // ABI 6: the declared length (= serialised_len)
        a.ref = slot;
        return ONC_OK;
    }
    const uint32_t kind = fl == ONC_AUTH_NONE ? ONC_KIND_NONE : (fl == ONC_AUTH_SHORT ? ONC_KIND_SHORT : ONC_KIND_UNKNOWN);
    a.kind_len = ONC_AUTH_PACK(kind, n);
    a.ref = rec_off + bstart;
    return ONC_OK;
}

template <int MODE, class RdT>
__device__ __forceinline__ int32_t auth_any(const RdT& R, uint32_t& pos, uint32_t end, uint64_t rec_off,
                                            uint64_t slot, onc_auth& a, UnixSlots& us) {
    if (MODE == ONC_DECODE_BYTES) return auth_bytes(R, pos, end, rec_off, slot, a, us);
    return auth_slice(R, pos, end, rec_off, slot, a, us);
}

// RpcMessage::try_from (rpc_message.rs:243-271 / :277-313), flattened.
template <int MODE, class RdT>
__device__ __forceinline__ int32_t parse_record(const RdT& R, uint64_t L, uint64_t rec_off, uint64_t i,
                                                onc_msg& m, uint32_t& aux0, uint32_t& aux1,
                                                UnixSlots& us) {
    constexpr int32_t kShort = Rules<MODE>::kShort;
    // expected_message_len (rpc_message.rs:343-367) + exact-length check
    if (L < 4) return ONC_ERR_INCOMPLETE_HEADER;
    const uint32_t hdr = R.be32(0);
    if ((hdr & 0x80000000u) == 0) return ONC_ERR_FRAGMENTED;
    const uint32_t want = (hdr & 0x7FFFFFFFu) + 4u;
    if (L != want) {
        aux0 = uint32_t(L);
        aux1 = want;
        return ONC_ERR_INCOMPLETE_MESSAGE;
    }
    const uint32_t end = want;
    uint32_t pos = 4;
    uint32_t v;
    ONC_RD(m.xid);
    ONC_RD(v);
    if (v == ONC_MSG_CALL) {
        m.msg_type = ONC_MSG_CALL;
        uint32_t rv;
        ONC_RD(rv);
        if (rv != 2u) {                                    // call_body.rs:39-42
            aux0 = rv;
            return ONC_ERR_INVALID_RPC_VERSION;
        }
        ONC_RD(m.u.call.program);
        ONC_RD(m.u.call.program_version);
        ONC_RD(m.u.call.procedure);
        int32_t st = auth_any<MODE>(R, pos, end, rec_off, 2 * i, m.cred, us);
        if (st != ONC_OK) return st;
        st = auth_any<MODE>(R, pos, end, rec_off, 2 * i + 1, m.verf, us);
        if (st != ONC_OK) return st;
        m.payload_off = rec_off + pos;                     // call_body.rs:53-59 (zero copy)
        m.payload_len = end - pos;
        return ONC_OK;                                     // serialised_len == L for every call
    }
    if (v != ONC_MSG_REPLY) {
        aux0 = v;
        return ONC_ERR_INVALID_MESSAGE_TYPE;               // rpc_message.rs:43
    }
    m.msg_type = ONC_MSG_REPLY;
    ONC_RD(v);
    if (v == ONC_REPLY_ACCEPTED) {
        m.reply_stat = ONC_REPLY_ACCEPTED;
        const int32_t st = auth_any<MODE>(R, pos, end, rec_off, 2 * i + 1, m.verf, us);
        if (st != ONC_OK) return st;
        ONC_RD(v);
        m.stat = uint8_t(v);
        switch (v) {                                       // accepted_reply.rs:158-174
            case ONC_ACCEPT_SUCCESS:
                m.payload_off = rec_off + pos;
                m.payload_len = end - pos;
                pos = end;
                break;
            case ONC_ACCEPT_PROG_UNAVAIL:
            case ONC_ACCEPT_PROC_UNAVAIL:
            case ONC_ACCEPT_GARBAGE_ARGS:
            case ONC_ACCEPT_SYSTEM_ERR:
                break;
            case ONC_ACCEPT_PROG_MISMATCH:
                ONC_RD(m.u.mismatch.low);
                ONC_RD(m.u.mismatch.high);
                break;
            default:
                aux0 = v;
                return ONC_ERR_INVALID_REPLY_STATUS;
        }
    } else if (v == ONC_REPLY_DENIED) {
        m.reply_stat = ONC_REPLY_DENIED;
        ONC_RD(v);
        m.stat = uint8_t(v);
        if (v == ONC_REJECT_RPC_MISMATCH) {                // rejected_reply.rs:46-57
            ONC_RD(m.u.mismatch.low);
            ONC_RD(m.u.mismatch.high);
        } else if (v == ONC_REJECT_AUTH_ERROR) {
            ONC_RD(v);
            if (v > ONC_AUTH_STAT_MAX) {                   // rejected_reply.rs:187
                aux0 = v;
                return ONC_ERR_INVALID_AUTH_ERROR;
            }
            m.auth_stat = uint8_t(v);
        } else {
            aux0 = v;
            return ONC_ERR_INVALID_REJECTED_REPLY_TYPE;
        }
    } else {
        aux0 = v;
        return ONC_ERR_INVALID_REPLY_TYPE;                 // reply_body.rs:33
    }
    // serialised_len() of a reply == bytes consumed; trailing bytes are
    // IncompleteMessage{buffer_len, expected} (rpc_message.rs:261-267).
    if (pos != end) {
        aux0 = uint32_t(L);
        aux1 = pos;
        return ONC_ERR_INCOMPLETE_MESSAGE;
    }
    return ONC_OK;
}

// ---------------------------------------------------------------------------
// Body-level roots (onc_decode_body, ONC_ROOT_*): the TryFrom of one type of
// the message tree over the whole record — no record-marking header, no
// trailing-bytes check (the reference's body decoders return what they
// parsed); `consumed` = the cursor's final position. Bound of every opaque:
// the record (the Cursor / Bytes covers exactly the slice given).
// ---------------------------------------------------------------------------

// AuthUnixParams::from_cursor(r, expected_len) (unix_params.rs:90-129, slice)
// / AuthUnixParams::try_from(Bytes) (:252-276: no consumed check).
template <int MODE>
__device__ __forceinline__ int32_t unix_params_root(const Rd& R, uint32_t& pos, uint32_t end, uint64_t rec_off,
                                                    uint64_t slot, uint32_t expected, UnixSlots& us) {
    constexpr int32_t kShort = Rules<MODE>::kShort;
    const uint32_t start = pos;
    uint32_t stamp, nl, uid, gid, ng;
    ONC_RD(stamp);
    ONC_RD(nl);                                                           // opaque.rs:76 / bytes_ext.rs:26
    if (nl > ONC_MAX_MACHINE_NAME_LEN) return ONC_ERR_INVALID_LENGTH;
    if (uint64_t(pos) + nl + pad4(nl) > end) return ONC_ERR_INVALID_LENGTH;
    const uint32_t name_pos = pos;
    pos += nl + pad4(nl);
    ONC_RD(uid);
    ONC_RD(gid);
    ONC_RD(ng);
    if (ng > ONC_MAX_GIDS) return ONC_ERR_INVALID_AUTH_DATA;             // unix_params.rs:112 / :266
    if (uint64_t(pos) + 4ull * ng > end) return kShort;                  // every short gid read alike
    uint32_t gids[ONC_MAX_GIDS];
    R.words16(pos, ng, gids);
    pos += 4u * ng;
    if (MODE == ONC_DECODE_SLICE && pos - start != expected) return ONC_ERR_INVALID_AUTH_DATA;   // :117-119
    put_unix(us, slot, stamp, uid, gid, ng, rec_off + name_pos, nl, gids);
    return ONC_OK;
}

template <int MODE>
__device__ __forceinline__ int32_t parse_root(const Rd& R, uint32_t end, uint64_t rec_off, uint64_t i, uint32_t root,
                                              uint32_t param, onc_msg& m, uint32_t& aux0, UnixSlots& us,
                                              uint32_t& consumed) {
    constexpr int32_t kShort = Rules<MODE>::kShort;
    uint32_t pos = 0, v;
    if (root == ONC_ROOT_AUTH_FLAVOR || root == ONC_ROOT_AUTH_UNIX_PARAMS || root == ONC_ROOT_OPAQUE) {
        m.msg_type = ONC_MSG_CALL;
        int32_t st;
        if (root == ONC_ROOT_AUTH_FLAVOR) {                    // flavor.rs:177-184 / :186-222
            st = auth_any<MODE>(R, pos, end, rec_off, 2 * i, m.cred, us);
        } else if (root == ONC_ROOT_AUTH_UNIX_PARAMS) {
            st = unix_params_root<MODE>(R, pos, end, rec_off, 2 * i, param, us);
            m.cred.id = ONC_AUTH_UNIX;
            m.cred.kind_len = ONC_AUTH_PACK(ONC_KIND_UNIX, pos);   // serialised_len (cursor from 0)
            m.cred.ref = 2 * i;
        } else {                                               // opaque.rs:72-98 / bytes_ext.rs:25-42
            const uint32_t max_len = min(param, ONC_OPAQUE_MAX_LEN);
            uint32_t n;
            ONC_RD(n);
            if (n > max_len) return ONC_ERR_INVALID_LENGTH;
            if (uint64_t(pos) + n + pad4(n) > end) return ONC_ERR_INVALID_LENGTH;
            m.cred.kind_len = ONC_AUTH_PACK(ONC_KIND_NONE, n);
            m.cred.ref = rec_off + pos;
            pos += n + pad4(n);
            st = ONC_OK;
        }
        consumed = pos;
        return st;
    }
    uint32_t node = root;
    if (node == ONC_ROOT_MESSAGE_TYPE) {                       // rpc_message.rs:39-45 / :84-92
        ONC_RD(v);
        if (v == ONC_MSG_CALL) node = ONC_ROOT_CALL_BODY;
        else if (v == ONC_MSG_REPLY) node = ONC_ROOT_REPLY_BODY;
        else { aux0 = v; return ONC_ERR_INVALID_MESSAGE_TYPE; }
    }
    if (node == ONC_ROOT_CALL_BODY) {                          // call_body.rs:37-69 / :181-209
        m.msg_type = ONC_MSG_CALL;
        uint32_t rv;
        ONC_RD(rv);
        if (rv != 2u) { aux0 = rv; return ONC_ERR_INVALID_RPC_VERSION; }
        ONC_RD(m.u.call.program);
        ONC_RD(m.u.call.program_version);
        ONC_RD(m.u.call.procedure);
        int32_t st = auth_any<MODE>(R, pos, end, rec_off, 2 * i, m.cred, us);
        if (st != ONC_OK) return st;
        st = auth_any<MODE>(R, pos, end, rec_off, 2 * i + 1, m.verf, us);
        if (st != ONC_OK) return st;
        m.payload_off = rec_off + pos;
        m.payload_len = end - pos;
        consumed = end;
        return ONC_OK;
    }
    m.msg_type = ONC_MSG_REPLY;
    if (node == ONC_ROOT_REPLY_BODY) {                         // reply_body.rs:29-35 / :89-97
        ONC_RD(v);
        if (v == ONC_REPLY_ACCEPTED) node = ONC_ROOT_ACCEPTED_REPLY;
        else if (v == ONC_REPLY_DENIED) node = ONC_ROOT_REJECTED_REPLY;
        else { aux0 = v; return ONC_ERR_INVALID_REPLY_TYPE; }
    }
    if (node == ONC_ROOT_ACCEPTED_REPLY) {                     // accepted_reply.rs:35-40 / :92-104
        m.reply_stat = ONC_REPLY_ACCEPTED;
        const int32_t st = auth_any<MODE>(R, pos, end, rec_off, 2 * i + 1, m.verf, us);
        if (st != ONC_OK) return st;
        node = ONC_ROOT_ACCEPTED_STATUS;
    }
    if (node == ONC_ROOT_ACCEPTED_STATUS) {                    // accepted_reply.rs:158-186 / :247-264
        m.reply_stat = ONC_REPLY_ACCEPTED;
        ONC_RD(v);
        m.stat = uint8_t(v);
        switch (v) {
            case ONC_ACCEPT_SUCCESS:
                m.payload_off = rec_off + pos;
                m.payload_len = end - pos;
                pos = end;
                break;
            case ONC_ACCEPT_PROG_UNAVAIL:
            case ONC_ACCEPT_PROC_UNAVAIL:
            case ONC_ACCEPT_GARBAGE_ARGS:
            case ONC_ACCEPT_SYSTEM_ERR:
                break;
            case ONC_ACCEPT_PROG_MISMATCH:
                ONC_RD(m.u.mismatch.low);
                ONC_RD(m.u.mismatch.high);
                break;
            default:
                aux0 = v;
                return ONC_ERR_INVALID_REPLY_STATUS;
        }
        consumed = pos;
        return ONC_OK;
    }
    m.reply_stat = ONC_REPLY_DENIED;
    if (node == ONC_ROOT_REJECTED_REPLY) {                     // rejected_reply.rs:46-57 / :111-124
        ONC_RD(v);
        m.stat = uint8_t(v);
        if (v == ONC_REJECT_RPC_MISMATCH) {
            ONC_RD(m.u.mismatch.low);
            ONC_RD(m.u.mismatch.high);
            consumed = pos;
            return ONC_OK;
        }
        if (v != ONC_REJECT_AUTH_ERROR) { aux0 = v; return ONC_ERR_INVALID_REJECTED_REPLY_TYPE; }
    }
    // AuthError (rejected_reply.rs:176-190 / :219-235)
    m.stat = ONC_REJECT_AUTH_ERROR;
    ONC_RD(v);
    if (v > ONC_AUTH_STAT_MAX) { aux0 = v; return ONC_ERR_INVALID_AUTH_ERROR; }
    m.auth_stat = uint8_t(v);
    consumed = pos;
    return ONC_OK;
}
#undef ONC_RD

// decode_kernel: lane per record. The 64-byte descriptors of the
// workgroup's 256 records are staged in LDS and written out as 16 KiB of
// contiguous dwordx4 stores (1 KiB per wave instruction, whole 128-byte
// lines) instead of four scattered 16-byte stores per lane.
// kExact (the product): the first round loads only the chunks holding the
// record's first 44 bytes (the shortest Call header: AUTH_NONE credential
// and verifier; every Reply header with an AUTH_NONE verifier is shorter)
// instead of a fixed 64-byte window, so fewer 128-byte lines are fetched per
// record: the decode is bound by the count of scattered line fetches
// (tools/dec_lab.hip: 1 / 2 / 3 / 4 chunks per record, 1M records 300 B
// apart, cold: 53 / 59 / 65 / 71 us — ~53 us per million lines). Measured
// c1 decode 59.6 -> 56.0 us, c2 90.1 -> 88.5 us, c3 unchanged.
// kFromLen (onc_decode_lengths): the record's offset comes from the lengths
// inside the kernel — the byte totals of the 4096-record blocks before this
// workgroup's (summed here, or their scan beyond kDecLenFusedBlocks blocks),
// the totals of the workgroups before it in its block and a wave scan of its
// own lengths, all loads issued together — instead of an offsets pass over
// the whole batch (onc_scan_lengths: 8 bytes written and read back per
// record, one launch more).
static_assert(kDecTile == 64, "kFromLen: one wave per workgroup, 64 workgroup totals per block");
// kRoot (onc_decode_body): a.root selects the decoded type; the window
// takes the record's first kWinChunks chunks in two rounds (the header-extent
// guess below is the RpcMessage layout's).
// The line policy (message decode, kLine). A header longer than the first
// round re-fetches, in round 2, the 128-byte line round 1 read — by then that
// line has left L2 (configs[3]: 128-byte AUTH_UNIX headers 1152 bytes apart,
// 270 B fetched per record for one line of header). Round 1 can instead take
// the rest of the record's first line (no extra line): that saves the second
// fetch when headers are long and costs load issue when they are not — the
// decode's time follows its scattered load instructions (c3 decode 367 -> 257
// us, c0 85 -> 80, but c1 50.5 -> 64.5, c2 58 -> 61;
// profiles/lab_r03_decode_line.log). So the policy is chosen per launch
// (codec.hip launch_decode) from the records the previous launch on the same
// codec saw: every 64th workgroup stores how many of its 64 records needed a
// second round under the standard policy into the codec's hint word, which
// lives in mapped host memory, so the host reads it at the next launch
// without a synchronisation and launches the kernel instance of that policy
// (kLine1Min, kernels.h; break-even measured at ~1/3) — no policy code in
// either kernel. A device-memory word read by every workgroup cost the c1
// decode 1-2 us of prologue; results never depend on the policy (only which
// chunks each round loads); onc_codec_set_decode_policy pins either (tests).

// Round 1 of a record's window (L != 0): the chunks it takes under the
// policy. avail: the record's chunks inside the window; r44: the standard
// round (the first 44 bytes).
template <bool kLine, bool kPolicy>
__device__ __forceinline__ uint32_t round1_chunks(uintptr_t win, uint32_t q0, uint64_t L, uint32_t& avail,
                                                  uint32_t& r44) {
    avail = uint32_t(min(uint64_t(kWinChunks), (q0 + L + 15) >> 4));
    r44 = kPolicy ? uint32_t(min(uint64_t(kWin1), (q0 + min(L, uint64_t(44)) + 15) >> 4)) : kWin1;
    // line policy: also the rest of the record's first 128-byte line, and
    // at least the record's first 128 bytes (a record starting inside a line
    // takes the next line in round 1 too: configs[0]'s 128-byte headers 192
    // bytes apart, half of them across a line boundary)
    const uint32_t rln = uint32_t((((win | 127u) + 1u) - win) >> 4);
    const uint32_t r128 = uint32_t((q0 + min(L, uint64_t(128)) + 15) >> 4);
    const uint32_t r1 = kLine ? min(kWin1L, max(max(r44, rln), r128)) : r44;
    return min(r1, avail);
}

// Round 1's loads for the whole wave (every lane, nch = 0 for a lane with no
// record). They go through a buffer resource based at the first record's
// window when every window lies within 2 GiB above it (records back to
// back: always, short of multi-GiB records): a chunk past a record's round
// gets an out-of-range offset, so its load returns zeros without a memory
// request (it used to re-read the record's last granule: a second request
// on a mapped host wire on some hosts, profiles/lab_r06_decode_buffer_round1.log).
// kCoop: the lanes load the wave's records granule by granule — lane t of
// instruction k takes granule t % G of record k * (64 / G) + t / G, so one
// instruction reads 64 / G records' windows contiguously — and hand them
// over through LDS: over PCIe the link then sees a record's round as one
// contiguous request rather than G (tools/link_lab.hip coop rows).
// No branch separates the loads: under branches the compiler waited for
// chunk 2 before issuing chunk 3.
template <bool kLine, bool kCoop>
__device__ __forceinline__ void load_round1(uint32_t* s_win, int t, uintptr_t win, uint32_t nch, u32x4 (&v)[kWin1L]) {
    constexpr uint32_t G = kLine ? kWin1L : kWin1;
    static_assert(kWin1 == 4 && kWin1L == 8, "pin lists below");
    static_assert(kDecTile == 64, "one wave per workgroup: the hand-over needs no workgroup barrier");
#pragma unroll
    for (uint32_t j = 0; j < kWin1L; ++j) v[j] = u32x4{0u, 0u, 0u, 0u};
    const uint64_t act = __ballot(nch != 0);
    if (act == 0) return;
    const int first = __builtin_ctzll(act);
    const uintptr_t rb = uintptr_t(__builtin_amdgcn_readlane(uint32_t(win), first)) |
                         (uintptr_t(__builtin_amdgcn_readlane(uint32_t(win >> 32), first)) << 32);
    const bool near = nch == 0 || (win >= rb && win - rb < (uintptr_t(1) << 31) - 256);
    const uint32_t wo = uint32_t(win - rb);
    if (__ballot(!near) == 0) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<void*>(rb), int16_t(0), int32_t(0x7FFFFFF0), int32_t(0x00020000));
        if constexpr (kCoop) {
            constexpr uint32_t R = 64 / G;                   // records per instruction
            u32x4 x[G];
#pragma unroll
            for (uint32_t k = 0; k < G; ++k) {
                const int r = int(k * R + uint32_t(t) / G);
                const uint32_t g = uint32_t(t) % G;
                const uint32_t wr = uint32_t(__shfl(int(wo), r));
                const uint32_t nr = uint32_t(__shfl(int(nch), r));
                x[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                     rs, g < nr ? wr + 16 * g : 0x80000000u, 0, 0));
            }
            // record r's granule g at raw[r * G + g] (the window is free
            // until staging; one wave per workgroup, LDS in issue order)
            u32x4* raw = reinterpret_cast<u32x4*>(s_win);
#pragma unroll
            for (uint32_t k = 0; k < G; ++k) raw[(k * R + uint32_t(t) / G) * G + uint32_t(t) % G] = x[k];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (uint32_t j = 0; j < G; ++j) v[j] = raw[uint32_t(t) * G + j];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        } else {
#pragma unroll
            for (uint32_t j = 0; j < G; ++j)
                v[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                     rs, j < nch ? wo + 16 * j : 0x80000000u, 0, 0));
        }
    } else if (nch != 0) {
        // windows too far apart for one resource: per-lane loads, chunks
        // past the round re-reading the record's last granule
        const uintptr_t last = win + 16 * (nch - 1);
#pragma unroll
        for (uint32_t j = 0; j < G; ++j) v[j] = gload<u32x4>(min(win + 16 * j, last));
    }
    if constexpr (kLine) {
        asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
                     "+v"(v[7]));
    } else {
        asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
    }
}

// Round 2 covers chunks [nch, want) from kR2 on (the first chunk round 1 may
// have skipped) up to the window's end.
template <bool kPolicy>
struct Round2 {
    static constexpr uint32_t kR2 = kPolicy ? 3u : kWin1;     // round 1 held >= 3 chunks if L >= 44
    static constexpr uint32_t kN2 = kWinChunks > kR2 ? kWinChunks - kR2 : 1;
};

// The window of one record (L != 0), round 1 loaded (v, nch: load_round1):
// round 1 staged in LDS and the header extent read from it. Returns the
// chunks the header needs (want; > nch: round 2); needs2: the header
// reaches past the standard policy's first round; last: round 1's last
// word, whose upper bytes round 2 brings. kLine: the line policy.
template <bool kLine, bool kPolicy, bool kRoot>
__device__ __forceinline__ uint32_t stage_round1(uint32_t* s_win, int t, uintptr_t base, uint32_t q0, uint32_t d0,
                                                 uint64_t L, bool& needs2, const u32x4 (&v)[kWin1L], uint32_t nch,
                                                 uint32_t avail, uint32_t r44, uint32_t& last) {
    // column word c = record bytes [4c, 4c + 4): loaded words d0 + c and
    // d0 + c + 1 funnelled by the record's byte offset in its dword. The
    // last word of the round (its upper bytes in the next chunk) is
    // rewritten if round 2 loads that chunk; otherwise it lies past `lim`.
    const uint32_t sh = q0 & 3u;
    uint32_t e[4 * kWin1L + 1];
#pragma unroll
    for (uint32_t j = 0; j < kWin1L; ++j) {
        e[4 * j] = v[j].x;
        e[4 * j + 1] = v[j].y;
        e[4 * j + 2] = v[j].z;
        e[4 * j + 3] = v[j].w;
    }
    e[4 * kWin1L] = 0u;
#pragma unroll
    for (uint32_t r = 0; r < 4 * kWin1; ++r)
        if (r >= d0 && r < 4 * nch) s_win[(r - d0) * kDecTile + t] = funnel(e[r], e[r + 1], sh);
    if constexpr (kLine) {
#pragma unroll
        for (uint32_t r = 4 * kWin1; r < 4 * kWin1L; ++r)       // r >= 16 > d0
            if (r < 4 * nch) s_win[(r - d0) * kDecTile + t] = funnel(e[r], e[r + 1], sh);
    }
    last = e[4 * kWin1L - 1];
#pragma unroll
    for (uint32_t c = 1; c < kWin1L; ++c)
        if (nch == c) last = e[4 * c - 1];
    // Header extent from the first round: call -> 36 + cred body + verf
    // flavor/length + the verifier body (its length when the first round
    // holds it, else a 16-byte guess); reply -> up to 12 bytes past an
    // accepted verifier.
    const Rd R1{base, 16 * nch - q0, &s_win[t]};
    uint32_t need = uint32_t(min(L, uint64_t(16 * kWinChunks)));
    if (!kRoot && L >= 36 && 16 * nch >= q0 + 36) {
        const uint32_t mt = R1.be32(8);
        if (mt == ONC_MSG_CALL) {
            const uint32_t cl = R1.be32(32);
            const uint32_t vpos = 36 + cl + pad4(cl) + 4;      // verifier length field
            if (cl > ONC_MAX_AUTH_LEN) {
                need = 36;
            } else if (q0 + vpos + 4 <= 16 * nch && vpos + 4 <= L) {
                const uint32_t vl = R1.be32(vpos);
                need = vpos + 4 + (vl <= ONC_MAX_AUTH_LEN ? vl + pad4(vl) : 0);
            } else {
                need = vpos + 4 + 16;
            }
        } else if (mt == ONC_MSG_REPLY) {
            const uint32_t vl = R1.be32(20);
            need = vl <= ONC_MAX_AUTH_LEN ? 24 + vl + pad4(vl) + 12 : 24;
        }
    }
    const uint32_t want = min(avail, (q0 + need + 15) >> 4);
    needs2 = want > min(r44, avail);
    return want;
}

// Round 2's loads for the whole wave, cooperatively (the standard policy:
// round 1 held 3 or 4 chunks, so a record's round 2 is at most 7): two
// passes of 4 slots, lane t of instruction k taking slot t % 4 of record
// 16 k + t / 4 — chunk nch + 4 p + slot when below want, else an
// out-of-range offset (no request) — handed over through LDS rows [16, 32)
// of the window (above round 1's staged rows). w[j - kR2] receives chunk j
// of the lane's record for j in [nch, want), zeros elsewhere.
template <bool kPolicy>
__device__ __forceinline__ void load_round2_coop(uint32_t* s_win, int t, uintptr_t win, uint32_t nch, uint32_t want,
                                                 u32x4 (&w)[Round2<kPolicy>::kN2]) {
    constexpr uint32_t kR2 = Round2<kPolicy>::kR2, kN2 = Round2<kPolicy>::kN2;
    static_assert(kR2 == 3 && kN2 == 7, "two passes of 4 slots cover round 2 after 3 or 4 round-1 chunks");
#pragma unroll
    for (uint32_t j = 0; j < kN2; ++j) w[j] = u32x4{0u, 0u, 0u, 0u};
    const bool r2 = want > nch;
    const uint64_t act = __ballot(r2);
    if (act == 0) return;
    const int first = __builtin_ctzll(act);
    const uintptr_t rb = uintptr_t(__builtin_amdgcn_readlane(uint32_t(win), first)) |
                         (uintptr_t(__builtin_amdgcn_readlane(uint32_t(win >> 32), first)) << 32);
    const bool near = !r2 || (win >= rb && win - rb < (uintptr_t(1) << 31) - 256);
    if (__ballot(!near) != 0) {                        // windows too far apart: per-lane loads
#pragma unroll
        for (uint32_t j = kR2; j < kWinChunks; ++j)
            if (j >= nch && j < want) w[j - kR2] = gload<u32x4>(win + 16 * j);
        return;
    }
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(rb), int16_t(0), int32_t(0x7FFFFFF0), int32_t(0x00020000));
    const uint32_t wo = uint32_t(win - rb);
    const uint32_t nw = r2 ? nch | (want << 8) : 0u;    // (nch, want) of the lane's record
    const uint32_t slot = uint32_t(t) & 3u;
    u32x4* raw = reinterpret_cast<u32x4*>(s_win + 16 * kDecTile);
    u32x4 g[8];
    const uint32_t passes = __ballot(r2 && want > nch + 4) ? 2u : 1u;   // wave-uniform
#pragma unroll
    for (uint32_t p = 0; p < 2; ++p) {
        g[4 * p] = g[4 * p + 1] = g[4 * p + 2] = g[4 * p + 3] = u32x4{0u, 0u, 0u, 0u};
        if (p < passes) {
            u32x4 x[4];
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
                const int r = int(16 * k + uint32_t(t) / 4);
                const uint32_t wr = uint32_t(__shfl(int(wo), r));
                const uint32_t q = uint32_t(__shfl(int(nw), r));
                const uint32_t j = (q & 0xFFu) + 4 * p + slot;
                x[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                     rs, j < (q >> 8) ? wr + 16 * j : 0x80000000u, 0, 0));
            }
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) raw[4 * (16 * k + uint32_t(t) / 4) + slot] = x[k];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (uint32_t m = 0; m < 4; ++m) g[4 * p + m] = raw[4 * uint32_t(t) + m];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    // slot m holds chunk nch + m: w[i] = chunk kR2 + i = slot i + kR2 - nch
    // (nch is 3 or 4 for a record with a round 2)
    if (r2) {
#pragma unroll
        for (uint32_t i = 0; i < kN2; ++i) w[i] = nch == kR2 ? g[i] : (i ? g[i - 1] : u32x4{0u, 0u, 0u, 0u});
    }
}

// Round 2 of one record's window (want > nch): chunks [nch, want) staged
// from w (loaded here when !kPre), and round 1's last word completed.
// Returns the chunks staged (want).
template <bool kPolicy, bool kPre>
__device__ __forceinline__ uint32_t stage_round2(uint32_t* s_win, int t, uintptr_t win, uint32_t q0, uint32_t d0,
                                                 uint32_t nch, uint32_t want, uint32_t last,
                                                 u32x4 (&w)[Round2<kPolicy>::kN2]) {
    constexpr uint32_t kR2 = Round2<kPolicy>::kR2, kN2 = Round2<kPolicy>::kN2;
    const uint32_t sh = q0 & 3u;
    if constexpr (!kPre) {
#pragma unroll
        for (uint32_t j = 0; j < kN2; ++j) w[j] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
        for (uint32_t j = kR2; j < kWinChunks; ++j)
#if defined(ONC_LAB_NO_R2)
            (void)0;                     // lab build only (wrong results): what round 2's loads cost
#else
            if (j >= nch && j < want) w[j - kR2] = gload<u32x4>(win + 16 * j);
#endif
    }
    uint32_t f[4 * kN2 + 1];
#pragma unroll
    for (uint32_t j = 0; j < kN2; ++j) {
        f[4 * j] = w[j].x;
        f[4 * j + 1] = w[j].y;
        f[4 * j + 2] = w[j].z;
        f[4 * j + 3] = w[j].w;
    }
    f[4 * kN2] = 0u;
#pragma unroll
    for (uint32_t r = 4 * kR2; r < 4 * kWinChunks; ++r)       // r >= 12 > d0
        if (r >= 4 * nch && r < 4 * want) s_win[(r - d0) * kDecTile + t] = funnel(f[r - 4 * kR2], f[r - 4 * kR2 + 1], sh);
    // round 1's last word, now with its upper bytes (nch >= kR2 here)
    uint32_t hi = w[0].x;
#pragma unroll
    for (uint32_t c = kR2; c < kWin1L; ++c)
        if (nch == c) hi = w[c - kR2].x;
    if (nch == kWin1L && kWin1L - kR2 < kN2) hi = w[kWin1L - kR2].x;
    s_win[(4 * nch - 1 - d0) * kDecTile + t] = funnel(last, hi, sh);
    return want;
}

template <int MODE, bool kExact = false, bool kNTOut = false, bool kFromLen = false, bool kBlkFused = false,
          bool kRoot = false, bool kLine = false>
__global__ __launch_bounds__(kDecTile) void decode_kernel(DecArgs a) {
    __shared__ uint32_t s_win[kWinWords * kDecTile];
    static_assert(kWinWords * kDecTile * 4 >= kDecTile * sizeof(onc_msg), "descriptor staging reuses the window");
    const int t = threadIdx.x;
    const uint64_t i0 = uint64_t(blockIdx.x) * kDecTile;
    const uint64_t i = i0 + t;
    const bool valid = i < a.n;
    constexpr bool kPolicy = kExact && !kRoot;
    bool needs2 = false;                           // a second round under the standard policy
    uint64_t b = 0, L = 0;
    if constexpr (kFromLen) {
        const uint64_t wg = blockIdx.x;
        const uint64_t blk = wg / (kDecLenBlk / kDecTile);
        const uint64_t w0 = blk * (kDecLenBlk / kDecTile);
        // every prologue load issued unconditionally (clamped indices) and
        // pinned, then masked: one memory round trip (loads under
        // per-lane branches made the compiler wait for the length before
        // issuing the totals: two)
        const uint64_t nwg = (a.n + kDecTile - 1) / kDecTile;
        const auto clamp = [](uint64_t x, uint64_t hi) { return x < hi ? x : hi; };
        uint32_t len = a.rec_len[clamp(i, a.n - 1)];
        uint64_t ts = a.tile_sum[clamp(w0 + t, nwg - 1)];
        constexpr int kPre = kBlkFused ? int(kDecLenFusedBlocks / 64) : 1;
        uint64_t pv[kPre];
#pragma unroll
        for (int k = 0; k < kPre; ++k)
            pv[k] = kBlkFused ? a.blk_sum[clamp(uint64_t(t) + 64ull * k, a.nblk - 1)] : a.blk_base[blk];
        static_assert(kPre == 1 || kPre == 8, "pin list below");
        if constexpr (kPre == 8)
            asm volatile("" : "+v"(len), "+v"(ts), "+v"(pv[0]), "+v"(pv[1]), "+v"(pv[2]), "+v"(pv[3]), "+v"(pv[4]),
                         "+v"(pv[5]), "+v"(pv[6]), "+v"(pv[7]));
        else
            asm volatile("" : "+v"(len), "+v"(ts), "+v"(pv[0]));
        len = valid ? len : 0u;
        ts = w0 + t < wg ? ts : 0;
        uint64_t pre = 0;
        if constexpr (kBlkFused) {
#pragma unroll
            for (int k = 0; k < kPre; ++k) pre += uint64_t(t) + 64ull * k < blk ? pv[k] : 0;
        } else {
            pre = t == 0 ? pv[0] : 0;
        }
        const uint64_t incl = wave_incl_scan_u64(uint64_t(len));
        const uint64_t wbase = a.base + lane_u64(wave_incl_scan_u64(pre + ts), 63);
        b = wbase + incl - len;
        L = len;
        if (a.rec_off_out && valid) {
            a.rec_off_out[i] = b;
            if (i + 1 == a.n) a.rec_off_out[a.n] = b + L;
        }
    } else if (valid) {
        b = a.rec_off[i];
        L = a.rec_off[i + 1] - b;
    }
    const uintptr_t wire = reinterpret_cast<uintptr_t>(a.wire);
    const uintptr_t base = wire + b;
    const uintptr_t win = base & ~uintptr_t(15);
    const uint32_t q0 = uint32_t(base - win);
    const uint32_t d0 = q0 >> 2;                      // record byte 0's dword in its first granule
    // Stage the window. Chunks past the record's last byte are not loaded;
    // empty records read nothing.
    constexpr bool kLineP = kLine && kPolicy;
    uint32_t nch = 0, avail = 0, r44 = 0;
    if (L != 0) nch = round1_chunks<kLineP, kPolicy>(win, q0, L, avail, r44);
    u32x4 v1[kWin1L];
    load_round1<kLineP, ONC_DEC_COOP>(s_win, t, win, nch, v1);
    uint32_t want = 0, last = 0;
    if (L != 0) want = stage_round1<kLineP, kPolicy, kRoot>(s_win, t, base, q0, d0, L, needs2, v1, nch, avail, r44, last);
    // round 2 (headers longer than round 1): cooperative under the standard
    // policy (the whole wave), else per lane
    constexpr bool kCoop2 = ONC_DEC_COOP2 && kPolicy && !kLineP;
    u32x4 w2[Round2<kPolicy>::kN2];
    if constexpr (kCoop2) load_round2_coop<kPolicy>(s_win, t, win, nch, want, w2);
    if (L != 0 && want > nch) nch = stage_round2<kPolicy, kCoop2>(s_win, t, win, q0, d0, nch, want, last, w2);
    if constexpr (kPolicy) {
        // every 64th workgroup reports for the next launch how many of its
        // records needed a second round under the standard policy
        const uint32_t cnt = uint32_t(__popcll(__ballot(needs2)));
        if (a.hint && (blockIdx.x & 63) == 0 && t == 0)
            __hip_atomic_store(a.hint, cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    const uint32_t lim = nch ? 16 * nch - q0 : 0u;
    const Rd R{base, lim, &s_win[t]};
    onc_msg m;
    uint4* mz = reinterpret_cast<uint4*>(&m);
#pragma unroll
    for (int k = 0; k < 4; ++k) mz[k] = make_uint4(0, 0, 0, 0);
    uint32_t aux0 = 0, aux1 = 0;
    int32_t st = ONC_OK;
    UnixSlots us;
    us.mask = 0;
    uint32_t consumed = 0;
    if (valid) {
        if constexpr (kRoot) {
            // records of 4 GiB or more: their payload does not fit the
            // descriptor's 32-bit length
            if (a.root == ONC_ROOT_RPC_MESSAGE) {
                st = parse_record<MODE>(R, L, b, i, m, aux0, aux1, us);
                consumed = uint32_t(L);               // an RpcMessage is the whole record
            } else {
                st = L > 0xFFFFFFFFull ? ONC_ERR_INVALID_LENGTH
                                       : parse_root<MODE>(R, uint32_t(L), b, i, a.root, a.param ? a.param[i] : 0u, m,
                                                          aux0, us, consumed);
            }
        } else {
            st = parse_record<MODE>(R, L, b, i, m, aux0, aux1, us);
        }
        if (st != ONC_OK) {
#pragma unroll
            for (int k = 0; k < 4; ++k) mz[k] = make_uint4(0, 0, 0, 0);
        }
        if (kRoot && a.consumed) a.consumed[i] = st == ONC_OK ? consumed : 0u;
        if (kNTOut) {
            __builtin_nontemporal_store(st, a.out.status + i);
            __builtin_nontemporal_store(aux0, a.out.aux0 + i);
            __builtin_nontemporal_store(aux1, a.out.aux1 + i);
        } else {
            a.out.status[i] = st;
            a.out.aux0[i] = aux0;
            a.out.aux1[i] = aux1;
        }
    }
    // AUTH_UNIX slots, compacted per 64-record group: the group's OK records'
    // parameter sets take consecutive slots from 2 * i0 (record order,
    // credential before verifier; onc_auth.ref names the slot), staged in the
    // window and written as whole contiguous lines with nontemporal stores.
    // Scattered slots (slot 2i / 2i + 1, lane by lane, 192 bytes apart) cost
    // the configs[2] decode ~20 of its 70 us for 24 % AUTH_UNIX records
    // (lab build without slot stores: 50.5 us; tools/line_lab.hip: 128 B at
    // 192 * i 21 us, compacted per lane 13 us).
    const bool okr = valid && st == ONC_OK;
    const uint64_t bc = __ballot(okr && (us.mask & 1u)), bv = __ballot(okr && (us.mask & 2u));
    const uint32_t nslots = uint32_t(__popcll(bc) + __popcll(bv));
    __syncthreads();                                  // every lane is done with its window
    if (nslots) {
        const uint64_t below = (1ull << t) - 1;
        const uint32_t rank = uint32_t(__popcll(bc & below) + __popcll(bv & below));
        const uint64_t sbase = 2 * i0;
        if (okr && (us.mask & 1u)) m.cred.ref = sbase + rank;
        if (okr && (us.mask & 2u)) m.verf.ref = sbase + rank + (us.mask & 1u);
        static_assert(kWinWords * kDecTile * 4 >= kSlotPass * sizeof(onc_unix_params), "slot staging fits the window");
        uint4* stg = reinterpret_cast<uint4*>(s_win);
        u32x4* dst = reinterpret_cast<u32x4*>(a.out.unix_params + sbase);
        for (uint32_t p0 = 0; p0 < nslots; p0 += kSlotPass) {
            if (p0) __syncthreads();                  // the previous pass's stores have read the window
            if (okr) {
#pragma unroll
                for (uint32_t k = 0; k < 2; ++k) {
                    const uint32_t r = rank + (k ? (us.mask & 1u) : 0u) - p0;
                    if (((us.mask >> k) & 1u) && r < kSlotPass) {
                        uint4* d = stg + 6 * r;
#pragma unroll
                        for (int q = 0; q < 6; ++q)
                            d[q] = make_uint4(us.w[k][4 * q], us.w[k][4 * q + 1], us.w[k][4 * q + 2], us.w[k][4 * q + 3]);
                    }
                }
            }
            __syncthreads();
            const uint32_t nq = 6 * min(kSlotPass, nslots - p0);
            for (uint32_t q = t; q < nq; q += kDecTile) {
                const uint4 v = stg[q];
                __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, dst + 6 * p0 + q);
            }
        }
        __syncthreads();                              // the window is reused below
    }
    uint4* stage = reinterpret_cast<uint4*>(s_win);
#pragma unroll
    for (int k = 0; k < 4; ++k) stage[4 * t + k] = mz[k];
    __syncthreads();
    const uint64_t nblk = min(uint64_t(kDecTile), a.n - i0);
    uint4* dst = reinterpret_cast<uint4*>(a.out.msgs + i0);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t j = uint32_t(k * kDecTile + t);
        if (j < 4 * nblk) {
            if (kNTOut) {
                const uint4 v = stage[j];
                __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4*>(dst + j));
            }
            else dst[j] = stage[j];
        }
    }
}

// dlen_tiles: per 4096-record block (256 threads x 16 lengths) the byte
// total of every 64-record decode workgroup (4 threads) and of the block.
__global__ __launch_bounds__(256) void dlen_tiles_kernel(const uint32_t* len, uint64_t n, uint64_t* tile_sum,
                                                         uint64_t* blk_sum) {
    __shared__ uint64_t s_wave[4];
    const uint64_t lo = uint64_t(blockIdx.x) * kDecLenBlk + 16ull * threadIdx.x;
    uint64_t sum = 0;
    if (lo + 16 <= n && (reinterpret_cast<uintptr_t>(len + lo) & 15) == 0) {
        const uint4* p = reinterpret_cast<const uint4*>(len + lo);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 w = p[k];
            sum += uint64_t(w.x) + w.y + w.z + w.w;
        }
    } else {
        for (int k = 0; k < 16; ++k) sum += lo + k < n ? len[lo + k] : 0u;
    }
    // groups of 4 threads = one 64-record workgroup
    const uint64_t incl = wave_incl_scan_u64(sum);
    const int lane = threadIdx.x & 63;
    const uint64_t prev4_all = __shfl(incl, (lane + 60) & 63, 64);   // lane - 4 (wrapping)
    const uint64_t prev4 = lane >= 4 ? prev4_all : 0;
    const uint64_t wgi = (uint64_t(blockIdx.x) * kDecLenBlk + 64ull * (threadIdx.x >> 2)) / kDecTile;
    if ((lane & 3) == 3 && wgi * kDecTile < n) tile_sum[wgi] = incl - prev4;
    uint64_t total;
    block_excl_scan_u64<256>(sum, s_wave, &total);
    if (threadIdx.x == 0) blk_sum[blockIdx.x] = total;
}

hipError_t launch_dlen_tiles(const uint32_t* rec_len, uint64_t n, uint64_t* tile_sum, uint64_t* blk_sum, hipStream_t s) {
    ONC_LAUNCH(dlen_tiles_kernel, dim3(uint32_t((n + kDecLenBlk - 1) / kDecLenBlk)), dim3(256), 0, s, rec_len, n, tile_sum,
               blk_sum);
    return hipGetLastError();
}

// The message decode (onc_decode / onc_decode_lengths) under one first-round
// policy (kLine, decode_kernel).
template <bool kLine>
hipError_t launch_message_decode(const DecArgs& a, int mode, hipStream_t s) {
    const uint64_t wgs = (a.n + kDecTile - 1) / kDecTile;
    const dim3 g{uint32_t(wgs)}, b{uint32_t(kDecTile)};
    if (a.rec_len) {
        const bool fused = a.blk_base == nullptr;
        if (mode == ONC_DECODE_BYTES) {
            if (fused) ONC_LAUNCH((decode_kernel<ONC_DECODE_BYTES, true, true, true, true, false, kLine>), g, b, 0, s, a);
            else ONC_LAUNCH((decode_kernel<ONC_DECODE_BYTES, true, true, true, false, false, kLine>), g, b, 0, s, a);
        } else {
            if (fused) ONC_LAUNCH((decode_kernel<ONC_DECODE_SLICE, true, true, true, true, false, kLine>), g, b, 0, s, a);
            else ONC_LAUNCH((decode_kernel<ONC_DECODE_SLICE, true, true, true, false, false, kLine>), g, b, 0, s, a);
        }
        return hipGetLastError();
    }
    if (mode == ONC_DECODE_BYTES)
        ONC_LAUNCH((decode_kernel<ONC_DECODE_BYTES, true, true, false, false, false, kLine>), g, b, 0, s, a);
    else
        ONC_LAUNCH((decode_kernel<ONC_DECODE_SLICE, true, true, false, false, false, kLine>), g, b, 0, s, a);
    return hipGetLastError();
}

hipError_t launch_decode(const DecArgs& a, int mode, hipStream_t s) {
    if (a.body) {
        const uint64_t tiles = (a.n + kDecTile - 1) / kDecTile;
        if (mode == ONC_DECODE_BYTES)
            ONC_LAUNCH((decode_kernel<ONC_DECODE_BYTES, true, true, false, false, true>), dim3(uint32_t(tiles)),
                       dim3(kDecTile), 0, s, a);
        else
            ONC_LAUNCH((decode_kernel<ONC_DECODE_SLICE, true, true, false, false, true>), dim3(uint32_t(tiles)),
                       dim3(kDecTile), 0, s, a);
        return hipGetLastError();
    }
    if (a.line) return launch_message_decode<true>(a, mode, s);
    return launch_message_decode<false>(a, mode, s);
}

}  // namespace onc
