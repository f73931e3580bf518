/*
 * onc_oracle.c — CPU restatement of domodwyer/onc-rpc v0.3.3 (TEST INFRASTRUCTURE).
 *
 * THE PARITY CHECKER, NOT THE PRODUCT: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg use this file (see onc_oracle.h).
 *
 * Citations are file:line in the reference (/root/reference). The third-party
 * pieces the reference leans on are restated here as well:
 *   byteorder 1.5.0  (Cargo.lock:54-56): read_u32/write_u32::<BigEndian>
 *   bytes 1.11.1     (Cargo.lock:60-62): Buf::get_u32 (big endian), slice, advance
 *   std::io::Cursor::read_exact: short read -> io::ErrorKind::UnexpectedEof
 *     ("failed to fill whole buffer"), surfaced through errors.rs:99-103.
 *   std::io::Write::write_all on a bounded buffer: partial write, then
 *     io::ErrorKind::WriteZero.
 */
#include "onc_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------------- */
/* Result type: Result<_, crate::Error> as (code, payload words)          */
/* ---------------------------------------------------------------------- */
typedef struct {
    int32_t code;
    uint32_t a0, a1;
} o_err;

static const o_err O_OK = {ONC_OK, 0, 0};
static o_err o_error(int32_t code, uint32_t a0, uint32_t a1) {
    o_err e = {code, a0, a1};
    return e;
}
#define TRY(expr)                    \
    do {                             \
        o_err _e = (expr);           \
        if (_e.code != ONC_OK) return _e; \
    } while (0)

/* A borrowed byte slice (&'a [u8] / Bytes) */
typedef struct {
    const uint8_t* ptr;
    uint64_t len;
} o_slice;

static uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

/* pad_length — opaque.rs:115-121 */
uint32_t oracle_pad_length(uint32_t l) {
    if (l % 4 == 0) return 0;
    return 4 - (l % 4);
}

/* ---------------------------------------------------------------------- */
/* std::io::Cursor<&[u8]> + ReadBytesExt::read_u32::<BigEndian>           */
/* ---------------------------------------------------------------------- */
typedef struct {
    const uint8_t* data;
    uint64_t len;
    uint64_t pos;
} o_cursor;

static o_err cur_read_u32(o_cursor* c, uint32_t* v) {
    if (c->pos > c->len || c->len - c->pos < 4) {
        /* Cursor::read_exact: position moves to the end, UnexpectedEof. */
        c->pos = c->len;
        return o_error(ONC_ERR_IO_UNEXPECTED_EOF, 0, 0);
    }
    *v = be32(c->data + c->pos);
    c->pos += 4;
    return O_OK;
}

/* ---------------------------------------------------------------------- */
/* bytes::Bytes view + BytesReaderExt (bytes_ext.rs:7-43)                 */
/* ---------------------------------------------------------------------- */
typedef struct {
    const uint8_t* ptr; /* current start (advance moves it) */
    uint64_t len;       /* remaining */
} o_bytes;

static void bytes_advance(o_bytes* v, uint64_t n) {
    /* Buf::advance panics when n > remaining; the reference never does
     * that (the advanced length equals the parsed length). */
    if (n > v->len) abort();
    v->ptr += n;
    v->len -= n;
}

/* try_u32 — bytes_ext.rs:17-22 */
static o_err bytes_try_u32(o_bytes* v, uint32_t* out) {
    if (v->len < 4) return o_error(ONC_ERR_INVALID_LENGTH, 0, 0);
    *out = be32(v->ptr); /* Buf::get_u32 is big endian */
    v->ptr += 4;
    v->len -= 4;
    return O_OK;
}

/* try_array — bytes_ext.rs:25-42 */
static o_err bytes_try_array(o_bytes* v, uint64_t max_len, o_bytes* body) {
    uint32_t n32;
    TRY(bytes_try_u32(v, &n32));
    uint64_t payload_len = n32;
    if (payload_len > max_len) return o_error(ONC_ERR_INVALID_LENGTH, 0, 0);
    uint64_t end_plus_padding = payload_len + oracle_pad_length(n32);
    if (end_plus_padding > v->len) return o_error(ONC_ERR_INVALID_LENGTH, 0, 0);
    body->ptr = v->ptr;
    body->len = payload_len;
    bytes_advance(v, end_plus_padding);
    return O_OK;
}

/* ---------------------------------------------------------------------- */
/* std::io::Write over a bounded buffer                                   */
/* ---------------------------------------------------------------------- */
typedef struct {
    uint8_t* buf;
    uint64_t cap;
    uint64_t pos;
} o_writer;

static o_err w_write_all(o_writer* w, const uint8_t* src, uint64_t n) {
    uint64_t room = w->cap > w->pos ? w->cap - w->pos : 0;
    uint64_t k = n < room ? n : room;
    if (k) memcpy(w->buf + w->pos, src, k);
    w->pos += k;
    if (k < n) return o_error(ONC_ENC_WRITE_ZERO, 0, 0);
    return O_OK;
}

/* WriteBytesExt::write_u32::<BigEndian> */
static o_err w_write_u32(o_writer* w, uint32_t v) {
    uint8_t b[4] = {(uint8_t)(v >> 24), (uint8_t)(v >> 16), (uint8_t)(v >> 8), (uint8_t)v};
    return w_write_all(w, b, 4);
}

/* ---------------------------------------------------------------------- */
/* Value types (the Rust enums/structs, borrowed form)                    */
/* ---------------------------------------------------------------------- */

/* AuthUnixParams — unix_params.rs:72-82 (Gids: [u32;16] + len, :16-23) */
typedef struct {
    uint32_t stamp;
    o_slice machine_name;
    uint32_t uid, gid;
    uint32_t gids[16];
    uint32_t ngids;
} o_unix;

/* AuthFlavor — flavor.rs:18-49 */
enum { O_AUTH_NONE = 0, O_AUTH_UNIX = 1, O_AUTH_SHORT = 2, O_AUTH_UNKNOWN = 3 };
typedef struct {
    int kind;
    int some;     /* AuthNone(Some(_)) vs AuthNone(None) */
    uint32_t id;  /* Unknown { id } */
    o_slice data; /* AuthNone(Some)/AuthShort/Unknown data */
    o_unix unix;  /* AuthUnix */
} o_auth;

/* AcceptedStatus — accepted_reply.rs:108-150 (variant = wire value) */
typedef struct {
    uint32_t variant;
    o_slice payload; /* Success */
    uint32_t low, high;
} o_accepted_status;

typedef struct {
    o_auth verf;
    o_accepted_status status;
} o_accepted_reply;

/* RejectedReply — rejected_reply.rs:23-38; AuthError :129-173 */
typedef struct {
    uint32_t variant; /* 0 RpcVersionMismatch, 1 AuthError */
    uint32_t low, high;
    uint32_t auth_error;
} o_rejected_reply;

/* ReplyBody — reply_body.rs:15-26 */
typedef struct {
    uint32_t variant; /* 0 Accepted, 1 Denied */
    o_accepted_reply accepted;
    o_rejected_reply denied;
} o_reply_body;

/* CallBody — call_body.rs:17-30 */
typedef struct {
    uint32_t program, program_version, procedure;
    o_auth cred, verf;
    o_slice payload;
} o_call_body;

/* RpcMessage + MessageType — rpc_message.rs:22-32, :97-105 */
typedef struct {
    uint32_t xid;
    uint32_t msg_type; /* 0 Call, 1 Reply */
    o_call_body call;
    o_reply_body reply;
} o_message;

/* ---------------------------------------------------------------------- */
/* serialised_len family                                                  */
/* Lengths are computed in u64; the reference uses u32 (see DESIGN.md:    */
/* totals >= 2^31 are ONC_ENC_TOO_LONG, rpc_message.rs:146).              */
/* ---------------------------------------------------------------------- */

/* Opaque::serialised_len — opaque.rs:60-63 */
static uint64_t opaque_serialised_len(uint64_t len) {
    return 4 + len + oracle_pad_length((uint32_t)len);
}

/* AuthUnixParams::serialised_len — unix_params.rs:219-230 */
static uint64_t unix_serialised_len(const o_unix* p) {
    return 4 * 3 + opaque_serialised_len(p->machine_name.len) + ((uint64_t)p->ngids + 1) * 4;
}

/* AuthUnixParams::associated_data_len — unix_params.rs:234-245 */
static uint64_t unix_associated_data_len(const o_unix* p) {
    return 4 * 3 + p->machine_name.len + 4ull * p->ngids;
}

/* AuthFlavor::serialised_len — flavor.rs:154-174 */
static uint64_t auth_serialised_len(const o_auth* a) {
    uint64_t l = 4;
    if (a->kind == O_AUTH_NONE && !a->some)
        l += 4 + 0;
    else if (a->kind == O_AUTH_UNIX)
        l += 4 + unix_serialised_len(&a->unix);
    else
        l += opaque_serialised_len(a->data.len);
    return l;
}

/* AuthFlavor::associated_data_len — flavor.rs:142-150 */
static uint64_t auth_associated_data_len(const o_auth* a) {
    switch (a->kind) {
        case O_AUTH_NONE: return a->some ? a->data.len : 0;
        case O_AUTH_UNIX: return unix_associated_data_len(&a->unix);
        default: return a->data.len;
    }
}

/* AuthFlavor::id — flavor.rs:132-139 */
static uint32_t auth_id(const o_auth* a) {
    switch (a->kind) {
        case O_AUTH_NONE: return ONC_AUTH_NONE;
        case O_AUTH_UNIX: return ONC_AUTH_UNIX;
        case O_AUTH_SHORT: return ONC_AUTH_SHORT;
        default: return a->id;
    }
}

/* AcceptedStatus::serialised_len — accepted_reply.rs:214-231 */
static uint64_t accepted_status_serialised_len(const o_accepted_status* s) {
    uint64_t len = 4;
    if (s->variant == ONC_ACCEPT_SUCCESS) len += s->payload.len;
    else if (s->variant == ONC_ACCEPT_PROG_MISMATCH) len += 8;
    return len;
}

/* RejectedReply::serialised_len — rejected_reply.rs:76-95; AuthError :210-212 */
static uint64_t rejected_serialised_len(const o_rejected_reply* r) {
    return 4 + (r->variant == ONC_REJECT_RPC_MISMATCH ? 8 : 4);
}

/* ReplyBody::serialised_len — reply_body.rs:60-73; AcceptedReply :64-66 */
static uint64_t reply_serialised_len(const o_reply_body* r) {
    uint64_t len = 4;
    if (r->variant == ONC_REPLY_ACCEPTED)
        len += auth_serialised_len(&r->accepted.verf) +
               accepted_status_serialised_len(&r->accepted.status);
    else
        len += rejected_serialised_len(&r->denied);
    return len;
}

/* CallBody::serialised_len — call_body.rs:111-119 */
static uint64_t call_serialised_len(const o_call_body* c) {
    return 4 * 4 + auth_serialised_len(&c->cred) + auth_serialised_len(&c->verf) + c->payload.len;
}

/* MessageType::serialised_len — rpc_message.rs:72-77; RpcMessage :201-204 */
static uint64_t message_serialised_len(const o_message* m) {
    uint64_t body = m->msg_type == ONC_MSG_CALL ? call_serialised_len(&m->call)
                                                : reply_serialised_len(&m->reply);
    return (body + 4) + 4 + 4;
}

/* ---------------------------------------------------------------------- */
/* Encode: serialise_into family                                          */
/* ---------------------------------------------------------------------- */

/* Opaque::serialise_into — opaque.rs:38-56 */
static o_err opaque_serialise_into(o_writer* w, o_slice body) {
    TRY(w_write_u32(w, (uint32_t)body.len));
    TRY(w_write_all(w, body.ptr, body.len));
    static const uint8_t PADDING[3] = {0, 0, 0};
    uint32_t fill = oracle_pad_length((uint32_t)body.len);
    if (fill > 0) TRY(w_write_all(w, PADDING, fill));
    return O_OK;
}

/* AuthUnixParams::serialise_into — unix_params.rs:162-176 */
static o_err unix_serialise_into(o_writer* w, const o_unix* p) {
    TRY(w_write_u32(w, p->stamp));
    TRY(opaque_serialise_into(w, p->machine_name));
    TRY(w_write_u32(w, p->uid));
    TRY(w_write_u32(w, p->gid));
    TRY(w_write_u32(w, p->ngids));
    for (uint32_t i = 0; i < p->ngids; i++) TRY(w_write_u32(w, p->gids[i]));
    return O_OK;
}

/* AuthFlavor::serialise_into — flavor.rs:106-129.
 * The reference writes the id, then panics on assert!(assoc <= 200)
 * (:110). The batch contract reports ONC_ENC_AUTH_GT_200 and writes
 * nothing for the record, so the assertion is checked up front by
 * encode_validate() below; here it is an internal invariant. */
static o_err auth_serialise_into(o_writer* w, const o_auth* a) {
    TRY(w_write_u32(w, auth_id(a)));
    if (auth_associated_data_len(a) > ONC_MAX_AUTH_LEN) abort();
    if ((a->kind == O_AUTH_NONE && a->some) || a->kind == O_AUTH_SHORT || a->kind == O_AUTH_UNKNOWN)
        return opaque_serialise_into(w, a->data);
    if (a->kind == O_AUTH_NONE) return w_write_u32(w, 0);
    TRY(w_write_u32(w, (uint32_t)unix_serialised_len(&a->unix)));
    return unix_serialise_into(w, &a->unix);
}

/* CallBody::serialise_into — call_body.rs:98-108 */
static o_err call_serialise_into(o_writer* w, const o_call_body* c) {
    TRY(w_write_u32(w, 2)); /* RPC_VERSION call_body.rs:10 */
    TRY(w_write_u32(w, c->program));
    TRY(w_write_u32(w, c->program_version));
    TRY(w_write_u32(w, c->procedure));
    TRY(auth_serialise_into(w, &c->cred));
    TRY(auth_serialise_into(w, &c->verf));
    return w_write_all(w, c->payload.ptr, c->payload.len);
}

/* AcceptedStatus::serialise_into — accepted_reply.rs:195-211 */
static o_err accepted_status_serialise_into(o_writer* w, const o_accepted_status* s) {
    TRY(w_write_u32(w, s->variant));
    if (s->variant == ONC_ACCEPT_SUCCESS) return w_write_all(w, s->payload.ptr, s->payload.len);
    if (s->variant == ONC_ACCEPT_PROG_MISMATCH) {
        TRY(w_write_u32(w, s->low));
        return w_write_u32(w, s->high);
    }
    return O_OK;
}

/* ReplyBody::serialise_into — reply_body.rs:45-56; AcceptedReply :58-61;
 * RejectedReply rejected_reply.rs:61-73; AuthError :194-207 */
static o_err reply_serialise_into(o_writer* w, const o_reply_body* r) {
    TRY(w_write_u32(w, r->variant));
    if (r->variant == ONC_REPLY_ACCEPTED) {
        TRY(auth_serialise_into(w, &r->accepted.verf));
        return accepted_status_serialise_into(w, &r->accepted.status);
    }
    TRY(w_write_u32(w, r->denied.variant));
    if (r->denied.variant == ONC_REJECT_RPC_MISMATCH) {
        TRY(w_write_u32(w, r->denied.low));
        return w_write_u32(w, r->denied.high);
    }
    return w_write_u32(w, r->denied.auth_error);
}

/* RpcMessage::serialise_into — rpc_message.rs:136-164 (+ MessageType :55-68) */
static o_err message_serialise_into(o_writer* w, const o_message* m) {
    uint64_t len = message_serialised_len(m);
    if (len & 0xFFFFFFFF80000000ull) /* LAST_FRAGMENT_BIT set (or beyond u32) */
        return o_error(ONC_ENC_TOO_LONG, 0, 0);
    uint32_t header = (uint32_t)(len - 4) | 0x80000000u;
    TRY(w_write_u32(w, header));
    TRY(w_write_u32(w, m->xid));
    TRY(w_write_u32(w, m->msg_type));
    if (m->msg_type == ONC_MSG_CALL) return call_serialise_into(w, &m->call);
    return reply_serialise_into(w, &m->reply);
}

/* ---------------------------------------------------------------------- */
/* Descriptor <-> value conversion ("construction" of the Rust values)    */
/* ---------------------------------------------------------------------- */

/* Builds an AuthFlavor from a descriptor. AuthUnixParams::new panics for a
 * machine name > 255 (unix_params.rs:149) and Gids::from_iter for > 16 gids
 * (:47); those become ONC_ENC_NAME_GT_255 / ONC_ENC_GIDS_GT_16. */
static o_err auth_from_desc(const onc_auth* d, const onc_unix_params* unix_table,
                            const uint8_t* arena, o_auth* a) {
    memset(a, 0, sizeof(*a));
    uint32_t kind = ONC_AUTH_KIND(*d), len = ONC_AUTH_LEN(*d);
    if (kind > ONC_KIND_UNKNOWN) return o_error(ONC_ENC_BAD_DESCRIPTOR, 0, 0);
    a->kind = (int)kind;
    if (kind == ONC_KIND_UNIX) {
        const onc_unix_params* p = &unix_table[d->ref];
        if (p->name_len > ONC_MAX_MACHINE_NAME_LEN) return o_error(ONC_ENC_NAME_GT_255, 0, 0);
        if (p->ngids > ONC_MAX_GIDS) return o_error(ONC_ENC_GIDS_GT_16, 0, 0);
        a->unix.stamp = p->stamp;
        a->unix.machine_name.ptr = arena + p->name_off;
        a->unix.machine_name.len = p->name_len;
        a->unix.uid = p->uid;
        a->unix.gid = p->gid;
        a->unix.ngids = p->ngids;
        memcpy(a->unix.gids, p->gids, sizeof(uint32_t) * p->ngids);
        /* ABI 6 (include/onc_rpc.h onc_auth): a declared length must be the
         * block's serialised_len (a descriptor the Rust types cannot hold) */
        if (len != 0 && len != unix_serialised_len(&a->unix)) return o_error(ONC_ENC_BAD_DESCRIPTOR, 0, 0);
        return O_OK;
    }
    a->id = d->id;
    a->some = len > 0;
    a->data.ptr = arena + d->ref;
    a->data.len = len;
    return O_OK;
}

static o_err message_from_desc(const onc_msg* d, const onc_unix_params* unix_table,
                               const uint8_t* auth_arena, const uint8_t* payload_arena,
                               o_message* m) {
    memset(m, 0, sizeof(*m));
    m->xid = d->xid;
    m->msg_type = d->msg_type;
    o_slice payload = {payload_arena + d->payload_off, d->payload_len};
    if (d->msg_type == ONC_MSG_CALL) {
        m->call.program = d->u.call.program;
        m->call.program_version = d->u.call.program_version;
        m->call.procedure = d->u.call.procedure;
        TRY(auth_from_desc(&d->cred, unix_table, auth_arena, &m->call.cred));
        TRY(auth_from_desc(&d->verf, unix_table, auth_arena, &m->call.verf));
        m->call.payload = payload;
        return O_OK;
    }
    if (d->msg_type != ONC_MSG_REPLY) return o_error(ONC_ENC_BAD_DESCRIPTOR, 0, 0);
    m->reply.variant = d->reply_stat;
    if (d->reply_stat == ONC_REPLY_ACCEPTED) {
        if (d->stat > ONC_ACCEPT_SYSTEM_ERR) return o_error(ONC_ENC_BAD_DESCRIPTOR, 0, 0);
        TRY(auth_from_desc(&d->verf, unix_table, auth_arena, &m->reply.accepted.verf));
        m->reply.accepted.status.variant = d->stat;
        m->reply.accepted.status.low = d->u.mismatch.low;
        m->reply.accepted.status.high = d->u.mismatch.high;
        m->reply.accepted.status.payload = payload;
        return O_OK;
    }
    if (d->reply_stat != ONC_REPLY_DENIED) return o_error(ONC_ENC_BAD_DESCRIPTOR, 0, 0);
    if (d->stat > ONC_REJECT_AUTH_ERROR) return o_error(ONC_ENC_BAD_DESCRIPTOR, 0, 0);
    m->reply.denied.variant = d->stat;
    if (d->stat == ONC_REJECT_AUTH_ERROR && d->auth_stat > ONC_AUTH_STAT_MAX)
        return o_error(ONC_ENC_BAD_DESCRIPTOR, 0, 0);
    m->reply.denied.low = d->u.mismatch.low;
    m->reply.denied.high = d->u.mismatch.high;
    m->reply.denied.auth_error = d->auth_stat;
    return O_OK;
}

/* Encode-time checks of serialise_into in reference order: oversize
 * (rpc_message.rs:146) before the per-auth assert (flavor.rs:110; cred is
 * written before verf, call_body.rs:104-105). */
static o_err encode_validate(const o_message* m) {
    if (message_serialised_len(m) & 0xFFFFFFFF80000000ull) return o_error(ONC_ENC_TOO_LONG, 0, 0);
    if (m->msg_type == ONC_MSG_CALL) {
        if (auth_associated_data_len(&m->call.cred) > ONC_MAX_AUTH_LEN)
            return o_error(ONC_ENC_AUTH_GT_200, 0, 0);
        if (auth_associated_data_len(&m->call.verf) > ONC_MAX_AUTH_LEN)
            return o_error(ONC_ENC_AUTH_GT_200, 0, 0);
    } else if (m->reply.variant == ONC_REPLY_ACCEPTED) {
        if (auth_associated_data_len(&m->reply.accepted.verf) > ONC_MAX_AUTH_LEN)
            return o_error(ONC_ENC_AUTH_GT_200, 0, 0);
    }
    return O_OK;
}

static void auth_to_desc(const o_auth* a, const uint8_t* base, uint64_t slot, onc_auth* d,
                         onc_unix_params* u) {
    memset(d, 0, sizeof(*d));
    d->id = a->kind == O_AUTH_UNKNOWN ? a->id : (uint32_t)a->kind;
    if (a->kind == O_AUTH_UNIX) {
        /* ABI 6: the decoded credential declares its serialised length */
        d->kind_len = ONC_AUTH_PACK(ONC_KIND_UNIX, (uint32_t)unix_serialised_len(&a->unix));
        d->ref = slot;
        memset(u, 0, sizeof(*u));
        u->stamp = a->unix.stamp;
        u->uid = a->unix.uid;
        u->gid = a->unix.gid;
        u->ngids = a->unix.ngids;
        u->name_off = (uint64_t)(a->unix.machine_name.ptr - base);
        u->name_len = (uint32_t)a->unix.machine_name.len;
        memcpy(u->gids, a->unix.gids, sizeof(uint32_t) * a->unix.ngids);
        return;
    }
    d->kind_len = ONC_AUTH_PACK(a->kind, a->data.len);
    d->ref = (uint64_t)(a->data.ptr - base);
}

static void message_to_desc(const o_message* m, const uint8_t* base, uint64_t slot_base,
                            onc_msg* d, onc_unix_params unix[2]) {
    memset(d, 0, sizeof(*d));
    d->xid = m->xid;
    d->msg_type = (uint8_t)m->msg_type;
    if (m->msg_type == ONC_MSG_CALL) {
        d->u.call.program = m->call.program;
        d->u.call.program_version = m->call.program_version;
        d->u.call.procedure = m->call.procedure;
        auth_to_desc(&m->call.cred, base, slot_base, &d->cred, &unix[0]);
        auth_to_desc(&m->call.verf, base, slot_base + 1, &d->verf, &unix[1]);
        d->payload_off = (uint64_t)(m->call.payload.ptr - base);
        d->payload_len = (uint32_t)m->call.payload.len;
        return;
    }
    d->reply_stat = (uint8_t)m->reply.variant;
    if (m->reply.variant == ONC_REPLY_ACCEPTED) {
        const o_accepted_status* s = &m->reply.accepted.status;
        auth_to_desc(&m->reply.accepted.verf, base, slot_base + 1, &d->verf, &unix[1]);
        d->stat = (uint8_t)s->variant;
        if (s->variant == ONC_ACCEPT_PROG_MISMATCH) {
            d->u.mismatch.low = s->low;
            d->u.mismatch.high = s->high;
        }
        if (s->variant == ONC_ACCEPT_SUCCESS) {
            d->payload_off = (uint64_t)(s->payload.ptr - base);
            d->payload_len = (uint32_t)s->payload.len;
        }
        return;
    }
    d->stat = (uint8_t)m->reply.denied.variant;
    if (m->reply.denied.variant == ONC_REJECT_RPC_MISMATCH) {
        d->u.mismatch.low = m->reply.denied.low;
        d->u.mismatch.high = m->reply.denied.high;
    } else {
        d->auth_stat = (uint8_t)m->reply.denied.auth_error;
    }
}

/* ---------------------------------------------------------------------- */
/* Decode, slice mode (TryFrom<&[u8]>)                                    */
/* ---------------------------------------------------------------------- */

/* Opaque::from_wire — opaque.rs:72-98. The bound is the cursor's whole
 * underlying slice (`*c.get_ref()`), not an enclosing length. */
static o_err opaque_from_wire(o_cursor* c, uint64_t max_len, o_slice* body) {
    uint32_t payload_len;
    TRY(cur_read_u32(c, &payload_len));
    if ((uint64_t)payload_len > max_len) return o_error(ONC_ERR_INVALID_LENGTH, 0, 0);
    uint64_t start = c->pos;
    uint64_t end = start + payload_len;
    uint64_t end_plus_padding = end + oracle_pad_length(payload_len);
    if (end_plus_padding > c->len) return o_error(ONC_ERR_INVALID_LENGTH, 0, 0);
    body->ptr = c->data + start;
    body->len = payload_len;
    c->pos = end_plus_padding;
    return O_OK;
}

/* AuthUnixParams::from_cursor — unix_params.rs:90-129 */
static o_err unix_from_cursor(o_cursor* c, uint32_t expected_len, o_unix* p) {
    uint64_t start_pos = c->pos;
    memset(p, 0, sizeof(*p));
    TRY(cur_read_u32(c, &p->stamp));
    TRY(opaque_from_wire(c, ONC_MAX_MACHINE_NAME_LEN, &p->machine_name));
    TRY(cur_read_u32(c, &p->uid));
    TRY(cur_read_u32(c, &p->gid));
    uint32_t gids_count;
    TRY(cur_read_u32(c, &gids_count));
    if (gids_count == 0) {
        p->ngids = 0;
    } else if (gids_count <= 16) {
        for (uint32_t i = 0; i < gids_count; i++) TRY(cur_read_u32(c, &p->gids[i]));
        p->ngids = gids_count;
    } else {
        return o_error(ONC_ERR_INVALID_AUTH_DATA, 0, 0);
    }
    if (c->pos - start_pos != (uint64_t)expected_len) return o_error(ONC_ERR_INVALID_AUTH_DATA, 0, 0);
    return O_OK;
}

/* AuthFlavor::from_cursor — flavor.rs:52-69; new_none :71-78;
 * new_unix :80-88; new_short :90-94 */
static o_err auth_from_cursor(o_cursor* c, o_auth* a) {
    memset(a, 0, sizeof(*a));
    uint32_t flavor;
    TRY(cur_read_u32(c, &flavor));
    switch (flavor) {
        case ONC_AUTH_NONE: {
            o_slice payload;
            TRY(opaque_from_wire(c, 200, &payload));
            a->kind = O_AUTH_NONE;
            a->data = payload;
            a->some = payload.len != 0;
            return O_OK;
        }
        case ONC_AUTH_UNIX: {
            uint32_t len;
            TRY(cur_read_u32(c, &len));
            if (len > 200) return o_error(ONC_ERR_INVALID_LENGTH, 0, 0);
            a->kind = O_AUTH_UNIX;
            return unix_from_cursor(c, len, &a->unix);
        }
        case ONC_AUTH_SHORT:
            a->kind = O_AUTH_SHORT;
            return opaque_from_wire(c, 200, &a->data);
        default:
            a->kind = O_AUTH_UNKNOWN;
            a->id = flavor;
            return opaque_from_wire(c, 200, &a->data);
    }
}

/* CallBody::from_cursor — call_body.rs:37-69 */
static o_err call_from_cursor(o_cursor* c, o_call_body* b) {
    uint32_t rpc_version;
    TRY(cur_read_u32(c, &rpc_version));
    if (rpc_version != 2) return o_error(ONC_ERR_INVALID_RPC_VERSION, rpc_version, 0);
    TRY(cur_read_u32(c, &b->program));
    TRY(cur_read_u32(c, &b->program_version));
    TRY(cur_read_u32(c, &b->procedure));
    TRY(auth_from_cursor(c, &b->cred));
    TRY(auth_from_cursor(c, &b->verf));
    uint64_t start = c->pos;
    if (start > c->len) return o_error(ONC_ERR_INCOMPLETE_HEADER, 0, 0);
    b->payload.ptr = c->data + start;
    b->payload.len = c->len - start;
    return O_OK;
}

/* AcceptedStatus::from_cursor — accepted_reply.rs:158-174; new_success :176-186 */
static o_err accepted_status_from_cursor(o_cursor* c, o_accepted_status* s) {
    uint32_t v;
    TRY(cur_read_u32(c, &v));
    s->variant = v;
    switch (v) {
        case ONC_ACCEPT_SUCCESS:
            s->payload.ptr = c->data + c->pos;
            s->payload.len = c->len - c->pos;
            return O_OK;
        case ONC_ACCEPT_PROG_UNAVAIL:
        case ONC_ACCEPT_PROC_UNAVAIL:
        case ONC_ACCEPT_GARBAGE_ARGS:
        case ONC_ACCEPT_SYSTEM_ERR:
            return O_OK;
        case ONC_ACCEPT_PROG_MISMATCH:
            TRY(cur_read_u32(c, &s->low));
            return cur_read_u32(c, &s->high);
        default:
            return o_error(ONC_ERR_INVALID_REPLY_STATUS, v, 0);
    }
}

/* AuthError::from_cursor — rejected_reply.rs:176-190 */
static o_err auth_error_from_cursor(o_cursor* c, uint32_t* e) {
    uint32_t v;
    TRY(cur_read_u32(c, &v));
    if (v > ONC_AUTH_STAT_MAX) return o_error(ONC_ERR_INVALID_AUTH_ERROR, v, 0);
    *e = v;
    return O_OK;
}

/* RejectedReply::from_cursor — rejected_reply.rs:46-57 */
static o_err rejected_from_cursor(o_cursor* c, o_rejected_reply* r) {
    uint32_t v;
    TRY(cur_read_u32(c, &v));
    r->variant = v;
    if (v == ONC_REJECT_RPC_MISMATCH) {
        TRY(cur_read_u32(c, &r->low));
        return cur_read_u32(c, &r->high);
    }
    if (v == ONC_REJECT_AUTH_ERROR) return auth_error_from_cursor(c, &r->auth_error);
    return o_error(ONC_ERR_INVALID_REJECTED_REPLY_TYPE, v, 0);
}

/* ReplyBody::from_cursor — reply_body.rs:29-35; AcceptedReply accepted_reply.rs:35-40 */
static o_err reply_from_cursor(o_cursor* c, o_reply_body* r) {
    uint32_t v;
    TRY(cur_read_u32(c, &v));
    r->variant = v;
    if (v == ONC_REPLY_ACCEPTED) {
        TRY(auth_from_cursor(c, &r->accepted.verf));
        return accepted_status_from_cursor(c, &r->accepted.status);
    }
    if (v == ONC_REPLY_DENIED) return rejected_from_cursor(c, &r->denied);
    return o_error(ONC_ERR_INVALID_REPLY_TYPE, v, 0);
}

/* MessageType::from_cursor — rpc_message.rs:39-45 */
static o_err message_type_from_cursor(o_cursor* c, o_message* m) {
    uint32_t v;
    TRY(cur_read_u32(c, &v));
    m->msg_type = v;
    if (v == ONC_MSG_CALL) return call_from_cursor(c, &m->call);
    if (v == ONC_MSG_REPLY) return reply_from_cursor(c, &m->reply);
    return o_error(ONC_ERR_INVALID_MESSAGE_TYPE, v, 0);
}

/* expected_message_len — rpc_message.rs:343-367 */
static o_err expected_message_len(const uint8_t* data, uint64_t len, uint32_t* want) {
    if (len < 4) return o_error(ONC_ERR_INCOMPLETE_HEADER, 0, 0);
    uint32_t header = be32(data);
    if ((header & 0x80000000u) == 0) return o_error(ONC_ERR_FRAGMENTED, 0, 0);
    *want = (header & 0x7FFFFFFFu) + 4;
    return O_OK;
}

/* unwrap_header — rpc_message.rs:320-335 */
static o_err unwrap_header(const uint8_t* data, uint64_t len, o_slice* rest) {
    uint32_t want;
    TRY(expected_message_len(data, len, &want));
    if (len != (uint64_t)want) return o_error(ONC_ERR_INCOMPLETE_MESSAGE, (uint32_t)len, want);
    rest->ptr = data + 4;
    rest->len = len - 4;
    return O_OK;
}

/* RpcMessage::try_from(&[u8]) — rpc_message.rs:243-271 */
static o_err message_try_from_slice(const uint8_t* v, uint64_t len, o_message* m) {
    memset(m, 0, sizeof(*m));
    o_slice data;
    TRY(unwrap_header(v, len, &data));
    o_cursor r = {data.ptr, data.len, 0};
    TRY(cur_read_u32(&r, &m->xid));
    TRY(message_type_from_cursor(&r, m));
    uint64_t want_len = len;
    uint64_t got = message_serialised_len(m);
    if (got != want_len) return o_error(ONC_ERR_INCOMPLETE_MESSAGE, (uint32_t)len, (uint32_t)got);
    return O_OK;
}

/* ---------------------------------------------------------------------- */
/* Decode, Bytes mode (TryFrom<Bytes>)                                    */
/* ---------------------------------------------------------------------- */

/* AuthUnixParams::try_from(Bytes) — unix_params.rs:252-276 */
static o_err unix_try_from_bytes(o_bytes v, o_unix* p) {
    memset(p, 0, sizeof(*p));
    TRY(bytes_try_u32(&v, &p->stamp));
    o_bytes name;
    TRY(bytes_try_array(&v, ONC_MAX_MACHINE_NAME_LEN, &name));
    p->machine_name.ptr = name.ptr;
    p->machine_name.len = name.len;
    TRY(bytes_try_u32(&v, &p->uid));
    TRY(bytes_try_u32(&v, &p->gid));
    uint32_t gids_count;
    TRY(bytes_try_u32(&v, &gids_count));
    if (gids_count == 0) {
        p->ngids = 0;
    } else if (gids_count <= 16) {
        for (uint32_t i = 0; i < gids_count; i++) TRY(bytes_try_u32(&v, &p->gids[i]));
        p->ngids = gids_count;
    } else {
        return o_error(ONC_ERR_INVALID_AUTH_DATA, 0, 0);
    }
    return O_OK;
}

/* AuthFlavor::try_from(Bytes) — flavor.rs:190-222 */
static o_err auth_try_from_bytes(o_bytes v, o_auth* a) {
    memset(a, 0, sizeof(*a));
    uint32_t flavor;
    TRY(bytes_try_u32(&v, &flavor));
    o_bytes auth_data;
    TRY(bytes_try_array(&v, 200, &auth_data));
    o_slice data = {auth_data.ptr, auth_data.len};
    switch (flavor) {
        case ONC_AUTH_NONE:
            a->kind = O_AUTH_NONE;
            a->some = auth_data.len != 0;
            a->data = data;
            return O_OK;
        case ONC_AUTH_UNIX: {
            uint64_t should_consume = auth_data.len;
            a->kind = O_AUTH_UNIX;
            TRY(unix_try_from_bytes(auth_data, &a->unix));
            if (unix_serialised_len(&a->unix) != should_consume)
                return o_error(ONC_ERR_INVALID_AUTH_DATA, 0, 0);
            return O_OK;
        }
        case ONC_AUTH_SHORT:
            a->kind = O_AUTH_SHORT;
            a->data = data;
            return O_OK;
        default:
            a->kind = O_AUTH_UNKNOWN;
            a->id = flavor;
            a->data = data;
            return O_OK;
    }
}

/* CallBody::try_from(Bytes) — call_body.rs:181-209 */
static o_err call_try_from_bytes(o_bytes v, o_call_body* b) {
    uint32_t rpc_version;
    TRY(bytes_try_u32(&v, &rpc_version));
    if (rpc_version != 2) return o_error(ONC_ERR_INVALID_RPC_VERSION, rpc_version, 0);
    TRY(bytes_try_u32(&v, &b->program));
    TRY(bytes_try_u32(&v, &b->program_version));
    TRY(bytes_try_u32(&v, &b->procedure));
    TRY(auth_try_from_bytes(v, &b->cred));
    bytes_advance(&v, auth_serialised_len(&b->cred));
    TRY(auth_try_from_bytes(v, &b->verf));
    bytes_advance(&v, auth_serialised_len(&b->verf));
    b->payload.ptr = v.ptr;
    b->payload.len = v.len;
    return O_OK;
}

/* AcceptedStatus::try_from(Bytes) — accepted_reply.rs:247-264 */
static o_err accepted_status_try_from_bytes(o_bytes v, o_accepted_status* s) {
    uint32_t x;
    TRY(bytes_try_u32(&v, &x));
    s->variant = x;
    switch (x) {
        case ONC_ACCEPT_SUCCESS:
            s->payload.ptr = v.ptr;
            s->payload.len = v.len;
            return O_OK;
        case ONC_ACCEPT_PROG_UNAVAIL:
        case ONC_ACCEPT_PROC_UNAVAIL:
        case ONC_ACCEPT_GARBAGE_ARGS:
        case ONC_ACCEPT_SYSTEM_ERR:
            return O_OK;
        case ONC_ACCEPT_PROG_MISMATCH:
            TRY(bytes_try_u32(&v, &s->low));
            return bytes_try_u32(&v, &s->high);
        default:
            return o_error(ONC_ERR_INVALID_REPLY_STATUS, x, 0);
    }
}

/* RejectedReply::try_from(Bytes) — rejected_reply.rs:107-125;
 * AuthError::try_from(Bytes) :215-236 */
static o_err rejected_try_from_bytes(o_bytes v, o_rejected_reply* r) {
    uint32_t x;
    TRY(bytes_try_u32(&v, &x));
    r->variant = x;
    if (x == ONC_REJECT_RPC_MISMATCH) {
        TRY(bytes_try_u32(&v, &r->low));
        return bytes_try_u32(&v, &r->high);
    }
    if (x == ONC_REJECT_AUTH_ERROR) {
        uint32_t e;
        TRY(bytes_try_u32(&v, &e));
        if (e > ONC_AUTH_STAT_MAX) return o_error(ONC_ERR_INVALID_AUTH_ERROR, e, 0);
        r->auth_error = e;
        return O_OK;
    }
    return o_error(ONC_ERR_INVALID_REJECTED_REPLY_TYPE, x, 0);
}

/* ReplyBody::try_from(Bytes) — reply_body.rs:85-98; AcceptedReply accepted_reply.rs:92-104 */
static o_err reply_try_from_bytes(o_bytes v, o_reply_body* r) {
    uint32_t x;
    TRY(bytes_try_u32(&v, &x));
    r->variant = x;
    if (x == ONC_REPLY_ACCEPTED) {
        TRY(auth_try_from_bytes(v, &r->accepted.verf));
        bytes_advance(&v, auth_serialised_len(&r->accepted.verf));
        return accepted_status_try_from_bytes(v, &r->accepted.status);
    }
    if (x == ONC_REPLY_DENIED) return rejected_try_from_bytes(v, &r->denied);
    return o_error(ONC_ERR_INVALID_REPLY_TYPE, x, 0);
}

/* MessageType::try_from(Bytes) — rpc_message.rs:84-92 */
static o_err message_type_try_from_bytes(o_bytes v, o_message* m) {
    uint32_t x;
    TRY(bytes_try_u32(&v, &x));
    m->msg_type = x;
    if (x == ONC_MSG_CALL) return call_try_from_bytes(v, &m->call);
    if (x == ONC_MSG_REPLY) return reply_try_from_bytes(v, &m->reply);
    return o_error(ONC_ERR_INVALID_MESSAGE_TYPE, x, 0);
}

/* RpcMessage::try_from(Bytes) — rpc_message.rs:277-313 */
static o_err message_try_from_bytes(const uint8_t* buf, uint64_t len, o_message* m) {
    memset(m, 0, sizeof(*m));
    o_bytes v = {buf, len};
    uint64_t original_buffer_len = len;
    uint32_t want32;
    TRY(expected_message_len(buf, len, &want32));
    uint64_t want = want32;
    if (original_buffer_len != want)
        return o_error(ONC_ERR_INCOMPLETE_MESSAGE, (uint32_t)original_buffer_len, (uint32_t)want);
    bytes_advance(&v, 4);
    TRY(bytes_try_u32(&v, &m->xid));
    TRY(message_type_try_from_bytes(v, m));
    uint64_t parsed_len = message_serialised_len(m);
    if (parsed_len != original_buffer_len)
        return o_error(ONC_ERR_INCOMPLETE_MESSAGE, (uint32_t)original_buffer_len, (uint32_t)parsed_len);
    return O_OK;
}

/* ---------------------------------------------------------------------- */
/* Public entry points                                                    */
/* ---------------------------------------------------------------------- */

int32_t oracle_decode_message(const uint8_t* base, const uint8_t* buf, uint64_t len, int mode,
                              uint64_t unix_slot_base, onc_msg* msg, onc_unix_params unix[2],
                              uint32_t* aux0, uint32_t* aux1) {
    o_message m;
    o_err e = mode == ONC_DECODE_BYTES ? message_try_from_bytes(buf, len, &m)
                                       : message_try_from_slice(buf, len, &m);
    *aux0 = e.a0;
    *aux1 = e.a1;
    if (e.code != ONC_OK) {
        memset(msg, 0, sizeof(*msg));
        return e.code;
    }
    message_to_desc(&m, base, unix_slot_base, msg, unix);
    return ONC_OK;
}

int32_t oracle_encode_message(const onc_msg* msg, const onc_unix_params* unix_table,
                              const uint8_t* auth_arena, const uint8_t* payload_arena,
                              uint8_t* out, uint64_t cap, uint64_t* written,
                              uint64_t* serialised_len) {
    o_message m;
    *written = 0;
    *serialised_len = 0;
    o_err e = message_from_desc(msg, unix_table, auth_arena, payload_arena, &m);
    if (e.code != ONC_OK) return e.code;
    e = encode_validate(&m);
    if (e.code != ONC_OK) return e.code;
    *serialised_len = message_serialised_len(&m);
    o_writer w = {out, cap, 0};
    e = message_serialise_into(&w, &m);
    *written = w.pos;
    return e.code;
}

/* The library's placement of a record whose Call credential is an AUTH_UNIX
 * auth that declares its length (include/onc_rpc.h onc_auth, ABI 6/7 — the
 * library's own contract, not a reference behaviour): its length pass plans
 * that credential from the descriptor alone and checks the parameter block
 * only while writing. So a record whose only failure is that block's check
 * (a panic of AuthUnixParams::new / Gids, or declared != serialised length)
 * still takes the extent the descriptor declares: its header is a
 * placeholder — the record mark of the extent (rpc_message.rs:156), then
 * zero bytes — and its payload is in place, so the stream stays framable.
 * Returns 1 with that extent and header size when the credential is such a
 * declared auth, its block fails, and every check of the declared plan
 * passes (encode.hip plan_record<true>); else 0 (the record takes no bytes). */
static int declared_extent(const onc_msg* d, const onc_unix_params* unix_table, uint64_t* len, uint64_t* hdr) {
    /* one auth: serialised_len (id + body) and associated_data_len bound */
    uint64_t aw[2] = {0, 0}, assoc[2] = {0, 0};
    const onc_auth* auths[2] = {&d->cred, &d->verf};
    if (d->msg_type != ONC_MSG_CALL) return 0;       /* only a Call's credential is deferred */
    if (ONC_AUTH_KIND(d->cred) != ONC_KIND_UNIX || ONC_AUTH_LEN(d->cred) == 0) return 0;
    {   /* the deferred block check itself must be what fails */
        const onc_unix_params* p = &unix_table[d->cred.ref];
        const int bad = p->name_len > ONC_MAX_MACHINE_NAME_LEN || p->ngids > ONC_MAX_GIDS ||
                        ONC_AUTH_LEN(d->cred) != 20 + 4 * ((p->name_len + 3) / 4) + 4 * p->ngids;
        if (!bad) return 0;
    }
    for (int k = 0; k < 2; k++) {
        const onc_auth* a = auths[k];
        const uint32_t kind = ONC_AUTH_KIND(*a), l = ONC_AUTH_LEN(*a);
        if (kind > ONC_KIND_UNKNOWN) return 0;
        if (k == 0) {                                 /* the declared credential */
            if (l < 20 || (l & 3) || l > 20 + 4 * 64 + 4 * 16) return 0;   /* implausible */
            aw[k] = 8 + l;
            assoc[k] = l - 8;                         /* > 200 exactly when the true value is */
        } else if (kind == ONC_KIND_UNIX) {
            const onc_unix_params* p = &unix_table[a->ref];
            if (p->name_len > ONC_MAX_MACHINE_NAME_LEN || p->ngids > ONC_MAX_GIDS) return 0;
            if (l != 0 && l != 20 + 4 * ((p->name_len + 3) / 4) + 4 * p->ngids) return 0;   /* declared != serialised */
            aw[k] = 8 + 20 + 4 * ((p->name_len + 3) / 4) + 4ull * p->ngids;
            assoc[k] = 12 + p->name_len + 4ull * p->ngids;
        } else {
            aw[k] = 8 + l + oracle_pad_length(l);
            assoc[k] = l;
        }
    }
    const uint64_t h = 28 + aw[0] + aw[1], body = d->payload_len;
    if ((h + body) & 0xFFFFFFFF80000000ull) return 0;
    if (assoc[0] > ONC_MAX_AUTH_LEN || assoc[1] > ONC_MAX_AUTH_LEN) return 0;
    *len = h + body;
    *hdr = h;
    return 1;
}

void oracle_encode_batch(uint64_t n, const onc_msg* msgs, const onc_unix_params* unix_table,
                         const uint8_t* auth_arena, const uint8_t* payload_arena,
                         uint8_t* out, uint64_t out_cap, uint64_t* rec_off,
                         int32_t* status, uint32_t* rec_len) {
    uint64_t off = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t written, slen;
        uint64_t cap = out_cap > off ? out_cap - off : 0;
        int32_t st = oracle_encode_message(&msgs[i], unix_table, auth_arena, payload_arena,
                                           cap ? out + off : out, cap, &written, &slen);
        uint64_t len = (st == ONC_OK || st == ONC_ENC_WRITE_ZERO) ? slen : 0;
        uint64_t dlen, dhdr;
        if (len == 0 && st != ONC_OK && declared_extent(&msgs[i], unix_table, &dlen, &dhdr)) {
            /* failed a deferred block check only: the declared extent, the
             * placeholder header (record mark, zeros), payload copied */
            len = dlen;
            const onc_msg* d = &msgs[i];
            const uint32_t mark = (uint32_t)(dlen - 4) | 0x80000000u;
            for (uint64_t b = 0; b < dlen && b < cap; b++)
                out[off + b] = b < 4 ? (uint8_t)(mark >> (24 - 8 * b))
                                     : b < dhdr ? 0 : payload_arena[d->payload_off + (b - dhdr)];
        }
        if (rec_off) rec_off[i] = off;
        if (status) status[i] = st;
        if (rec_len) rec_len[i] = (uint32_t)len;
        off += len;
    }
    if (rec_off) rec_off[n] = off;
}

/* AUTH_UNIX slots (the library's output layout, include/onc_rpc.h
 * onc_decoded): the OK records of each 64-record group [64g, 64g + 64) put
 * their parameter sets in consecutive slots from 128g, in record order,
 * credential before verifier; onc_auth.ref names the slot. `k` counts the
 * group's slots so far (reset at every group start). */
static void place_unix(uint64_t i, uint64_t* k, onc_msg* m, onc_unix_params* unix_params,
                       const onc_unix_params u[2], int cred_unix, int verf_unix) {
    if ((i & 63) == 0) *k = 0;
    const uint64_t g = 2 * (i & ~(uint64_t)63);
    if (cred_unix) {
        m->cred.ref = g + *k;
        unix_params[g + (*k)++] = u[0];
    }
    if (verf_unix) {
        m->verf.ref = g + *k;
        unix_params[g + (*k)++] = u[1];
    }
}

/* lo is a multiple of 64 (or 0): groups are never split between calls */
static void decode_range(const uint8_t* wire, const uint64_t* rec_off, uint64_t lo, uint64_t hi,
                         int mode, onc_msg* msgs, onc_unix_params* unix_params, int32_t* status,
                         uint32_t* aux0, uint32_t* aux1) {
    uint64_t k = 0;
    for (uint64_t i = lo; i < hi; i++) {
        onc_unix_params u[2];
        memset(u, 0, sizeof(u));
        uint64_t a = rec_off[i], b = rec_off[i + 1];
        int32_t st = oracle_decode_message(wire, wire + a, b - a, mode, 2 * i, &msgs[i], u,
                                           &aux0[i], &aux1[i]);
        status[i] = st;
        int cred_unix = 0, verf_unix = 0;
        if (st == ONC_OK) {
            cred_unix = ONC_AUTH_KIND(msgs[i].cred) == ONC_KIND_UNIX && msgs[i].msg_type == ONC_MSG_CALL;
            verf_unix = ONC_AUTH_KIND(msgs[i].verf) == ONC_KIND_UNIX &&
                        (msgs[i].msg_type == ONC_MSG_CALL || msgs[i].reply_stat == ONC_REPLY_ACCEPTED);
        }
        place_unix(i, &k, &msgs[i], unix_params, u, cred_unix, verf_unix);
    }
}

void oracle_decode_batch(const uint8_t* wire, const uint64_t* rec_off, uint64_t n, int mode,
                         onc_msg* msgs, onc_unix_params* unix_params, int32_t* status,
                         uint32_t* aux0, uint32_t* aux1) {
    decode_range(wire, rec_off, 0, n, mode, msgs, unix_params, status, aux0, aux1);
}

typedef struct {
    const uint8_t* wire;
    const uint64_t* rec_off;
    uint64_t lo, hi;
    int mode;
    onc_msg* msgs;
    onc_unix_params* unix_params;
    int32_t* status;
    uint32_t *aux0, *aux1;
} decode_job;

static void* decode_thread(void* arg) {
    decode_job* j = (decode_job*)arg;
    decode_range(j->wire, j->rec_off, j->lo, j->hi, j->mode, j->msgs, j->unix_params, j->status,
                 j->aux0, j->aux1);
    return NULL;
}

void oracle_decode_batch_mt(const uint8_t* wire, const uint64_t* rec_off, uint64_t n, int mode,
                            onc_msg* msgs, onc_unix_params* unix_params, int32_t* status,
                            uint32_t* aux0, uint32_t* aux1, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    decode_job jobs[256];
    for (int t = 0; t < threads; t++) {
        /* whole 64-record groups per thread (place_unix) */
        const uint64_t lo = (n * t / threads) & ~(uint64_t)63;
        const uint64_t hi = t + 1 == threads ? n : (n * (t + 1) / threads) & ~(uint64_t)63;
        decode_job j = {wire, rec_off, lo, hi, mode, msgs, unix_params, status, aux0, aux1};
        jobs[t] = j;
        pthread_create(&tid[t], NULL, decode_thread, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
}

/* Framing of a byte stream of back-to-back records: the loop a caller of the
 * reference runs over a socket buffer — expected_message_len
 * (rpc_message.rs:343-367) on the remaining bytes, then a one-message slice
 * of that length (the slice every TryFrom<&[u8]> requires,
 * rpc_message.rs:238-242), until the buffer is used up or the next record
 * is not complete. Writes up to max_records + 1 offsets; result =
 * {n, consumed, status, aux0, aux1}: status ONC_OK when the buffer ends on a
 * record boundary (or max_records were framed), else the expected_message_len
 * error or IncompleteMessage{remaining bytes, wanted} for a record that runs
 * past the end. */
/* serialise_into writes nothing for a message that fails: its panics fire
 * before the first write (flavor.rs:110 assert!, unix_params.rs:47 / :149
 * in the constructors) and the length check returns before it
 * (rpc_message.rs:146-151). A batch output restated as that loop's buffer:
 * the OK records' bytes, in order, from rec_off[0] on (memmove: every record
 * moves toward the start). */
uint64_t oracle_compact(uint8_t* wire, uint64_t* rec_off, const int32_t* status, uint64_t n) {
    uint64_t w = n ? rec_off[0] : 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t a = rec_off[i], len = rec_off[i + 1] - a;
        rec_off[i] = w;
        if (status[i] != ONC_OK) continue;
        if (w != a) memmove(wire + w, wire + a, len);
        w += len;
    }
    if (n) rec_off[n] = w;
    return w;
}

void oracle_frame_stream(const uint8_t* data, uint64_t len, uint64_t* rec_off, uint64_t max_records,
                         uint64_t* result) {
    uint64_t pos = 0, n = 0;
    int32_t st = ONC_OK;
    uint64_t aux0 = 0, aux1 = 0;
    while (pos < len && n < max_records) {
        uint32_t want = 0;
        o_err e = expected_message_len(data + pos, len - pos, &want);
        if (e.code != ONC_OK) {
            st = e.code;
            break;
        }
        if (len - pos < (uint64_t)want) {
            st = ONC_ERR_INCOMPLETE_MESSAGE;
            aux0 = len - pos;
            aux1 = want;
            break;
        }
        rec_off[n++] = pos;
        pos += want;
    }
    rec_off[n] = pos;
    result[0] = n;
    result[1] = pos;
    result[2] = (uint64_t)(int64_t)st;
    result[3] = aux0;
    result[4] = aux1;
}

/* Multi-threaded batch encode (CPU-baseline leg only): what a multi-core
 * caller of the reference does — serialised_len() per record
 * (src/rpc_message.rs:201-204) on every thread, an exclusive scan of the
 * lengths, then serialise_into() of each thread's contiguous record range
 * into its own region of the shared buffer. Same outputs as
 * oracle_encode_batch when out_cap covers the total. */
typedef struct {
    uint64_t lo, hi;
    const onc_msg* msgs;
    const onc_unix_params* unix_table;
    const uint8_t *auth_arena, *payload_arena;
    uint8_t* out;
    uint64_t* rec_off;
    int32_t* status;
    uint32_t* rec_len;
    int phase;
} encode_job;

static void* encode_thread(void* arg) {
    encode_job* j = (encode_job*)arg;
    for (uint64_t i = j->lo; i < j->hi; i++) {
        uint64_t written = 0, slen = 0;
        if (j->phase == 0) {
            int32_t st = oracle_encode_message(&j->msgs[i], j->unix_table, j->auth_arena,
                                               j->payload_arena, NULL, 0, &written, &slen);
            j->rec_len[i] = (st == ONC_OK || st == ONC_ENC_WRITE_ZERO) ? (uint32_t)slen : 0;
        } else {
            const uint64_t off = j->rec_off[i];
            j->status[i] = oracle_encode_message(&j->msgs[i], j->unix_table, j->auth_arena,
                                                 j->payload_arena, j->out + off, j->rec_len[i],
                                                 &written, &slen);
        }
    }
    return NULL;
}

void oracle_encode_batch_mt(uint64_t n, const onc_msg* msgs, const onc_unix_params* unix_table,
                            const uint8_t* auth_arena, const uint8_t* payload_arena, uint8_t* out,
                            uint64_t* rec_off, int32_t* status, uint32_t* rec_len, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    encode_job jobs[256];
    for (int phase = 0; phase < 2; phase++) {
        if (phase == 1) {
            uint64_t off = 0;
            for (uint64_t i = 0; i < n; i++) {
                rec_off[i] = off;
                off += rec_len[i];
            }
            rec_off[n] = off;
        }
        for (int t = 0; t < threads; t++) {
            encode_job j = {n * t / threads, n * (t + 1) / threads, msgs, unix_table, auth_arena,
                            payload_arena, out, rec_off, status, rec_len, phase};
            jobs[t] = j;
            pthread_create(&tid[t], NULL, encode_thread, &jobs[t]);
        }
        for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    }
}

int32_t oracle_expected_message_len(const uint8_t* data, uint64_t len, uint32_t* out) {
    uint32_t want = 0;
    o_err e = expected_message_len(data, len, &want);
    *out = want;
    return e.code;
}

int32_t oracle_auth_decode(const uint8_t* buf, uint64_t len, int mode, onc_auth* auth,
                           onc_unix_params* unix, uint64_t* consumed) {
    o_auth a;
    o_err e;
    if (mode == ONC_DECODE_BYTES) {
        o_bytes v = {buf, len};
        e = auth_try_from_bytes(v, &a);
        *consumed = e.code == ONC_OK ? auth_serialised_len(&a) : 0;
    } else {
        o_cursor c = {buf, len, 0};
        e = auth_from_cursor(&c, &a);
        *consumed = c.pos;
    }
    if (e.code != ONC_OK) return e.code;
    auth_to_desc(&a, buf, 0, auth, unix);
    return ONC_OK;
}

int32_t oracle_auth_encode(const onc_auth* auth, const onc_unix_params* unix_table,
                           const uint8_t* arena, uint8_t* out, uint64_t cap, uint64_t* written) {
    o_auth a;
    *written = 0;
    o_err e = auth_from_desc(auth, unix_table, arena, &a);
    if (e.code != ONC_OK) return e.code;
    if (auth_associated_data_len(&a) > ONC_MAX_AUTH_LEN) return ONC_ENC_AUTH_GT_200;
    o_writer w = {out, cap, 0};
    e = auth_serialise_into(&w, &a);
    *written = w.pos;
    return e.code;
}

uint32_t oracle_auth_serialised_len(const onc_auth* auth, const onc_unix_params* unix_table) {
    o_auth a;
    static const uint8_t dummy[1] = {0};
    if (auth_from_desc(auth, unix_table, dummy, &a).code != ONC_OK) return 0;
    return (uint32_t)auth_serialised_len(&a);
}

uint32_t oracle_auth_associated_data_len(const onc_auth* auth, const onc_unix_params* unix_table) {
    o_auth a;
    static const uint8_t dummy[1] = {0};
    if (auth_from_desc(auth, unix_table, dummy, &a).code != ONC_OK) return 0;
    return (uint32_t)auth_associated_data_len(&a);
}

int32_t oracle_unix_params_decode(const uint8_t* buf, uint64_t len, int mode, uint32_t expected_len,
                                  onc_unix_params* out, uint64_t* consumed) {
    o_unix p;
    o_err e;
    if (mode == ONC_DECODE_BYTES) {
        o_bytes v = {buf, len};
        e = unix_try_from_bytes(v, &p);
        *consumed = e.code == ONC_OK ? unix_serialised_len(&p) : 0;
    } else {
        o_cursor c = {buf, len, 0};
        e = unix_from_cursor(&c, expected_len, &p);
        *consumed = c.pos;
    }
    if (e.code != ONC_OK) return e.code;
    o_auth a;
    memset(&a, 0, sizeof(a));
    a.kind = O_AUTH_UNIX;
    a.unix = p;
    onc_auth d;
    auth_to_desc(&a, buf, 0, &d, out);
    return ONC_OK;
}

int32_t oracle_unix_params_encode(const onc_unix_params* p, const uint8_t* arena, uint8_t* out,
                                  uint64_t cap, uint64_t* written) {
    onc_auth d = {ONC_AUTH_UNIX, ONC_AUTH_PACK(ONC_KIND_UNIX, 0), 0};
    o_auth a;
    *written = 0;
    o_err e = auth_from_desc(&d, p, arena, &a);
    if (e.code != ONC_OK) return e.code;
    o_writer w = {out, cap, 0};
    e = unix_serialise_into(&w, &a.unix);
    *written = w.pos;
    return e.code;
}

int32_t oracle_opaque_from_wire(const uint8_t* buf, uint64_t len, uint64_t max_len,
                                uint64_t* body_off, uint64_t* body_len, uint64_t* consumed) {
    o_cursor c = {buf, len, 0};
    o_slice s = {buf, 0};
    o_err e = opaque_from_wire(&c, max_len, &s);
    *consumed = c.pos;
    *body_off = (uint64_t)(s.ptr - buf);
    *body_len = s.len;
    return e.code;
}

int32_t oracle_opaque_encode(const uint8_t* body, uint32_t len, uint8_t* out, uint64_t cap,
                             uint64_t* written) {
    o_writer w = {out, cap, 0};
    o_slice s = {body, len};
    o_err e = opaque_serialise_into(&w, s);
    *written = w.pos;
    return e.code;
}

/* ---------------------------------------------------------------------- */
/* Body-level roots (ONC_ROOT_*): each type's own TryFrom / serialise_into */
/* ---------------------------------------------------------------------- */

/* AuthError::try_from(Bytes) — rejected_reply.rs:215-236 */
static o_err auth_error_try_from_bytes(o_bytes v, uint32_t* e) {
    uint32_t x;
    TRY(bytes_try_u32(&v, &x));
    if (x > ONC_AUTH_STAT_MAX) return o_error(ONC_ERR_INVALID_AUTH_ERROR, x, 0);
    *e = x;
    return O_OK;
}

/* AcceptedReply::from_cursor — accepted_reply.rs:35-40 */
static o_err accepted_reply_from_cursor(o_cursor* c, o_accepted_reply* r) {
    TRY(auth_from_cursor(c, &r->verf));
    return accepted_status_from_cursor(c, &r->status);
}

/* AcceptedReply::try_from(Bytes) — accepted_reply.rs:92-104 */
static o_err accepted_reply_try_from_bytes(o_bytes v, o_accepted_reply* r) {
    TRY(auth_try_from_bytes(v, &r->verf));
    bytes_advance(&v, auth_serialised_len(&r->verf));
    return accepted_status_try_from_bytes(v, &r->status);
}

/* The decoded value of a root as a descriptor (include/onc_rpc.h "Descriptor
 * shape of a root's value"); *consumed = the value's serialised_len(). */
int32_t oracle_decode_body(int root, const uint8_t* base, const uint8_t* buf, uint64_t len, int mode,
                           uint32_t param, uint64_t unix_slot_base, onc_msg* msg, onc_unix_params unix[2],
                           uint32_t* aux0, uint32_t* aux1, uint32_t* consumed) {
    o_message m;
    memset(&m, 0, sizeof(m));
    memset(msg, 0, sizeof(*msg));
    *consumed = 0;
    *aux0 = *aux1 = 0;
    if (root == ONC_ROOT_RPC_MESSAGE) {
        int32_t st = oracle_decode_message(base, buf, len, mode, unix_slot_base, msg, unix, aux0, aux1);
        if (st == ONC_OK) *consumed = (uint32_t)len;
        return st;
    }
    const int bytes = mode == ONC_DECODE_BYTES;
    o_cursor c = {buf, len, 0};
    o_bytes v = {buf, len};
    o_err e = O_OK;
    uint64_t slen = 0;
    /* the message-shaped roots fill m, then message_to_desc */
    switch (root) {
        case ONC_ROOT_MESSAGE_TYPE:
            e = bytes ? message_type_try_from_bytes(v, &m) : message_type_from_cursor(&c, &m);
            if (e.code == ONC_OK) slen = message_serialised_len(&m) - 8;
            break;
        case ONC_ROOT_CALL_BODY:
            m.msg_type = ONC_MSG_CALL;
            e = bytes ? call_try_from_bytes(v, &m.call) : call_from_cursor(&c, &m.call);
            if (e.code == ONC_OK) slen = call_serialised_len(&m.call);
            break;
        case ONC_ROOT_REPLY_BODY:
            m.msg_type = ONC_MSG_REPLY;
            e = bytes ? reply_try_from_bytes(v, &m.reply) : reply_from_cursor(&c, &m.reply);
            if (e.code == ONC_OK) slen = reply_serialised_len(&m.reply);
            break;
        case ONC_ROOT_ACCEPTED_REPLY:
            m.msg_type = ONC_MSG_REPLY;
            m.reply.variant = ONC_REPLY_ACCEPTED;
            e = bytes ? accepted_reply_try_from_bytes(v, &m.reply.accepted)
                      : accepted_reply_from_cursor(&c, &m.reply.accepted);
            /* AcceptedReply::serialised_len — accepted_reply.rs:64-66 */
            if (e.code == ONC_OK)
                slen = auth_serialised_len(&m.reply.accepted.verf) +
                       accepted_status_serialised_len(&m.reply.accepted.status);
            break;
        case ONC_ROOT_ACCEPTED_STATUS:
            m.msg_type = ONC_MSG_REPLY;
            m.reply.variant = ONC_REPLY_ACCEPTED;
            e = bytes ? accepted_status_try_from_bytes(v, &m.reply.accepted.status)
                      : accepted_status_from_cursor(&c, &m.reply.accepted.status);
            if (e.code == ONC_OK) slen = accepted_status_serialised_len(&m.reply.accepted.status);
            break;
        case ONC_ROOT_REJECTED_REPLY:
            m.msg_type = ONC_MSG_REPLY;
            m.reply.variant = ONC_REPLY_DENIED;
            e = bytes ? rejected_try_from_bytes(v, &m.reply.denied) : rejected_from_cursor(&c, &m.reply.denied);
            if (e.code == ONC_OK) slen = rejected_serialised_len(&m.reply.denied);
            break;
        case ONC_ROOT_AUTH_ERROR:
            m.msg_type = ONC_MSG_REPLY;
            m.reply.variant = ONC_REPLY_DENIED;
            m.reply.denied.variant = ONC_REJECT_AUTH_ERROR;
            e = bytes ? auth_error_try_from_bytes(v, &m.reply.denied.auth_error)
                      : auth_error_from_cursor(&c, &m.reply.denied.auth_error);
            if (e.code == ONC_OK) slen = 4; /* AuthError::serialised_len rejected_reply.rs:210-212 */
            break;
        case ONC_ROOT_AUTH_FLAVOR:
        case ONC_ROOT_AUTH_UNIX_PARAMS:
        case ONC_ROOT_OPAQUE: {
            o_auth a;
            memset(&a, 0, sizeof(a));
            if (root == ONC_ROOT_AUTH_FLAVOR) {
                e = bytes ? auth_try_from_bytes(v, &a) : auth_from_cursor(&c, &a);
                if (e.code == ONC_OK) slen = auth_serialised_len(&a);
            } else if (root == ONC_ROOT_AUTH_UNIX_PARAMS) {
                a.kind = O_AUTH_UNIX;
                e = bytes ? unix_try_from_bytes(v, &a.unix) : unix_from_cursor(&c, param, &a.unix);
                if (e.code == ONC_OK) slen = unix_serialised_len(&a.unix);
            } else {
                /* the descriptor's 24-bit length bounds max_len (onc_rpc.h ONC_OPAQUE_MAX_LEN) */
                uint64_t max_len = param < ONC_OPAQUE_MAX_LEN ? param : ONC_OPAQUE_MAX_LEN;
                o_bytes body;
                if (bytes) {
                    e = bytes_try_array(&v, max_len, &body);
                } else {
                    o_slice s;
                    e = opaque_from_wire(&c, max_len, &s);
                    body.ptr = s.ptr;
                    body.len = s.len;
                }
                a.kind = O_AUTH_NONE;
                if (e.code == ONC_OK) {
                    a.data.ptr = body.ptr;
                    a.data.len = body.len;
                    slen = opaque_serialised_len(body.len);
                }
            }
            *aux0 = e.a0;
            *aux1 = e.a1;
            if (e.code != ONC_OK) return e.code;
            msg->msg_type = ONC_MSG_CALL;
            auth_to_desc(&a, base, unix_slot_base, &msg->cred, &unix[0]);
            if (root == ONC_ROOT_AUTH_UNIX_PARAMS) msg->cred.id = ONC_AUTH_UNIX;
            *consumed = (uint32_t)slen;
            return ONC_OK;
        }
        default:
            return ONC_RC_EINVAL;
    }
    *aux0 = e.a0;
    *aux1 = e.a1;
    if (e.code != ONC_OK) return e.code;
    message_to_desc(&m, base, unix_slot_base, msg, unix);
    if (root == ONC_ROOT_ACCEPTED_STATUS) memset(&msg->verf, 0, sizeof(msg->verf));   /* no verifier in the value */
    *consumed = (uint32_t)slen;
    return ONC_OK;
}

/* Shape check of a descriptor for `root` (include/onc_rpc.h). */
static int root_shape_ok(const onc_msg* d, int root) {
    int call = d->msg_type == ONC_MSG_CALL, reply = d->msg_type == ONC_MSG_REPLY;
    int acc = reply && d->reply_stat == ONC_REPLY_ACCEPTED, den = reply && d->reply_stat == ONC_REPLY_DENIED;
    uint32_t ck = ONC_AUTH_KIND(d->cred), cl = ONC_AUTH_LEN(d->cred);
    switch (root) {
        case ONC_ROOT_MESSAGE_TYPE: return call || reply;
        case ONC_ROOT_CALL_BODY:
        case ONC_ROOT_AUTH_FLAVOR: return call;
        case ONC_ROOT_AUTH_UNIX_PARAMS: return call && ck == ONC_KIND_UNIX;
        case ONC_ROOT_OPAQUE: return call && ck != ONC_KIND_UNIX && ck <= ONC_KIND_UNKNOWN && cl <= ONC_OPAQUE_ENCODE_MAX;
        case ONC_ROOT_REPLY_BODY: return reply;
        case ONC_ROOT_ACCEPTED_REPLY:
        case ONC_ROOT_ACCEPTED_STATUS: return acc;
        case ONC_ROOT_REJECTED_REPLY: return den;
        case ONC_ROOT_AUTH_ERROR: return den && d->stat == ONC_REJECT_AUTH_ERROR;
        default: return 0;
    }
}

/* `root`::serialise_into of a descriptor (include/onc_rpc.h
 * onc_encode_body_lengths for the checks and their order). */
int32_t oracle_encode_body(int root, const onc_msg* msg, const onc_unix_params* unix_table,
                           const uint8_t* auth_arena, const uint8_t* payload_arena, uint8_t* out, uint64_t cap,
                           uint64_t* written, uint64_t* serialised_len) {
    *written = 0;
    *serialised_len = 0;
    if (root == ONC_ROOT_RPC_MESSAGE)
        return oracle_encode_message(msg, unix_table, auth_arena, payload_arena, out, cap, written, serialised_len);
    if (!root_shape_ok(msg, root)) return ONC_ENC_BAD_DESCRIPTOR;
    o_message m;
    o_auth a;
    uint64_t slen = 0, assoc = 0, assoc2 = 0;
    o_err e = O_OK;
    if (root == ONC_ROOT_AUTH_FLAVOR || root == ONC_ROOT_AUTH_UNIX_PARAMS || root == ONC_ROOT_OPAQUE) {
        e = auth_from_desc(&msg->cred, unix_table, auth_arena, &a);
        if (e.code != ONC_OK) return e.code;
        if (root == ONC_ROOT_AUTH_FLAVOR) {
            slen = auth_serialised_len(&a);
            assoc = auth_associated_data_len(&a);
        } else if (root == ONC_ROOT_AUTH_UNIX_PARAMS) {
            slen = unix_serialised_len(&a.unix);
        } else {
            slen = opaque_serialised_len(a.data.len);
        }
    } else if (root == ONC_ROOT_ACCEPTED_STATUS) {
        /* only the status is serialised: the verifier is not read */
        if (msg->stat > ONC_ACCEPT_SYSTEM_ERR) return ONC_ENC_BAD_DESCRIPTOR;
        memset(&m, 0, sizeof(m));
        m.reply.accepted.status.variant = msg->stat;
        m.reply.accepted.status.low = msg->u.mismatch.low;
        m.reply.accepted.status.high = msg->u.mismatch.high;
        m.reply.accepted.status.payload.ptr = payload_arena + msg->payload_off;
        m.reply.accepted.status.payload.len = msg->payload_len;
        slen = accepted_status_serialised_len(&m.reply.accepted.status);
    } else {
        e = message_from_desc(msg, unix_table, auth_arena, payload_arena, &m);
        if (e.code != ONC_OK) return e.code;
        switch (root) {
            case ONC_ROOT_MESSAGE_TYPE: slen = message_serialised_len(&m) - 8; break;
            case ONC_ROOT_CALL_BODY: slen = call_serialised_len(&m.call); break;
            case ONC_ROOT_REPLY_BODY: slen = reply_serialised_len(&m.reply); break;
            case ONC_ROOT_ACCEPTED_REPLY:
                slen = auth_serialised_len(&m.reply.accepted.verf) +
                       accepted_status_serialised_len(&m.reply.accepted.status);
                break;
            case ONC_ROOT_REJECTED_REPLY: slen = rejected_serialised_len(&m.reply.denied); break;
            default: slen = 4; break; /* AUTH_ERROR */
        }
        if (m.msg_type == ONC_MSG_CALL) {
            assoc = auth_associated_data_len(&m.call.cred);
            assoc2 = auth_associated_data_len(&m.call.verf);
        } else if (m.reply.variant == ONC_REPLY_ACCEPTED && root != ONC_ROOT_ACCEPTED_STATUS) {
            assoc2 = auth_associated_data_len(&m.reply.accepted.verf);
        }
    }
    if (slen & 0xFFFFFFFF80000000ull) return ONC_ENC_TOO_LONG;
    if (assoc > ONC_MAX_AUTH_LEN || assoc2 > ONC_MAX_AUTH_LEN) return ONC_ENC_AUTH_GT_200;
    *serialised_len = slen;
    o_writer w = {out, cap, 0};
    switch (root) {
        case ONC_ROOT_MESSAGE_TYPE: /* MessageType::serialise_into rpc_message.rs:55-68 */
            e = w_write_u32(&w, m.msg_type);
            if (e.code == ONC_OK)
                e = m.msg_type == ONC_MSG_CALL ? call_serialise_into(&w, &m.call) : reply_serialise_into(&w, &m.reply);
            break;
        case ONC_ROOT_CALL_BODY: e = call_serialise_into(&w, &m.call); break;
        case ONC_ROOT_REPLY_BODY: e = reply_serialise_into(&w, &m.reply); break;
        case ONC_ROOT_ACCEPTED_REPLY: /* AcceptedReply::serialise_into accepted_reply.rs:58-61 */
            e = auth_serialise_into(&w, &m.reply.accepted.verf);
            if (e.code == ONC_OK) e = accepted_status_serialise_into(&w, &m.reply.accepted.status);
            break;
        case ONC_ROOT_ACCEPTED_STATUS: e = accepted_status_serialise_into(&w, &m.reply.accepted.status); break;
        case ONC_ROOT_REJECTED_REPLY: /* rejected_reply.rs:61-73 */
            e = w_write_u32(&w, m.reply.denied.variant);
            if (e.code == ONC_OK)
                e = m.reply.denied.variant == ONC_REJECT_RPC_MISMATCH
                        ? (w_write_u32(&w, m.reply.denied.low).code == ONC_OK ? w_write_u32(&w, m.reply.denied.high)
                                                                              : o_error(ONC_ENC_WRITE_ZERO, 0, 0))
                        : w_write_u32(&w, m.reply.denied.auth_error);
            break;
        case ONC_ROOT_AUTH_ERROR: e = w_write_u32(&w, m.reply.denied.auth_error); break;
        case ONC_ROOT_AUTH_FLAVOR: e = auth_serialise_into(&w, &a); break;
        case ONC_ROOT_AUTH_UNIX_PARAMS: e = unix_serialise_into(&w, &a.unix); break;
        default: e = opaque_serialise_into(&w, a.data); break; /* OPAQUE */
    }
    *written = w.pos;
    return e.code;
}

void oracle_encode_body_batch(int root, uint64_t n, const onc_msg* msgs, const onc_unix_params* unix_table,
                              const uint8_t* auth_arena, const uint8_t* payload_arena, uint8_t* out,
                              uint64_t out_cap, uint64_t* rec_off, int32_t* status, uint32_t* rec_len) {
    uint64_t off = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t written, slen;
        uint64_t cap = out_cap > off ? out_cap - off : 0;
        int32_t st = oracle_encode_body(root, &msgs[i], unix_table, auth_arena, payload_arena, cap ? out + off : out,
                                        cap, &written, &slen);
        uint64_t len = (st == ONC_OK || st == ONC_ENC_WRITE_ZERO) ? slen : 0;
        if (rec_off) rec_off[i] = off;
        if (status) status[i] = st;
        if (rec_len) rec_len[i] = (uint32_t)len;
        off += len;
    }
    if (rec_off) rec_off[n] = off;
}

void oracle_decode_body_batch(int root, const uint8_t* wire, const uint64_t* rec_off, uint64_t n, int mode,
                              const uint32_t* param, onc_msg* msgs, onc_unix_params* unix_params, int32_t* status,
                              uint32_t* aux0, uint32_t* aux1, uint32_t* consumed) {
    uint64_t k = 0;
    for (uint64_t i = 0; i < n; i++) {
        onc_unix_params u[2];
        memset(u, 0, sizeof(u));
        uint64_t a = rec_off[i], b = rec_off[i + 1];
        int32_t st = oracle_decode_body(root, wire, wire + a, b - a, mode, param ? param[i] : 0, 2 * i, &msgs[i], u,
                                        &aux0[i], &aux1[i], &consumed[i]);
        status[i] = st;
        int cred_unix = 0, verf_unix = 0;
        if (st == ONC_OK) {
            cred_unix = ONC_AUTH_KIND(msgs[i].cred) == ONC_KIND_UNIX && msgs[i].msg_type == ONC_MSG_CALL;
            verf_unix = ONC_AUTH_KIND(msgs[i].verf) == ONC_KIND_UNIX &&
                        (msgs[i].msg_type == ONC_MSG_CALL || msgs[i].reply_stat == ONC_REPLY_ACCEPTED) &&
                        root != ONC_ROOT_AUTH_FLAVOR && root != ONC_ROOT_AUTH_UNIX_PARAMS;
        }
        place_unix(i, &k, &msgs[i], unix_params, u, cred_unix, verf_unix);
    }
}
