/*
 * onc_rpc.h — C ABI of the MI355X (gfx950) batch ONC-RPC / XDR codec.
 *
 * This is the drop-in boundary for the reference crate's hot path
 * (domodwyer/onc-rpc v0.3.3, read at /root/reference). Every entry point
 * below names the reference interface it replaces. The reference is a Rust
 * crate whose API is one message per call:
 *
 *   RpcMessage::serialise_into(&self, W: Write)  src/rpc_message.rs:136-164
 *   RpcMessage::serialised_len(&self) -> u32      src/rpc_message.rs:201-204
 *   RpcMessage::try_from(&[u8])                   src/rpc_message.rs:235-271
 *   RpcMessage::try_from(Bytes)                   src/rpc_message.rs:273-314
 *   expected_message_len(&[u8])                   src/rpc_message.rs:343-367
 *
 * Here the caller's per-message loop is replaced by one batch call over N
 * independent records, executed by hand-written HIP kernels on one GPU.
 *
 * Conventions
 *  - Every pointer marked [dev] is device-accessible memory on the codec's
 *    device: device memory (hipMalloc / torch CUDA tensor), or host memory
 *    mapped for the device (onc_host_register, hipHostMalloc / torch pinned
 *    memory), which the kernels then read and write in place over PCIe — a
 *    decode of a socket buffer moves only the header granules it parses.
 *    Nothing is copied to or from the host by these calls; all calls are
 *    asynchronous on the codec's stream.
 *  - The caller owns every buffer (the reference never allocates on decode
 *    and reuses caller buffers on encode, README.md:10-14). The codec only
 *    keeps a small scratch area for the record-offset scan.
 *  - Messages are described by fixed 64-byte descriptors (onc_msg). Opaque
 *    bodies (auth bodies, machine names) and payloads are (offset, length)
 *    references into caller arenas, mirroring the borrowed slices of the
 *    reference's generic `T, P: AsRef<[u8]>` (src/call_body.rs:18-30).
 *  - Per-record results are status codes equal to the reference's Error
 *    variants in declaration order (src/errors.rs:6-97), plus encode-only
 *    codes for the reference's panics and io::Errors.
 */
#ifndef ONC_RPC_H
#define ONC_RPC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: onc_batch carries arena sizes (bounds-checked descriptors), onc_encode
 *    accepts any output address, retired kernel id ONC_K_ENC_FIXUP removed.
 * 3: timing id 10 is ONC_K_FRAME_OFFSETS (the framer's chunk verification
 *    now runs inside frame_chunks; ONC_K_FRAME_VERIFY is gone).
 * 4: body-level roots (ONC_ROOT_*, onc_decode_body, onc_encode_body,
 *    onc_encode_body_lengths); timing id 10 retired (ONC_K_FRAME_OFFSETS
 *    gone, the framer ids after it move down by one).
 * 5: decoded AUTH_UNIX slots compacted per 64-record group (onc_decoded):
 *    a slot's index is only what onc_auth.ref says, no longer 2i / 2i + 1.
 * 6: onc_codec_create_ex + onc_codec_options (kernel choices, chunk sizes and
 *    the decode policy are explicit options; the library reads no
 *    environment variable), onc_codec_set_decode_policy, calls refuse to grow
 *    scratch while the stream is being captured (ONC_RC_ECAPTURE); an
 *    AUTH_UNIX onc_auth carries its declared serialised length (kind_len
 *    bits 0..23, written by the decoder; 0 = not declared). */
/* 7: a record whose declared AUTH_UNIX credential fails a deferred block
 *    check keeps its extent with a placeholder header — the record mark of
 *    the extent, then zeros — instead of zeros alone, so that the stream
 *    stays framable (onc_encode_iov emits the same placeholder as its header
 *    iovec); onc_host_register / onc_host_unregister map a caller's host
 *    buffer (a socket buffer) for the kernels to read and write in place. */
/* 8: onc_compact / onc_compact_iov (a failing record's extent dropped from an
 *    encoded batch: the stream the reference's per-message loop writes);
 *    timing id ONC_K_COMPACT; onc_host_unregister takes a NULL codec and
 *    registrations are counted per range (a pinned range belongs to the
 *    process); the rejected-experiment variant bits (EMIT_PRELOAD,
 *    DEC_AUX_SPARSE, SINGLE_PASS, SP_*) are gone. */
#define ONC_RPC_ABI_VERSION 8

/* ------------------------------------------------------------------------ */
/* Wire discriminants (values are the on-wire u32s)                          */
/* ------------------------------------------------------------------------ */

/* msg_type — src/rpc_message.rs:16-17 */
#define ONC_MSG_CALL  0u
#define ONC_MSG_REPLY 1u

/* reply_stat — src/reply/reply_body.rs:11-12 */
#define ONC_REPLY_ACCEPTED 0u
#define ONC_REPLY_DENIED   1u

/* accept_stat — src/reply/accepted_reply.rs:10-15 */
#define ONC_ACCEPT_SUCCESS       0u
#define ONC_ACCEPT_PROG_UNAVAIL  1u
#define ONC_ACCEPT_PROG_MISMATCH 2u
#define ONC_ACCEPT_PROC_UNAVAIL  3u
#define ONC_ACCEPT_GARBAGE_ARGS  4u
#define ONC_ACCEPT_SYSTEM_ERR    5u

/* reject_stat — src/reply/rejected_reply.rs:10-11 */
#define ONC_REJECT_RPC_MISMATCH 0u
#define ONC_REJECT_AUTH_ERROR   1u

/* auth_stat — src/reply/rejected_reply.rs:13-20 (AUTH_OK .. AUTH_FAILED = 0..7) */
#define ONC_AUTH_STAT_MAX 7u

/* Auth flavor ids — src/auth/flavor.rs:10-12 */
#define ONC_AUTH_NONE  0u
#define ONC_AUTH_UNIX  1u
#define ONC_AUTH_SHORT 2u

/* AuthFlavor variant (descriptor "kind") — src/auth/flavor.rs:18-49.
 * NONE with length 0 is AuthNone(None); with length > 0 AuthNone(Some(_)).
 * UNKNOWN writes/reads `id` as the wire discriminant. */
#define ONC_KIND_NONE    0u
#define ONC_KIND_UNIX    1u
#define ONC_KIND_SHORT   2u
#define ONC_KIND_UNKNOWN 3u

/* Limits — src/auth/flavor.rs:110 (encode), :83 / opaque 200 (decode);
 * src/auth/unix_params.rs:11-12 */
#define ONC_MAX_AUTH_LEN         200u
#define ONC_MAX_MACHINE_NAME_LEN 255u
#define ONC_MAX_GIDS             16u

/* Decode modes: the two reference decoders */
#define ONC_DECODE_SLICE 0 /* TryFrom<&[u8]>  src/rpc_message.rs:235-271 */
#define ONC_DECODE_BYTES 1 /* TryFrom<Bytes>  src/rpc_message.rs:273-314 */

/* Roots: the reference type a body-level call decodes each record as, or
 * serialises each descriptor as (onc_decode_body / onc_encode_body). The
 * reference has TryFrom / serialise_into / serialised_len on every type of
 * a message, not only on RpcMessage; each root is one of
 * them. `param` is a per-record u32 the root needs (else ignored).
 *                               decode (slice | Bytes)              encode (serialise_into)
 *  RPC_MESSAGE      RpcMessage  rpc_message.rs:235-271 | :273-314   :136-164
 *  MESSAGE_TYPE     MessageType from_cursor :39-45 | TryFrom :80-93 :55-68
 *  CALL_BODY        CallBody    call_body.rs:168-175 | :177-210     :98-108
 *  REPLY_BODY       ReplyBody   reply_body.rs:76-83 | :85-98        :45-56
 *  ACCEPTED_REPLY   AcceptedReply accepted_reply.rs:79-86 | :88-105 :58-61
 *  ACCEPTED_STATUS  AcceptedStatus :234-241 | :243-265              :195-211
 *  REJECTED_REPLY   RejectedReply rejected_reply.rs:98-105 | :107-125 :61-73
 *  AUTH_ERROR       AuthError   from_cursor :176-190 | TryFrom :215-236 :194-207
 *  AUTH_FLAVOR      AuthFlavor  flavor.rs:177-184 | :186-222       :106-129
 *  AUTH_UNIX_PARAMS AuthUnixParams from_cursor(r, expected_len = param)
 *                               unix_params.rs:90-129 | TryFrom :248-276  :162-176
 *  OPAQUE           Opaque (crate-private) from_wire(r, max_len = param)
 *                               opaque.rs:72-98 | try_array bytes_ext.rs:25-42  :38-56
 * Descriptor shape of a root's value (decode writes it, encode reads it;
 * fields outside it are zero on decode and ignored on encode):
 *  MESSAGE_TYPE     as RPC_MESSAGE without xid
 *  CALL_BODY        msg_type CALL, u.call, cred, verf, payload
 *  REPLY_BODY       msg_type REPLY, reply_stat, stat, auth_stat, u.mismatch,
 *                   verf and payload (accepted)
 *  ACCEPTED_REPLY   the same with reply_stat ACCEPTED
 *  ACCEPTED_STATUS  msg_type REPLY, reply_stat ACCEPTED, stat, u.mismatch,
 *                   payload (no verifier)
 *  REJECTED_REPLY   msg_type REPLY, reply_stat DENIED, stat, u.mismatch / auth_stat
 *  AUTH_ERROR       msg_type REPLY, reply_stat DENIED, stat AUTH_ERROR, auth_stat
 *  AUTH_FLAVOR      msg_type CALL, the value in cred (AUTH_UNIX: slot cred.ref)
 *  AUTH_UNIX_PARAMS msg_type CALL, cred kind UNIX (slot cred.ref)
 *  OPAQUE           msg_type CALL, cred kind NONE, its body = the opaque's
 * A descriptor of another shape encodes as ONC_ENC_BAD_DESCRIPTOR. */
#define ONC_ROOT_RPC_MESSAGE      0
#define ONC_ROOT_MESSAGE_TYPE     1
#define ONC_ROOT_CALL_BODY        2
#define ONC_ROOT_REPLY_BODY       3
#define ONC_ROOT_ACCEPTED_REPLY   4
#define ONC_ROOT_ACCEPTED_STATUS  5
#define ONC_ROOT_REJECTED_REPLY   6
#define ONC_ROOT_AUTH_ERROR       7
#define ONC_ROOT_AUTH_FLAVOR      8
#define ONC_ROOT_AUTH_UNIX_PARAMS 9
#define ONC_ROOT_OPAQUE           10
#define ONC_ROOT_COUNT            11
/* Largest opaque body the OPAQUE root encodes: the crate serialises Opaque
 * only for auth bodies (<= 200, flavor.rs:110) and machine names (<= 255,
 * unix_params.rs:149); a longer one is ONC_ENC_BAD_DESCRIPTOR. Decode takes
 * max_len up to ONC_OPAQUE_MAX_LEN (the descriptor's 24-bit length field;
 * the reference calls from_wire with 200 and 255 only): a larger param acts
 * as ONC_OPAQUE_MAX_LEN. */
#define ONC_OPAQUE_ENCODE_MAX 255u
#define ONC_OPAQUE_MAX_LEN    0xFFFFFFu

/* ------------------------------------------------------------------------ */
/* Per-record status codes                                                   */
/* ------------------------------------------------------------------------ */
/* 1..13 are src/errors.rs:6-97 in declaration order.                        */
#define ONC_OK                               0
#define ONC_ERR_INCOMPLETE_MESSAGE           1  /* aux0 = buffer_len, aux1 = expected   errors.rs:14-21 */
#define ONC_ERR_INCOMPLETE_HEADER            2  /* errors.rs:24-25 */
#define ONC_ERR_FRAGMENTED                   3  /* errors.rs:32-33 */
#define ONC_ERR_INVALID_MESSAGE_TYPE         4  /* aux0 = value   errors.rs:42-43 */
#define ONC_ERR_INVALID_REPLY_TYPE           5  /* aux0 = value   errors.rs:52-53 */
#define ONC_ERR_INVALID_REPLY_STATUS         6  /* aux0 = value   errors.rs:59-60 */
#define ONC_ERR_INVALID_AUTH_DATA            7  /* errors.rs:63-64 */
#define ONC_ERR_INVALID_AUTH_ERROR           8  /* aux0 = value   errors.rs:70-71 */
#define ONC_ERR_INVALID_REJECTED_REPLY_TYPE  9  /* aux0 = value   errors.rs:77-78 */
#define ONC_ERR_INVALID_LENGTH              10  /* errors.rs:82-83 */
#define ONC_ERR_INVALID_RPC_VERSION         11  /* aux0 = value   errors.rs:86-87 */
#define ONC_ERR_INVALID_MACHINE_NAME        12  /* errors.rs:91-92 — never produced by a decoder */
#define ONC_ERR_IO_UNEXPECTED_EOF           13  /* IOError(UnexpectedEof, "failed to fill whole buffer")
                                                   errors.rs:95-103 (slice-mode short read) */
/* Encode-only codes (the reference panics or returns io::Error here). */
#define ONC_ENC_TOO_LONG        100 /* io::Error InvalidInput "message length exceeds maximum"
                                       rpc_message.rs:146-151 */
#define ONC_ENC_AUTH_GT_200     101 /* panic: assert!(associated_data_len() <= 200) flavor.rs:110 */
#define ONC_ENC_NAME_GT_255     102 /* panic: AuthUnixParams::new unix_params.rs:149 */
#define ONC_ENC_GIDS_GT_16      103 /* panic: Gids::from_iter unix_params.rs:47 */
#define ONC_ENC_BAD_DESCRIPTOR  104 /* a descriptor the Rust enums cannot represent */
#define ONC_ENC_WRITE_ZERO      105 /* io::Error WriteZero: output capacity exhausted */

/* Batch-level return codes of the API functions */
#define ONC_RC_OK        0
#define ONC_RC_EINVAL   -1
#define ONC_RC_EHIP     -2
#define ONC_RC_ENOMEM   -3
#define ONC_RC_EALIGN   -4
#define ONC_RC_ECAPTURE -5   /* the call would allocate scratch while its stream is being captured
                                into a hipGraph: call onc_codec_reserve before the capture */

/* ------------------------------------------------------------------------ */
/* Descriptors                                                               */
/* ------------------------------------------------------------------------ */

/* opaque_auth — AuthFlavor<T> (src/auth/flavor.rs:18-49). 16 bytes.
 *  id       : wire flavor discriminant. Encode writes 0/1/2 for kinds
 *             NONE/UNIX/SHORT and `id` for UNKNOWN; decode stores the value read.
 *  kind_len : bits 0..23 opaque body length (NONE/SHORT/UNKNOWN),
 *             bits 24..31 ONC_KIND_*.
 *             UNIX (ABI 6): the declared length — AuthUnixParams::serialised_len
 *             (unix_params.rs:219-230: 20 + 4 * ceil(name_len / 4) + 4 * ngids)
 *             — or 0 (not declared). The decoder always declares it. On
 *             encode a declared length lets the length pass (onc_encode,
 *             onc_encode_plan) size the record from the descriptor alone,
 *             without reading the 96-byte parameter block; the emit checks
 *             the block when it serialises it (the AuthUnixParams::new / Gids
 *             panics, the machine name inside the auth arena, and declared ==
 *             serialised length — a mismatch is ONC_ENC_BAD_DESCRIPTOR).
 *             Statuses are the reference order's either way. One placement
 *             difference: a record whose only failure is such a block check
 *             keeps the extent its descriptor declares in the output (every
 *             other failing record takes 0 bytes), so that the records after
 *             it stay where the length pass placed them. Its bytes there are a
 *             placeholder that keeps the stream framable (ABI 7): the record
 *             mark of the extent, BE32((extent - 4) | 1 << 31) as
 *             rpc_message.rs:156 writes it — a receiver's expected_message_len
 *             (:343-367) and onc_frame_stream cut it as one record and go on
 *             to the next — then zero bytes up to the payload, which is in
 *             place (a receiver's decode of it fails: InvalidRpcVersion(0)).
 *             onc_encode_lengths reports the same extents (with every check's
 *             status) and onc_encode_iov places records by them (such a
 *             record: its placeholder as the header iovec, its payload
 *             slice); the body roots check every block up front.
 *  ref      : NONE/SHORT/UNKNOWN: byte offset of the body in the auth arena
 *             (decode: in the wire buffer). UNIX: index into the unix table. */
typedef struct onc_auth {
    uint32_t id;
    uint32_t kind_len;
    uint64_t ref;
} onc_auth;

#define ONC_AUTH_KIND(a)        ((uint32_t)((a).kind_len >> 24))
#define ONC_AUTH_LEN(a)         ((uint32_t)((a).kind_len & 0xFFFFFFu))
#define ONC_AUTH_PACK(kind, len) ((uint32_t)(((uint32_t)(kind) << 24) | ((uint32_t)(len) & 0xFFFFFFu)))

/* RpcMessage<T, P> (src/rpc_message.rs:97-105) with its MessageType,
 * CallBody (src/call_body.rs:17-30) / ReplyBody (src/reply/ *.rs). 64 bytes.
 *
 *  msg_type    ONC_MSG_CALL | ONC_MSG_REPLY
 *  reply_stat  reply: ONC_REPLY_ACCEPTED | ONC_REPLY_DENIED
 *  stat        accepted: ONC_ACCEPT_*; denied: ONC_REJECT_*
 *  auth_stat   denied AUTH_ERROR: AuthError (0..7)
 *  call        program / program_version / procedure (CallBody)
 *  mismatch    low / high of ProgramMismatch or RpcVersionMismatch
 *  payload_*   Call payload or Success payload (raw, unpadded; call_body.rs:107,
 *              accepted_reply.rs:199): encode = payload arena offset,
 *              decode = wire offset
 *  cred        call credentials (unused for replies)
 *  verf        call verifier or accepted-reply verifier */
typedef struct onc_msg {
    uint32_t xid;
    uint8_t  msg_type;
    uint8_t  reply_stat;
    uint8_t  stat;
    uint8_t  auth_stat;
    union {
        struct { uint32_t program, program_version, procedure; } call;
        struct { uint32_t low, high, reserved; } mismatch;
    } u;
    uint32_t payload_len;
    uint64_t payload_off;
    onc_auth cred;
    onc_auth verf;
} onc_msg;

/* AuthUnixParams<T> (src/auth/unix_params.rs:72-82). 96 bytes.
 * name_off is an auth-arena offset (decode: wire offset). */
typedef struct onc_unix_params {
    uint32_t stamp;
    uint32_t uid;
    uint32_t gid;
    uint32_t ngids;
    uint64_t name_off;
    uint32_t name_len;
    uint32_t reserved;
    uint32_t gids[16];
} onc_unix_params;

/* A batch of messages to encode. [dev] pointers. auth_arena and
 * payload_arena may alias (e.g. both = the wire buffer of a decoded batch).
 * The three sizes bound every reference a descriptor makes: a unix-table
 * index >= unix_count, an auth body / machine name [off, off + len) beyond
 * auth_len or a payload beyond payload_len makes that record
 * ONC_ENC_BAD_DESCRIPTOR (checked before anything is read through it), so a
 * malformed descriptor can never make a kernel read outside the arenas.
 * Zero-length bodies and payloads are not checked (their offsets are never
 * dereferenced). The reference's owned types cannot express such a
 * reference; the check replaces an out-of-bounds read, not a reference
 * behaviour. The sizes must be true: the encoder may read any byte of
 * [payload_arena, payload_arena + payload_len) (it loads whole 16-byte
 * windows at each output chunk's own source bytes when they all lie in the
 * arena), never a byte outside it. */
typedef struct onc_batch {
    uint64_t               n;
    const onc_msg*         msgs;          /* [dev] n descriptors */
    const onc_unix_params* unix_params;   /* [dev] AUTH_UNIX table (may be NULL if unix_count == 0) */
    const uint8_t*         auth_arena;    /* [dev] auth bodies + machine names */
    const uint8_t*         payload_arena; /* [dev] payloads */
    uint64_t               unix_count;    /* entries in unix_params */
    uint64_t               auth_len;      /* bytes in auth_arena */
    uint64_t               payload_len;   /* bytes in payload_arena */
} onc_batch;

/* Decode outputs. [dev] pointers.
 * unix_params has 2*n slots. The AUTH_UNIX parameter sets of the OK records
 * of each 64-record group [64g, 64g + 64) (counted from the call's first
 * record) take consecutive slots from 128g, in record order, credential
 * before verifier; onc_auth.ref holds the slot index. Slots past a group's
 * last set are not written. (Packed, the sets of a group are written as
 * whole contiguous lines: a slot pair per record, 2i / 2i + 1, scattered
 * them 192 bytes apart.)
 * Offsets in the decoded descriptors are wire-buffer offsets, so a decoded
 * batch can be re-encoded with auth_arena = payload_arena = wire and
 * unix_params as the AUTH_UNIX table (unix_count = 2n).
 * For a record with status != ONC_OK the descriptor is all zero and it takes
 * no slot. */
typedef struct onc_decoded {
    onc_msg*         msgs;        /* n */
    onc_unix_params* unix_params; /* 2n */
    int32_t*         status;      /* n */
    uint32_t*        aux0;        /* n: buffer_len or the offending value */
    uint32_t*        aux1;        /* n: expected (IncompleteMessage) */
} onc_decoded;

/* ------------------------------------------------------------------------ */
/* Codec handle                                                              */
/* ------------------------------------------------------------------------ */

typedef struct onc_codec onc_codec;

/* Decode first-round policy (decode.hip): how much of each record's header
 * the decode's first load round fetches. Results never depend on it, only
 * the time. AUTO picks it per launch from the records the previous decode
 * launch on the handle sampled (a word the kernel writes to mapped host
 * memory, read at the next launch without a synchronisation); STANDARD
 * fetches the first 44 bytes (short headers: AUTH_NONE calls, replies);
 * LINE the rest of the record's first 128-byte line (long AUTH_UNIX
 * headers). A hipGraph captures the policy in force when it is captured. */
#define ONC_DECODE_POLICY_AUTO     0
#define ONC_DECODE_POLICY_STANDARD 1
#define ONC_DECODE_POLICY_LINE     2

/* Kernel-variant bits (onc_codec_options.variant): measurement and test
 * switches that force a kernel the codec would otherwise choose per batch.
 * Results are bit-identical under every combination; production leaves 0. */
#define ONC_VARIANT_EMIT_WS          0x200u    /* force the wave-specialised enc_emit */
#define ONC_VARIANT_EMIT_TILE        0x400u    /* force the wave-per-tile enc_emit */
#define ONC_VARIANT_WS_NO_INTERIOR   0x4000u   /* wave-specialised: no interior spans */
#define ONC_VARIANT_WS_NO_FULL       0x8000u   /* wave-specialised: no full-interior spans */
#define ONC_VARIANT_WS_PIPELINE      0x10000u  /* wave-specialised: the pipeline on header-heavy batches too */
#define ONC_VARIANT_EMIT_REPLAN      0x20000u  /* wave-per-tile enc_emit re-plans instead of reading the plan's lengths */
#define ONC_VARIANT_WHOLE_PLAN       0x40000u  /* plan a large batch whole instead of in chunks */

#define ONC_OPT_FORCE_SCAN 0x1u   /* always launch the separate block-scan kernels (tests of that path) */

/* Options of onc_codec_create_ex; all-zero (or a NULL pointer) = the
 * defaults, which are what onc_codec_create uses. The library reads nothing
 * from the environment. */
typedef struct onc_codec_options {
    uint32_t size;           /* sizeof(onc_codec_options), or 0 */
    uint32_t flags;          /* ONC_OPT_* */
    int32_t  decode_policy;  /* ONC_DECODE_POLICY_* */
    uint32_t variant;        /* ONC_VARIANT_* bits (A/B measurements and tests; 0 in production) */
    uint64_t enc_chunk;      /* records per plan + emit chunk of a large encode (rounded down to a
                                multiple of 1024; 0 = 1M) */
    uint64_t frame_chunk;    /* bytes per onc_frame_stream chunk (>= 64; 0 = 64 KiB) */
} onc_codec_options;

/* One handle per device: a HIP stream + scan scratch. `hip_stream` may be
 * NULL (the device's null stream) or a hipStream_t owned by the caller. */
int onc_codec_create(onc_codec** out, int device, void* hip_stream);
int onc_codec_create_ex(onc_codec** out, int device, void* hip_stream, const onc_codec_options* options);
int onc_codec_destroy(onc_codec* codec);
int onc_codec_set_stream(onc_codec* codec, void* hip_stream);
int onc_codec_set_decode_policy(onc_codec* codec, int policy);
int onc_codec_sync(onc_codec* codec);
/* Pre-size the scratch for batches of up to max_records (scan totals, the
 * plan's record lengths), so that later encode / decode / scan calls of up
 * to that many records perform no allocation. Required before capturing
 * calls into a hipGraph: a call that would grow the scratch while its
 * stream is capturing returns ONC_RC_ECAPTURE (outside a capture the
 * scratch grows on demand with a synchronous hipMalloc). onc_frame_stream
 * keeps its own per-chunk scratch, sized by its first call on a stream that
 * long or longer (growing it inside a capture is ONC_RC_ECAPTURE too). */
int onc_codec_reserve(onc_codec* codec, uint64_t max_records);
/* Map a caller's host buffer (a socket buffer: any malloc'd or mmap'd
 * range) for the kernels, so that an encode / decode reads and writes it in
 * place instead of through a staging copy: pins its pages
 * (hipHostRegister, mapped and portable) and returns the device address of
 * `host` in *dev_ptr, usable as any [dev] pointer of this header. The
 * zero-copy counterpart of the reference's borrowed slices
 * (call_body.rs:53-59, opaque.rs:92-97): onc_decode of a registered wire
 * fetches only the 16-byte granules holding the header bytes it parses over
 * the link, never the payloads. Synchronous. A pinned range belongs to the
 * process, not to the codec (destroying the codec leaves it pinned): a
 * register of a range inside one this library pinned maps it and counts one
 * more registration of that range; each onc_host_unregister counts one
 * down and the last unpins it. A range already pinned by its owner
 * (hipHostMalloc, torch's pin_memory) needs no registration: its device
 * address is returned and nothing is recorded (onc_host_unregister of it is
 * then a no-op). The address is for the codec's device. Returns
 * ONC_RC_EINVAL for a NULL pointer or length, or for a range that starts in
 * pinned memory but runs past that pinned allocation; ONC_RC_EHIP if the
 * runtime refuses the range (onc_codec_last_error says why). */
int onc_host_register(onc_codec* codec, void* host, uint64_t len, void** dev_ptr);
/* Undo one onc_host_register of a range this library pinned (`host`: any
 * address inside it; the kernels must be done with it); the last one unpins
 * the range. `codec` may be NULL (it is only where an error is reported):
 * a registration may outlive the codec that made it. */
int onc_host_unregister(onc_codec* codec, void* host);

/* Last HIP error string seen by this handle ("" if none). */
const char* onc_codec_last_error(const onc_codec* codec);
const char* onc_status_str(int32_t status);
int onc_abi_version(void);

/* Per-kernel event timing (for the bench's roofline). `enable` is a bitmask
 * of kernel ids (1 << ONC_K_*; ONC_TIMING_ALL = every kernel, 0 = off): each
 * launch of a selected kernel carries start/stop hipEvents on the codec
 * stream (hipExtLaunchKernelGGL: the dispatch's own timestamps); the
 * accumulated device time and launch count per kernel id are returned by
 * onc_codec_kernel_stats after a sync. Timing only the kernel of interest
 * keeps the event overhead off the other launches. An id names a launch
 * site: ONC_K_ENC_EMIT is either enc_emit kernel; ONC_K_LEN_TILES /
 * ONC_K_LEN_APPLY are onc_scan_lengths' first and second launch (lenblk /
 * lenoff up to 8M records); ONC_K_FRAME_COUNTS the framer's count pass
 * (frame_cblk, or frame_counts ahead of the three-launch scan beyond 512k
 * chunks); ONC_K_FRAME_WRITE its start copy, which up to 512k chunks also
 * sums each chunk's first record index. The body-level calls use the ids of
 * the kernels they launch (ONC_K_ENC_LEN / _ENC_EMIT / _DEC_PARSE). */
#define ONC_K_ENC_LEN      0
#define ONC_K_SCAN_TILES   1
#define ONC_K_ENC_EMIT     2
#define ONC_K_DEC_PARSE    3
#define ONC_K_LEN_TILES    4
#define ONC_K_LEN_APPLY    5
#define ONC_K_IOV_LEN      6
#define ONC_K_IOV_EMIT     7
#define ONC_K_FRAME        8
#define ONC_K_FRAME_WRITE  9
#define ONC_K_FRAME_WALK   10
#define ONC_K_FRAME_COUNTS 11
#define ONC_K_FRAME_GUESS  12
#define ONC_K_COMPACT      13
#define ONC_K_COUNT        14
#define ONC_TIMING_ALL    (-1)
int onc_codec_enable_timing(onc_codec* codec, int enable);
int onc_codec_kernel_stats(onc_codec* codec, double* ms_total /*[ONC_K_COUNT]*/,
                           uint64_t* launches /*[ONC_K_COUNT]*/);
int onc_codec_reset_stats(onc_codec* codec);
const char* onc_kernel_name(int kernel_id);

/* ------------------------------------------------------------------------ */
/* Encode — RpcMessage::serialise_into (src/rpc_message.rs:136-164)          */
/* ------------------------------------------------------------------------ */

/* serialised_len() of every record (src/rpc_message.rs:201-204) plus the
 * encode-time validation of serialise_into (oversize, panics).
 * rec_len[dev,n] receives the length (0 for a record whose status != OK,
 * except a declared AUTH_UNIX record failing only a parameter-block check:
 * its declared extent, as onc_encode places it — onc_auth), so the sum is
 * the size of onc_encode's output; status[dev,n] receives ONC_OK or an
 * ONC_ENC_* code. */
int onc_encode_lengths(onc_codec* codec, const onc_batch* batch,
                       uint32_t* rec_len, int32_t* status);

/* Encode every record back to back into out[dev] (out_cap bytes): the
 * batch equivalent of calling serialise_into for each message in order on
 * one Cursor<Vec<u8>> (a TCP send buffer). `out` may be any byte address —
 * the cursor's current position in a partly filled buffer — and bytes
 * before `out` or at/after out + out_cap are never written (the reference
 * writes at the writer's position, rpc_message.rs:136, and reuses buffers,
 * README.md:11). Whole 16-byte-aligned chunks are written with one store;
 * the chunks at either end of the batch are written byte by byte.
 *   rec_off[dev, n+1]: record i occupies out[rec_off[i], rec_off[i+1]);
 *                      rec_off[n] is the total byte count.
 *   status[dev, n]   : ONC_OK or ONC_ENC_*. Records that fail validation
 *                      occupy 0 bytes — except a declared AUTH_UNIX record
 *                      failing only its deferred parameter-block check, which
 *                      keeps its declared extent as a framable placeholder
 *                      (onc_auth). Bytes at or beyond out_cap are never
 *                      written; records ending beyond it get ONC_ENC_WRITE_ZERO.
 *   rec_len[dev, n]  : optional (may be NULL) serialised lengths.
 * Launches: a length pass and the emit per 1M-record chunk; a batch of at
 * most 512 records is planned and emitted in one launch (the results are the
 * same). */
int onc_encode(onc_codec* codec, const onc_batch* batch,
               uint8_t* out, uint64_t out_cap,
               uint64_t* rec_off, int32_t* status, uint32_t* rec_len);

/* onc_encode in two phases on the handle's stream, so that the length pass
 * of one batch can run while other work (the decode of the previous batch,
 * on another stream) is in flight:
 *   onc_encode_plan : serialised_len() + validation of every record
 *                     (status, optional rec_len) and the placement totals,
 *                     kept in this handle's scratch (enc_len);
 *   onc_encode_emit : the bytes, placed by that plan (enc_emit) — same
 *                     arguments and results as onc_encode.
 * The plan belongs to the handle: emit must name the batch last planned on
 * it (same msgs pointer and n) with the status array the plan filled (the
 * plan's statuses stand; emit adds ONC_ENC_WRITE_ZERO and the status of a
 * declared AUTH_UNIX auth's parameter-block check, onc_auth), else
 * ONC_RC_EINVAL; any other call on the handle in between that uses its
 * scratch (every encode, decode_lengths and scan_lengths call) discards the
 * plan (then ONC_RC_EINVAL too). The descriptors must not change in between,
 * nor the plan's rec_len array when one was given (for a batch with an
 * AUTH_UNIX table the emit reads the record lengths back from it instead of
 * re-planning). onc_encode = plan + emit (for more than 512 records; a
 * smaller batch it encodes in one launch). */
int onc_encode_plan(onc_codec* codec, const onc_batch* batch, int32_t* status, uint32_t* rec_len);
int onc_encode_emit(onc_codec* codec, const onc_batch* batch, uint8_t* out, uint64_t out_cap,
                    uint64_t* rec_off, int32_t* status);

/* Vectored encode (the zero-copy writer the reference
 * plans in README.md:71-75 and rpc_message.rs:19): only the header part of
 * every record (everything before the raw payload) is serialised, into
 * hdr_out[dev] back to back; payloads stay where they are in the batch's
 * payload arena. Record i on the wire is
 *     hdr_out[iov[i].hdr_off, +hdr_len) ++ payload_arena[iov[i].payload_off, +payload_len)
 * and starts at iov[i].wire_off of the equivalent packed send buffer, i.e.
 * the bytes onc_encode would produce, for a writev()/scatter-gather sender.
 *   iov[dev, n]    : one entry per record; all zero lengths for a record
 *                    whose status != ONC_OK (except a declared AUTH_UNIX
 *                    record failing only its deferred block check: its
 *                    placeholder header and payload slice, as onc_encode
 *                    writes them, onc_auth).
 *   status[dev, n] : ONC_OK or ONC_ENC_*; a record whose header would end
 *                    beyond hdr_cap gets ONC_ENC_WRITE_ZERO and none of its
 *                    header bytes are written.
 *   totals[dev, 2] : optional: {header bytes, wire bytes} of the batch. */
typedef struct onc_iov_rec {
    uint64_t hdr_off;
    uint64_t payload_off;
    uint64_t wire_off;
    uint32_t hdr_len;
    uint32_t payload_len;
} onc_iov_rec;

int onc_encode_iov(onc_codec* codec, const onc_batch* batch,
                   uint8_t* hdr_out, uint64_t hdr_cap,
                   onc_iov_rec* iov, int32_t* status, uint64_t* totals);

/* Drop the extent of every record whose status != ONC_OK from a buffer
 * onc_encode wrote, in place: afterwards out[rec_off[i], rec_off[i+1]) is
 * record i for an OK record and empty for any other, the OK records back to
 * back from rec_off[0] (unchanged) on — the bytes the reference's loop of
 * serialise_into calls on one Cursor<Vec<u8>> writes for the same messages,
 * since a message that panics (unix_params.rs:47,149, flavor.rs:110) or
 * fails writes nothing. Only placeholders (a declared AUTH_UNIX credential
 * failing its deferred block check, onc_auth) have an extent to drop; every
 * other failing record already takes 0 bytes, so a batch without a
 * placeholder moves nothing. `status` is onc_encode's. Bytes from the new
 * rec_off[n] up to the old one are left as they were. *total (host,
 * optional) receives the new rec_off[n]. Synchronous: it sizes its scratch
 * by the moved bytes, which it reads back, and returns with the buffer and
 * rec_off final (ONC_RC_ECAPTURE inside a stream capture). For the rare
 * path: call it only after seeing a failing status. */
int onc_compact(onc_codec* codec, uint8_t* out, uint64_t* rec_off, const int32_t* status, uint64_t n,
                uint64_t* total);

/* The same for onc_encode_iov's list: every entry whose status != ONC_OK
 * gets hdr_len = payload_len = 0 and every wire_off is the kept bytes before
 * it (rec_off[0] = 0); hdr_off / payload_off are kept. totals[dev, 2]
 * (optional): {kept header bytes, kept wire bytes}. Asynchronous. */
int onc_compact_iov(onc_codec* codec, onc_iov_rec* iov, const int32_t* status, uint64_t n, uint64_t* totals);

/* ------------------------------------------------------------------------ */
/* Decode — RpcMessage::try_from(&[u8]) / try_from(Bytes)                    */
/* ------------------------------------------------------------------------ */

/* Decode record i = wire[rec_off[i] .. rec_off[i+1]) for i < n, each
 * exactly as the reference decodes one buffer that must hold exactly one
 * message (src/rpc_message.rs:238-242). mode = ONC_DECODE_SLICE | _BYTES.
 * Memory access: the decoder reads its records' header bytes as whole
 * 16-byte-aligned granules (one dwordx4 per granule), so it may read up to
 * 15 bytes before rec_off[i] / after rec_off[i+1] — never outside the
 * aligned 16-byte granules that hold record bytes, so never across a page
 * or allocation boundary of a hipMalloc'd buffer. Those bytes never affect
 * the result; no byte of the wire is written. */
int onc_decode(onc_codec* codec, const uint8_t* wire, const uint64_t* rec_off,
               uint64_t n, int mode, const onc_decoded* out);

/* expected_message_len (src/rpc_message.rs:343-367) of one host buffer: the
 * record-marking header's length + 4. Returns ONC_OK, or
 * ONC_ERR_INCOMPLETE_HEADER (len < 4) / ONC_ERR_FRAGMENTED (last-fragment
 * bit clear). Host memory, synchronous; the framing helper a caller uses to
 * cut one message out of a socket buffer. */
int32_t onc_expected_message_len(const uint8_t* data, uint64_t len, uint32_t* out);

/* Framing of a stream buffer of back-to-back record-marked messages (a
 * socket read buffer): the caller's loop of expected_message_len
 * (src/rpc_message.rs:343-367) + one-message slices
 * (rpc_message.rs:238-242), in parallel on the device with the same result.
 * From offset 0, records are framed while the remaining bytes hold a whole
 * record and fewer than max_records were framed.
 *   rec_off[dev, max_records + 1]: starts of the framed records, then the
 *                     end of the last one (= bytes consumed).
 *   result[dev, 5]  : {n, consumed, status, aux0, aux1}; status is ONC_OK when
 *                     the buffer ends on a record boundary or max_records
 *                     were framed, else why the next record cannot be cut:
 *                     ONC_ERR_INCOMPLETE_HEADER (< 4 bytes left),
 *                     ONC_ERR_FRAGMENTED (last-fragment bit clear) or
 *                     ONC_ERR_INCOMPLETE_MESSAGE {aux0 = bytes left,
 *                     aux1 = record length} (wait for more data).
 * The stream is cut into 64 KiB chunks framed speculatively in parallel and
 * verified (frame.hip); onc_codec_options.frame_chunk overrides the chunk
 * size (tests use small chunks to exercise the multi-chunk logic).
 * SURVEY §8(f) rank 1. */
int onc_frame_stream(onc_codec* codec, const uint8_t* wire, uint64_t len,
                     uint64_t* rec_off, uint64_t max_records, uint64_t* result);

/* Exclusive scan of record lengths into offsets:
 * rec_off[0] = base, rec_off[i+1] = rec_off[i] + rec_len[i]  ([dev]). */
int onc_scan_lengths(onc_codec* codec, const uint32_t* rec_len, uint64_t n,
                     uint64_t base, uint64_t* rec_off);

/* onc_scan_lengths + onc_decode in one pass: record i is
 * wire[off_i, off_i + rec_len[i]) with off_0 = base, off_(i+1) = off_i +
 * rec_len[i] (the caller's length-delimited slices, each decoded as by
 * TryFrom<&[u8]> / TryFrom<Bytes>, rpc_message.rs:235-314). The offsets are
 * computed inside the decode (no offsets pass over the batch); rec_off
 * (optional, n + 1 entries, [dev]) receives them. Same outputs, over-read
 * rule and errors as onc_decode. */
int onc_decode_lengths(onc_codec* codec, const uint8_t* wire, const uint32_t* rec_len, uint64_t n,
                       uint64_t base, int mode, uint64_t* rec_off, const onc_decoded* out);

/* ------------------------------------------------------------------------ */
/* Body-level roots (ONC_ROOT_*)                                             */
/* ------------------------------------------------------------------------ */

/* Decode record i = wire[rec_off[i] .. rec_off[i+1]) as `root`'s TryFrom
 * over exactly that slice (slice mode: a Cursor over it, so every opaque
 * bound is the record; Bytes mode: a Bytes of it). Unlike RpcMessage, a body
 * has no framing header and no trailing-bytes check (the reference's body
 * TryFrom impls return what they parsed and ignore the rest).
 *   param[dev, n]   : AUTH_UNIX_PARAMS slice mode: expected_len; OPAQUE:
 *                     max_len (both modes); required for those, else ignored
 *                     (may be NULL).
 *   out             : as onc_decode (descriptor shape per root above).
 *   consumed[dev, n]: optional: bytes the value occupies (the cursor's final
 *                     position = its serialised_len(); Call / Success
 *                     payloads extend to the record's end); 0 on error.
 * ONC_ROOT_RPC_MESSAGE is onc_decode (consumed = the record length on OK).
 * Same over-read rule as onc_decode. */
int onc_decode_body(onc_codec* codec, int root, const uint8_t* wire, const uint64_t* rec_off, uint64_t n,
                    int mode, const uint32_t* param, const onc_decoded* out, uint32_t* consumed);

/* serialised_len() of every descriptor as `root` + the checks of that
 * root's serialise_into: shape (ONC_ENC_BAD_DESCRIPTOR), construction panics
 * (NAME_GT_255, GIDS_GT_16), a body >= 2^31 bytes (ONC_ENC_TOO_LONG: the
 * RpcMessage limit, rpc_message.rs:146-151, applied to every root), and the
 * assoc > 200 assert (flavor.rs:110) for roots that serialise an AuthFlavor
 * (MESSAGE_TYPE, CALL_BODY, REPLY_BODY, ACCEPTED_REPLY, AUTH_FLAVOR).
 * Outputs as onc_encode_lengths. */
int onc_encode_body_lengths(onc_codec* codec, int root, const onc_batch* batch, uint32_t* rec_len,
                            int32_t* status);

/* Every descriptor serialised as `root` back to back into out — the batch
 * form of `root`::serialise_into on one Cursor<Vec<u8>>. Same outputs, writer
 * position and capacity rules as onc_encode. */
int onc_encode_body(onc_codec* codec, int root, const onc_batch* batch, uint8_t* out, uint64_t out_cap,
                    uint64_t* rec_off, int32_t* status, uint32_t* rec_len);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* ONC_RPC_H */
