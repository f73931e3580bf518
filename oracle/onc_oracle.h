/*
 * onc_oracle.h — CPU restatement of domodwyer/onc-rpc v0.3.3 (TEST INFRASTRUCTURE).
 *
 * THIS IS THE PARITY CHECKER, NOT THE PRODUCT. Only tests/, the smoke()
 * entry point and bench.py's cpu_baseline leg may load or call it. The
 * product path (onc-rpc_amd/, the HIP kernels behind include/onc_rpc.h)
 * never links it and has no CPU fallback.
 *
 * Parity is pinned: every hex golden vector of the reference's own unit
 * tests (tests/golden/vectors.json, citations inside) is checked against
 * this restatement by tests/test_oracle_golden.py. The reference itself
 * (Rust) cannot be built in this image (no cargo/rustc, no crates), so
 * there is no oracle/_ref build; see DESIGN.md §Oracle.
 *
 * Each function names the reference function it restates (file:line,
 * relative to the reference root). The restatement keeps the reference's
 * structure: a recursive-descent reader over a std::io::Cursor (slice
 * mode) or a bytes::Bytes view (Bytes mode) and a std::io::Write writer.
 */
#ifndef ONC_ORACLE_H
#define ONC_ORACLE_H

#include <stdint.h>
#include "../include/onc_rpc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Single message: decode buf[0..len) in `mode`. On success the descriptor
 * holds offsets relative to `base` (normally buf itself or the start of
 * the wire buffer buf was sliced from); unix[0]/unix[1] receive the cred /
 * verf params and onc_auth.ref = unix_slot_base + 0 / + 1.
 * Returns the status code (ONC_OK or ONC_ERR_*), aux as in onc_decoded. */
int32_t oracle_decode_message(const uint8_t* base, const uint8_t* buf, uint64_t len, int mode,
                              uint64_t unix_slot_base, onc_msg* msg, onc_unix_params unix[2],
                              uint32_t* aux0, uint32_t* aux1);

/* Single message: serialise the descriptor into out[0..cap).
 * *written = bytes written (== serialised len on success). Returns ONC_OK or
 * an ONC_ENC_* code. *serialised_len = RpcMessage::serialised_len(). */
int32_t oracle_encode_message(const onc_msg* msg, const onc_unix_params* unix_table,
                              const uint8_t* auth_arena, const uint8_t* payload_arena,
                              uint8_t* out, uint64_t cap, uint64_t* written,
                              uint64_t* serialised_len);

/* Batch forms: the caller's loop of the reference (one Cursor<Vec<u8>> for
 * encode; one slice per record for decode). Same layouts as onc_encode /
 * onc_decode, host memory. */
void oracle_encode_batch(uint64_t n, const onc_msg* msgs, const onc_unix_params* unix_table,
                         const uint8_t* auth_arena, const uint8_t* payload_arena,
                         uint8_t* out, uint64_t out_cap, uint64_t* rec_off,
                         int32_t* status, uint32_t* rec_len);
void oracle_decode_batch(const uint8_t* wire, const uint64_t* rec_off, uint64_t n, int mode,
                         onc_msg* msgs, onc_unix_params* unix_params, int32_t* status,
                         uint32_t* aux0, uint32_t* aux1);
/* Same as oracle_decode_batch over records [lo, hi) using `threads` pthreads
 * (CPU-baseline leg only). */
void oracle_decode_batch_mt(const uint8_t* wire, const uint64_t* rec_off, uint64_t n, int mode,
                            onc_msg* msgs, onc_unix_params* unix_params, int32_t* status,
                            uint32_t* aux0, uint32_t* aux1, int threads);

/* Multi-threaded encode (CPU-baseline leg only): per-record lengths on all
 * threads, exclusive scan, then each thread serialises its contiguous range.
 * `out` must hold the total (no capacity handling). */
void oracle_encode_batch_mt(uint64_t n, const onc_msg* msgs, const onc_unix_params* unix_table,
                            const uint8_t* auth_arena, const uint8_t* payload_arena, uint8_t* out,
                            uint64_t* rec_off, int32_t* status, uint32_t* rec_len, int threads);

/* The caller's expected_message_len loop over a stream buffer (framing). */
void oracle_frame_stream(const uint8_t* data, uint64_t len, uint64_t* rec_off, uint64_t max_records,
                         uint64_t* result);

/* The bytes a loop of serialise_into calls on one Cursor<Vec<u8>> leaves
 * when some messages fail (a failing message writes nothing): the extents of
 * records with status != OK dropped from an encoded buffer in place, rec_off
 * re-placed (onc_compact). Returns the new rec_off[n]. */
uint64_t oracle_compact(uint8_t* wire, uint64_t* rec_off, const int32_t* status, uint64_t n);

/* Component-level entry points used by the golden-vector tests. */
/* expected_message_len — src/rpc_message.rs:343-367 */
int32_t oracle_expected_message_len(const uint8_t* data, uint64_t len, uint32_t* out);
/* AuthFlavor::try_from(&[u8]) (flavor.rs:177-184) / try_from(Bytes) (:186-222):
 * offsets relative to buf; unix params into *unix. *consumed = cursor pos. */
int32_t oracle_auth_decode(const uint8_t* buf, uint64_t len, int mode, onc_auth* auth,
                           onc_unix_params* unix, uint64_t* consumed);
/* AuthFlavor::serialise_into (flavor.rs:106-129); serialised_len (:154-174);
 * associated_data_len (:142-150) */
int32_t oracle_auth_encode(const onc_auth* auth, const onc_unix_params* unix_table,
                           const uint8_t* arena, uint8_t* out, uint64_t cap, uint64_t* written);
uint32_t oracle_auth_serialised_len(const onc_auth* auth, const onc_unix_params* unix_table);
uint32_t oracle_auth_associated_data_len(const onc_auth* auth, const onc_unix_params* unix_table);
/* AuthUnixParams::from_cursor (unix_params.rs:90-129) over buf with the
 * given expected_len, and AuthUnixParams::try_from(Bytes) (:248-276). */
int32_t oracle_unix_params_decode(const uint8_t* buf, uint64_t len, int mode, uint32_t expected_len,
                                  onc_unix_params* out, uint64_t* consumed);
/* AuthUnixParams::serialise_into (unix_params.rs:162-176) */
int32_t oracle_unix_params_encode(const onc_unix_params* p, const uint8_t* arena, uint8_t* out,
                                  uint64_t cap, uint64_t* written);
/* Opaque::from_wire (opaque.rs:72-98) and Opaque::serialise_into (:38-56) */
int32_t oracle_opaque_from_wire(const uint8_t* buf, uint64_t len, uint64_t max_len,
                                uint64_t* body_off, uint64_t* body_len, uint64_t* consumed);
int32_t oracle_opaque_encode(const uint8_t* body, uint32_t len, uint8_t* out, uint64_t cap,
                             uint64_t* written);
/* pad_length (opaque.rs:115-121) */
uint32_t oracle_pad_length(uint32_t l);

/* Body-level roots (ONC_ROOT_*, include/onc_rpc.h): `root`'s own TryFrom over
 * buf[0..len) (slice / Bytes), the descriptor shape of include/onc_rpc.h;
 * *consumed = the decoded value's serialised_len(). param = expected_len
 * (AUTH_UNIX_PARAMS, slice) / max_len (OPAQUE). */
int32_t oracle_decode_body(int root, const uint8_t* base, const uint8_t* buf, uint64_t len, int mode,
                           uint32_t param, uint64_t unix_slot_base, onc_msg* msg, onc_unix_params unix[2],
                           uint32_t* aux0, uint32_t* aux1, uint32_t* consumed);
/* `root`::serialise_into of a descriptor, with onc_encode_body_lengths' checks. */
int32_t oracle_encode_body(int root, const onc_msg* msg, const onc_unix_params* unix_table,
                           const uint8_t* auth_arena, const uint8_t* payload_arena, uint8_t* out, uint64_t cap,
                           uint64_t* written, uint64_t* serialised_len);
/* Batch forms (the caller's loop), layouts as onc_encode_body / onc_decode_body. */
void oracle_encode_body_batch(int root, uint64_t n, const onc_msg* msgs, const onc_unix_params* unix_table,
                              const uint8_t* auth_arena, const uint8_t* payload_arena, uint8_t* out,
                              uint64_t out_cap, uint64_t* rec_off, int32_t* status, uint32_t* rec_len);
void oracle_decode_body_batch(int root, const uint8_t* wire, const uint64_t* rec_off, uint64_t n, int mode,
                              const uint32_t* param, onc_msg* msgs, onc_unix_params* unix_params, int32_t* status,
                              uint32_t* aux0, uint32_t* aux1, uint32_t* consumed);

#ifdef __cplusplus
}
#endif

#endif
