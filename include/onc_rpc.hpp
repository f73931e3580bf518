// onc_rpc.hpp — C++ mirror of the reference crate's types over the C ABI.
//
// The reference (domodwyer/onc-rpc v0.3.3) is a Rust crate; the Rust
// toolchain is not in this image, so its public surface for the hot path is
// restated here in C++17 with the same names, argument meanings and error
// behaviour (see INTEGRATION.md for the Rust extern "C" binding):
//
//   RpcMessage      src/rpc_message.rs:97-233     new, xid, message, call_body,
//                                                 reply_body, serialised_len,
//                                                 serialise_into, serialise,
//                                                 try_from (slice / Bytes mode)
//   MessageType     src/rpc_message.rs:22-93      Call | Reply
//   CallBody        src/call_body.rs:17-166       new, rpc_version, program, ...
//   AuthFlavor      src/auth/flavor.rs:18-174     AuthNone(Option<T>) | AuthUnix |
//                                                 AuthShort | Unknown{id, data}
//   AuthUnixParams  src/auth/unix_params.rs:72-245
//   ReplyBody / AcceptedReply / AcceptedStatus / RejectedReply / AuthError
//                   src/reply/*.rs
//   Error           src/errors.rs:6-97            (thrown as onc_rpc::Error)
//   expected_message_len  src/rpc_message.rs:343-367
//
// Values are generic over byte storage in the reference (`T, P:
// AsRef<[u8]>`); here they hold non-owning `Bytes` views (pointer + length),
// exactly like the reference's `&'a [u8]` instantiation: decoded messages
// borrow the caller's wire buffer, encoded messages borrow the caller's
// payload and auth bodies.
//
// All codec work runs on the GPU through libonc_rpc_amd.so:
//   BatchEncoder  — the caller's serialise_into loop over many messages,
//                   one onc_encode_body call (one pass, no length pass).
//   BatchDecoder  — the caller's try_from loop over many records, one
//                   onc_decode_lengths call.
//   Both stage their inputs and outputs in the codec's mapped pinned host
//   memory (Codec::stage): the kernels read and write it in place over PCIe
//   — no device allocation and no copy calls, one synchronisation per call.
//   RpcMessage::serialise_into / serialised_len / try_from — single-message
//                   forms, implemented as batches of one (for API parity;
//                   use the batch classes for throughput).
// There is no CPU codec in this header: the value classes only describe
// messages; lengths, bytes and parse results always come from the kernels.
// The reference's panics (auth data > 200 bytes, machine name > 255 bytes,
// more than 16 gids) are thrown as std::logic_error where the reference
// panics (constructors) and reported as ONC_ENC_* statuses by the batch
// encoder.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <utility>
#include <variant>
#include <vector>

#include "onc_rpc.h"

namespace onc_rpc {

// ----------------------------------------------------------------------------
// Bytes: a borrowed byte slice (&[u8])
// ----------------------------------------------------------------------------
struct Bytes {
    const uint8_t* ptr = nullptr;
    size_t len = 0;
    Bytes() = default;
    Bytes(const uint8_t* p, size_t n) : ptr(p), len(n) {}
    Bytes(const std::vector<uint8_t>& v) : ptr(v.data()), len(v.size()) {}  // NOLINT
    const uint8_t* data() const { return ptr; }
    size_t size() const { return len; }
    bool empty() const { return len == 0; }
    std::vector<uint8_t> to_vec() const { return std::vector<uint8_t>(ptr, ptr + len); }
    bool operator==(const Bytes& o) const { return len == o.len && (len == 0 || std::memcmp(ptr, o.ptr, len) == 0); }
    bool operator!=(const Bytes& o) const { return !(*this == o); }
};

// ----------------------------------------------------------------------------
// Error — src/errors.rs:6-97 (Display strings follow the #[error] attributes)
// ----------------------------------------------------------------------------
class Error : public std::exception {
public:
    Error(int32_t code, uint32_t aux0 = 0, uint32_t aux1 = 0) : code_(code), aux0_(aux0), aux1_(aux1) {
        msg_ = describe(code, aux0, aux1);
    }
    int32_t code() const { return code_; }
    // IncompleteMessage{buffer_len, expected}; the offending value for the
    // Invalid*(u32) variants.
    uint32_t buffer_len() const { return aux0_; }
    uint32_t expected() const { return aux1_; }
    uint32_t value() const { return aux0_; }
    const char* what() const noexcept override { return msg_.c_str(); }
    bool operator==(const Error& o) const { return code_ == o.code_ && aux0_ == o.aux0_ && aux1_ == o.aux1_; }

    static std::string describe(int32_t code, uint32_t a0, uint32_t a1) {
        switch (code) {
            case ONC_ERR_INCOMPLETE_MESSAGE:
                return "incomplete rpc message (got " + std::to_string(a0) + " bytes, expected " +
                       std::to_string(a1) + ")";
            case ONC_ERR_INCOMPLETE_HEADER: return "incomplete fragment header";
            case ONC_ERR_FRAGMENTED: return "RPC message is fragmented";
            case ONC_ERR_INVALID_MESSAGE_TYPE: return "invalid rpc message type " + std::to_string(a0);
            case ONC_ERR_INVALID_REPLY_TYPE: return "invalid rpc reply type " + std::to_string(a0);
            case ONC_ERR_INVALID_REPLY_STATUS: return "invalid rpc reply status " + std::to_string(a0);
            case ONC_ERR_INVALID_AUTH_DATA: return "invalid rpc auth data";
            case ONC_ERR_INVALID_AUTH_ERROR: return "invalid rpc auth error status " + std::to_string(a0);
            case ONC_ERR_INVALID_REJECTED_REPLY_TYPE:
                return "invalid rpc rejected reply type " + std::to_string(a0);
            case ONC_ERR_INVALID_LENGTH: return "invalid length in rpc message";
            case ONC_ERR_INVALID_RPC_VERSION: return "invalid rpc version " + std::to_string(a0);
            case ONC_ERR_INVALID_MACHINE_NAME: return "invalid machine name";
            case ONC_ERR_IO_UNEXPECTED_EOF: return "i/o error (UnexpectedEof): failed to fill whole buffer";
            default: {
                const char* s = onc_status_str(code);
                return s ? std::string(s) : "error " + std::to_string(code);
            }
        }
    }

private:
    int32_t code_;
    uint32_t aux0_, aux1_;
    std::string msg_;
};

// Device/runtime failure (not a reference error): HIP error or bad argument.
class CodecError : public std::runtime_error {
public:
    using std::runtime_error::runtime_error;
};

enum class DecodeMode { Slice = ONC_DECODE_SLICE, Bytes = ONC_DECODE_BYTES };
class Codec;

// ----------------------------------------------------------------------------
// AuthUnixParams — src/auth/unix_params.rs:72-245
// ----------------------------------------------------------------------------
class AuthUnixParams {
public:
    // AuthUnixParams::from_cursor(r, expected_len) over `buf` (slice rules,
    // unix_params.rs:90-129) and TryFrom<Bytes> (:248-276); serialise_into
    // (:162-176) / serialised_len (:219-230). Body-level decode/encode on the
    // GPU (onc_decode_body / onc_encode_body, ONC_ROOT_AUTH_UNIX_PARAMS).
    static AuthUnixParams from_cursor(Codec& codec, Bytes buf, uint32_t expected_len);
    static AuthUnixParams try_from(Codec& codec, Bytes buf);
    void serialise_into(Codec& codec, std::vector<uint8_t>& buf) const;
    uint32_t serialised_len(Codec& codec) const;

    // AuthUnixParams::new (unix_params.rs:142-158): panics on a machine name
    // longer than 255 bytes (:149) or more than 16 gids (Gids, :47).
    AuthUnixParams(uint32_t stamp, Bytes machine_name, uint32_t uid, uint32_t gid, std::vector<uint32_t> gids)
        : stamp_(stamp), machine_name_(machine_name), uid_(uid), gid_(gid), gids_(std::move(gids)) {
        if (machine_name.len > ONC_MAX_MACHINE_NAME_LEN) throw std::logic_error("machine name longer than 255 bytes");
        if (gids_.size() > ONC_MAX_GIDS) throw std::logic_error("more than 16 gids");
    }
    uint32_t stamp() const { return stamp_; }
    Bytes machine_name() const { return machine_name_; }
    std::string machine_name_str() const {
        return std::string(reinterpret_cast<const char*>(machine_name_.ptr), machine_name_.len);
    }
    uint32_t uid() const { return uid_; }
    uint32_t gid() const { return gid_; }
    // None (nullopt) when there are no gids (unix_params.rs:210-216).
    std::optional<std::vector<uint32_t>> gids() const {
        if (gids_.empty()) return std::nullopt;
        return gids_;
    }
    const std::vector<uint32_t>& gids_vec() const { return gids_; }
    bool operator==(const AuthUnixParams& o) const {
        return stamp_ == o.stamp_ && machine_name_ == o.machine_name_ && uid_ == o.uid_ && gid_ == o.gid_ &&
               gids_ == o.gids_;
    }

private:
    uint32_t stamp_;
    Bytes machine_name_;
    uint32_t uid_, gid_;
    std::vector<uint32_t> gids_;
};

// ----------------------------------------------------------------------------
// AuthFlavor — src/auth/flavor.rs:18-174
// ----------------------------------------------------------------------------
class AuthFlavor {
public:
    enum class Kind { AuthNone, AuthUnix, AuthShort, Unknown };

    static AuthFlavor none(std::optional<Bytes> data = std::nullopt) {
        AuthFlavor a(Kind::AuthNone);
        a.data_ = data;
        return a;
    }
    static AuthFlavor unix(AuthUnixParams p) {
        AuthFlavor a(Kind::AuthUnix);
        a.unix_ = std::move(p);
        return a;
    }
    static AuthFlavor short_(Bytes data) {
        AuthFlavor a(Kind::AuthShort);
        a.data_ = data;
        return a;
    }
    static AuthFlavor unknown(uint32_t id, Bytes data) {
        AuthFlavor a(Kind::Unknown);
        a.id_ = id;
        a.data_ = data;
        return a;
    }

    Kind kind() const { return kind_; }
    // TryFrom<&[u8]> (flavor.rs:177-184) / TryFrom<Bytes> (:186-222);
    // serialise_into (:106-129) / serialised_len (:154-174) — on the GPU.
    static AuthFlavor try_from(Codec& codec, Bytes buf, DecodeMode mode = DecodeMode::Slice);
    void serialise_into(Codec& codec, std::vector<uint8_t>& buf) const;
    uint32_t serialised_len(Codec& codec) const;
    // associated_data_len (flavor.rs:142-150; unix_params.rs:234-245): the
    // body bytes without prefixes or padding (the value the 200-byte assert
    // of serialise_into checks).
    uint32_t associated_data_len() const {
        if (kind_ == Kind::AuthUnix)
            return uint32_t(12 + unix_->machine_name().len + 4 * unix_->gids_vec().size());
        return data_ ? uint32_t(data_->len) : 0u;
    }
    // Wire discriminant (flavor.rs:132-139).
    uint32_t id() const {
        switch (kind_) {
            case Kind::AuthNone: return ONC_AUTH_NONE;
            case Kind::AuthUnix: return ONC_AUTH_UNIX;
            case Kind::AuthShort: return ONC_AUTH_SHORT;
            default: return id_;
        }
    }
    // AuthNone's optional body / AuthShort / Unknown data.
    std::optional<Bytes> data() const { return data_; }
    const AuthUnixParams& unix_params() const {
        if (!unix_) throw std::logic_error("not AuthUnix");
        return *unix_;
    }
    bool operator==(const AuthFlavor& o) const {
        if (kind_ != o.kind_ || id() != o.id()) return false;
        if (kind_ == Kind::AuthUnix) return *unix_ == *o.unix_;
        if (data_.has_value() != o.data_.has_value()) return false;
        return !data_ || *data_ == *o.data_;
    }

private:
    explicit AuthFlavor(Kind k) : kind_(k) {}
    Kind kind_;
    uint32_t id_ = 0;
    std::optional<Bytes> data_;
    std::optional<AuthUnixParams> unix_;
};

// ----------------------------------------------------------------------------
// CallBody — src/call_body.rs:17-166
// ----------------------------------------------------------------------------
class CallBody {
public:
    CallBody(uint32_t program, uint32_t program_version, uint32_t procedure, AuthFlavor auth_credentials,
             AuthFlavor auth_verifier, Bytes payload)
        : program_(program), program_version_(program_version), procedure_(procedure),
          cred_(std::move(auth_credentials)), verf_(std::move(auth_verifier)), payload_(payload) {}
    uint32_t rpc_version() const { return 2; }   // RPC_VERSION call_body.rs:10
    // TryFrom<&[u8]> (call_body.rs:168-175) / TryFrom<Bytes> (:177-210);
    // serialise_into (:98-108) / serialised_len (:111-119) — on the GPU.
    static CallBody try_from(Codec& codec, Bytes buf, DecodeMode mode = DecodeMode::Slice);
    void serialise_into(Codec& codec, std::vector<uint8_t>& buf) const;
    uint32_t serialised_len(Codec& codec) const;
    uint32_t program() const { return program_; }
    uint32_t program_version() const { return program_version_; }
    uint32_t procedure() const { return procedure_; }
    const AuthFlavor& auth_credentials() const { return cred_; }
    const AuthFlavor& auth_verifier() const { return verf_; }
    Bytes payload() const { return payload_; }
    bool operator==(const CallBody& o) const {
        return program_ == o.program_ && program_version_ == o.program_version_ && procedure_ == o.procedure_ &&
               cred_ == o.cred_ && verf_ == o.verf_ && payload_ == o.payload_;
    }

private:
    uint32_t program_, program_version_, procedure_;
    AuthFlavor cred_, verf_;
    Bytes payload_;
};

// ----------------------------------------------------------------------------
// Replies — src/reply/*.rs
// ----------------------------------------------------------------------------
enum class AuthError : uint32_t {   // rejected_reply.rs:130-173
    Success = 0,
    BadCredentials = 1,
    RejectedCredentials = 2,
    BadVerifier = 3,
    RejectedVerifier = 4,
    TooWeak = 5,
    InvalidResponseVerifier = 6,
    Failed = 7,
};

class RejectedReply {   // rejected_reply.rs:24-95
public:
    enum class Kind { RpcVersionMismatch, AuthError };
    static RejectedReply rpc_version_mismatch(uint32_t low, uint32_t high) {
        RejectedReply r(Kind::RpcVersionMismatch);
        r.low_ = low;
        r.high_ = high;
        return r;
    }
    static RejectedReply auth_error(AuthError e) {
        RejectedReply r(Kind::AuthError);
        r.err_ = e;
        return r;
    }
    Kind kind() const { return kind_; }
    std::pair<uint32_t, uint32_t> mismatch() const { return {low_, high_}; }
    AuthError auth_error() const { return err_; }
    // TryFrom<&[u8]> (rejected_reply.rs:98-105) / TryFrom<Bytes> (:107-125);
    // serialise_into (:61-73) / serialised_len (:76-95) — on the GPU.
    static RejectedReply try_from(Codec& codec, Bytes buf, DecodeMode mode = DecodeMode::Slice);
    void serialise_into(Codec& codec, std::vector<uint8_t>& buf) const;
    uint32_t serialised_len(Codec& codec) const;
    bool operator==(const RejectedReply& o) const {
        return kind_ == o.kind_ && (kind_ == Kind::AuthError ? err_ == o.err_ : (low_ == o.low_ && high_ == o.high_));
    }

private:
    explicit RejectedReply(Kind k) : kind_(k) {}
    Kind kind_;
    uint32_t low_ = 0, high_ = 0;
    AuthError err_ = AuthError::Success;
};

class AcceptedStatus {   // accepted_reply.rs:109-231
public:
    enum class Kind { Success, ProgramUnavailable, ProgramMismatch, ProcedureUnavailable, GarbageArgs, SystemError };
    static AcceptedStatus success(Bytes payload) {
        AcceptedStatus s(Kind::Success);
        s.payload_ = payload;
        return s;
    }
    static AcceptedStatus program_mismatch(uint32_t low, uint32_t high) {
        AcceptedStatus s(Kind::ProgramMismatch);
        s.low_ = low;
        s.high_ = high;
        return s;
    }
    static AcceptedStatus of(Kind k) { return AcceptedStatus(k); }
    Kind kind() const { return kind_; }
    // TryFrom<&[u8]> (accepted_reply.rs:234-241) / TryFrom<Bytes> (:243-265);
    // serialise_into (:195-211) / serialised_len (:214-231) — on the GPU.
    static AcceptedStatus try_from(Codec& codec, Bytes buf, DecodeMode mode = DecodeMode::Slice);
    void serialise_into(Codec& codec, std::vector<uint8_t>& buf) const;
    uint32_t serialised_len(Codec& codec) const;
    Bytes payload() const { return payload_; }
    std::pair<uint32_t, uint32_t> mismatch() const { return {low_, high_}; }
    bool operator==(const AcceptedStatus& o) const {
        if (kind_ != o.kind_) return false;
        if (kind_ == Kind::Success) return payload_ == o.payload_;
        if (kind_ == Kind::ProgramMismatch) return low_ == o.low_ && high_ == o.high_;
        return true;
    }

private:
    explicit AcceptedStatus(Kind k) : kind_(k) {}
    Kind kind_;
    Bytes payload_;
    uint32_t low_ = 0, high_ = 0;
};

class AcceptedReply {   // accepted_reply.rs:20-77
public:
    AcceptedReply(AuthFlavor auth_verifier, AcceptedStatus status)
        : verf_(std::move(auth_verifier)), status_(std::move(status)) {}
    const AuthFlavor& auth_verifier() const { return verf_; }
    const AcceptedStatus& status() const { return status_; }
    // TryFrom<&[u8]> (accepted_reply.rs:79-86) / TryFrom<Bytes> (:88-105);
    // serialise_into (:58-61) / serialised_len (:64-66) — on the GPU.
    static AcceptedReply try_from(Codec& codec, Bytes buf, DecodeMode mode = DecodeMode::Slice);
    void serialise_into(Codec& codec, std::vector<uint8_t>& buf) const;
    uint32_t serialised_len(Codec& codec) const;
    bool operator==(const AcceptedReply& o) const { return verf_ == o.verf_ && status_ == o.status_; }

private:
    AuthFlavor verf_;
    AcceptedStatus status_;
};

class ReplyBody {   // reply_body.rs:16-73
public:
    static ReplyBody accepted(AcceptedReply r) { return ReplyBody(std::move(r)); }
    static ReplyBody denied(RejectedReply r) { return ReplyBody(std::move(r)); }
    bool is_accepted() const { return std::holds_alternative<AcceptedReply>(v_); }
    const AcceptedReply* accepted() const { return std::get_if<AcceptedReply>(&v_); }
    const RejectedReply* denied() const { return std::get_if<RejectedReply>(&v_); }
    bool operator==(const ReplyBody& o) const { return v_ == o.v_; }
    // TryFrom<&[u8]> (reply_body.rs:76-83) / TryFrom<Bytes> (:85-98);
    // serialise_into (:45-56) / serialised_len (:60-73) — on the GPU.
    static ReplyBody try_from(Codec& codec, Bytes buf, DecodeMode mode = DecodeMode::Slice);
    void serialise_into(Codec& codec, std::vector<uint8_t>& buf) const;
    uint32_t serialised_len(Codec& codec) const;

private:
    explicit ReplyBody(AcceptedReply r) : v_(std::move(r)) {}
    explicit ReplyBody(RejectedReply r) : v_(std::move(r)) {}
    std::variant<AcceptedReply, RejectedReply> v_;
};

// MessageType — rpc_message.rs:22-32
class MessageType {
public:
    static MessageType call(CallBody c) { return MessageType(std::move(c)); }
    static MessageType reply(ReplyBody r) { return MessageType(std::move(r)); }
    const CallBody* call_body() const { return std::get_if<CallBody>(&v_); }
    const ReplyBody* reply_body() const { return std::get_if<ReplyBody>(&v_); }
    bool operator==(const MessageType& o) const { return v_ == o.v_; }
    // from_cursor (rpc_message.rs:39-45) / TryFrom<Bytes> (:80-93);
    // serialise_into (:55-68) / serialised_len (:72-77) — on the GPU.
    static MessageType try_from(Codec& codec, Bytes buf, DecodeMode mode = DecodeMode::Slice);
    void serialise_into(Codec& codec, std::vector<uint8_t>& buf) const;
    uint32_t serialised_len(Codec& codec) const;

private:
    explicit MessageType(CallBody c) : v_(std::move(c)) {}
    explicit MessageType(ReplyBody r) : v_(std::move(r)) {}
    std::variant<CallBody, ReplyBody> v_;
};

// AuthError::from_cursor (rejected_reply.rs:176-190) / TryFrom<Bytes>
// (:215-236); serialise_into (:194-207) — on the GPU.
AuthError auth_error_try_from(Codec& codec, Bytes buf, DecodeMode mode = DecodeMode::Slice);
void serialise_into(Codec& codec, AuthError e, std::vector<uint8_t>& buf);

// ----------------------------------------------------------------------------
// Codec: one onc_codec handle (device + stream + scan scratch)
// ----------------------------------------------------------------------------
class Codec {
public:
    explicit Codec(int device = 0, hipStream_t stream = nullptr) {
        if (onc_codec_create(&h_, device, stream) != ONC_RC_OK) throw CodecError("onc_codec_create failed");
    }
    ~Codec() {
        if (h_) {
            (void)onc_codec_sync(h_);
            onc_codec_destroy(h_);
        }
        if (stage_host_) (void)hipHostFree(stage_host_);
    }
    Codec(const Codec&) = delete;
    Codec& operator=(const Codec&) = delete;
    onc_codec* get() const { return h_; }
    void check(int rc, const char* what) const {
        if (rc != ONC_RC_OK) throw CodecError(std::string(what) + ": " + onc_codec_last_error(h_));
    }
    void sync() const { check(onc_codec_sync(h_), "onc_codec_sync"); }

    // The mirror's staging area: mapped pinned host memory (hipHostMalloc,
    // hipHostMallocMapped). Every BatchEncoder / BatchDecoder call (and so
    // every single-message form) puts its inputs there and points the
    // kernels' outputs there, so the kernels read and write it in place over
    // PCIe (include/onc_rpc.h ABI 7: a [dev] pointer may be mapped host
    // memory) — no device allocation, no copy calls, one stream
    // synchronisation per call. `host` and `dev` address the same bytes;
    // valid until the next stage() call on this codec (every mirror call
    // synchronises before it returns). A stage that grows keeps its first
    // `keep` bytes (they move with it: re-derive pointers from offsets).
    struct Stage {
        uint8_t* host;
        uint8_t* dev;
    };
    size_t stage_capacity() const { return stage_cap_; }
    Stage stage(size_t n, size_t keep = 0) {
        if (n > stage_cap_) {
            size_t want = stage_cap_ ? stage_cap_ : (size_t(1) << 20);
            while (want < n) want *= 2;
            void* h = nullptr;
            if (hipHostMalloc(&h, want, hipHostMallocMapped) != hipSuccess) throw CodecError("hipHostMalloc(stage)");
            if (stage_host_) {
                sync();
                if (keep) std::memcpy(h, stage_host_, std::min(keep, stage_cap_));
                (void)hipHostFree(stage_host_);
                stage_host_ = stage_dev_ = nullptr;
                stage_cap_ = 0;
            }
            void* d = nullptr;
            if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
                (void)hipHostFree(h);
                throw CodecError("hipHostGetDevicePointer(stage)");
            }
            stage_host_ = static_cast<uint8_t*>(h);
            stage_dev_ = static_cast<uint8_t*>(d);
            stage_cap_ = want;
        }
        return Stage{stage_host_, stage_dev_};
    }

private:
    onc_codec* h_ = nullptr;
    uint8_t* stage_host_ = nullptr;
    uint8_t* stage_dev_ = nullptr;
    size_t stage_cap_ = 0;
};

namespace detail {

inline void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw CodecError(std::string(what) + ": " + hipGetErrorString(e));
}

// Typed regions of a staging area (256-byte aligned): sized first with
// need(), then taken in the same order from the codec's stage.
inline size_t rounded(size_t b) { return (b + 255) & ~size_t(255); }
template <class T>
struct Region {
    T* host;
    T* dev;
};
struct Carve {
    Codec::Stage s;
    size_t off = 0;
    template <class T>
    Region<T> take(size_t count) {
        const size_t a = off;
        off += rounded(count * sizeof(T) + 16);
        return Region<T>{reinterpret_cast<T*>(s.host + a), reinterpret_cast<T*>(s.dev + a)};
    }
};
template <class T>
inline size_t need(size_t count) { return rounded(count * sizeof(T) + 16); }

}  // namespace detail

// ----------------------------------------------------------------------------
// RpcMessage — src/rpc_message.rs:97-233
// ----------------------------------------------------------------------------
class RpcMessage {
public:
    RpcMessage(uint32_t xid, MessageType message) : xid_(xid), message_(std::move(message)) {}
    uint32_t xid() const { return xid_; }
    const MessageType& message() const { return message_; }
    const CallBody* call_body() const { return message_.call_body(); }
    const ReplyBody* reply_body() const { return message_.reply_body(); }
    bool operator==(const RpcMessage& o) const { return xid_ == o.xid_ && message_ == o.message_; }

    // Single-message calls: each is a whole GPU round trip (the message
    // staged in mapped host memory, the kernels reading and writing it in
    // place, a stream synchronisation) — tens of microseconds where the
    // reference's CPU call takes ~100 ns (tests/cpp/test_mirror.cpp
    // test_single_message_cost prints both). They exist for tests and tiny
    // batches; a caller with many messages uses BatchEncoder / BatchDecoder
    // (one launch per batch). The same holds for every body type's
    // serialised_len / serialise_into / try_from taking a Codec.
    //
    // serialised_len (rpc_message.rs:201-204), computed by the encoder's
    // length kernel. Throws std::logic_error where the reference panics.
    uint32_t serialised_len(Codec& codec) const;
    // serialise_into (rpc_message.rs:136-164): appends the record to `buf`.
    void serialise_into(Codec& codec, std::vector<uint8_t>& buf) const;
    // serialise (rpc_message.rs:193-197)
    std::vector<uint8_t> serialise(Codec& codec) const;
    // TryFrom<&[u8]> (rpc_message.rs:235-271) / TryFrom<Bytes> (:273-314):
    // `buf` must hold exactly one message; the result borrows `buf`.
    static RpcMessage try_from(Codec& codec, Bytes buf, DecodeMode mode = DecodeMode::Slice);

    // Encode statuses -> the reference's behaviour: panics for the
    // construction/assert failures, io::Error for TooLong/WriteZero.
    static void raise_encode_status(int32_t st) {
        switch (st) {
            case ONC_OK: return;
            case ONC_ENC_AUTH_GT_200: throw std::logic_error("auth associated data longer than 200 bytes");
            case ONC_ENC_NAME_GT_255: throw std::logic_error("machine name longer than 255 bytes");
            case ONC_ENC_GIDS_GT_16: throw std::logic_error("more than 16 gids");
            case ONC_ENC_BAD_DESCRIPTOR: throw std::logic_error("invalid message descriptor");
            case ONC_ENC_TOO_LONG: throw std::runtime_error("message length exceeds maximum");
            case ONC_ENC_WRITE_ZERO: throw std::runtime_error("failed to write whole buffer");
            default: throw std::runtime_error(onc_status_str(st));
        }
    }

private:
    uint32_t xid_;
    MessageType message_;
};

// ----------------------------------------------------------------------------
// BatchEncoder: serialise_into of many messages into one send buffer
// ----------------------------------------------------------------------------
class BatchEncoder {
public:
    // Describe one message (copies its borrowed bytes into the host arenas).
    void push(const RpcMessage& m);
    // Body-level values (ONC_ROOT_*): a batch holds values of one type and
    // is serialised as that type (onc_encode_body); mixing throws.
    void push(const MessageType& m);
    void push(const CallBody& c);
    void push(const ReplyBody& r);
    void push(const AcceptedReply& r);
    void push(const AcceptedStatus& s);
    void push(const RejectedReply& r);
    void push(AuthError e);
    void push(const AuthFlavor& a);
    void push(const AuthUnixParams& p);
    int root() const { return root_ < 0 ? ONC_ROOT_RPC_MESSAGE : root_; }
    size_t size() const { return msgs_.size(); }
    void clear() {
        msgs_.clear();
        unix_.clear();
        auth_.clear();
        payload_.clear();
        root_ = -1;
    }

    // Encode every pushed message back to back and APPEND the bytes to `out`
    // (the reference's serialise_into on a Cursor<Vec<u8>> positioned at the
    // end). Returns one status per message (ONC_OK or ONC_ENC_*; failing
    // messages occupy 0 bytes). rec_off, if given, receives n+1 offsets
    // relative to the start of the appended region.
    std::vector<int32_t> serialise_into(Codec& codec, std::vector<uint8_t>& out,
                                        std::vector<uint64_t>* rec_off = nullptr);
    // serialised_len() of every pushed message (0 for failing ones).
    std::vector<uint32_t> serialised_lens(Codec& codec, std::vector<int32_t>* status = nullptr);

private:
    // the batch's descriptors, AUTH_UNIX table and arenas copied into the
    // codec's mapped staging (the kernels read them there in place)
    size_t staged_bytes() const;
    onc_batch stage_batch(detail::Carve& c) const;
    void put_auth(const AuthFlavor& a, onc_auth& d);
    void put_payload(Bytes p, onc_msg& d);
    void put_call(const CallBody& c, onc_msg& d);
    void put_accepted(const AcceptedReply& a, onc_msg& d);
    void put_status(const AcceptedStatus& s, onc_msg& d);
    void put_rejected(const RejectedReply& r, onc_msg& d);
    void put_reply(const ReplyBody& r, onc_msg& d);
    void set_root(int root);

    int root_ = -1;

    std::vector<onc_msg> msgs_;
    std::vector<onc_unix_params> unix_;
    std::vector<uint8_t> auth_, payload_;
};

// Result of decoding one record (Result<RpcMessage<&[u8], &[u8]>, Error>).
struct Decoded {
    int32_t status = ONC_OK;
    uint32_t aux0 = 0, aux1 = 0;
    std::optional<RpcMessage> message;   // set iff status == ONC_OK
    bool ok() const { return status == ONC_OK; }
    Error error() const { return Error(status, aux0, aux1); }
};

// ----------------------------------------------------------------------------
// HostRegistration: a caller's receive buffer mapped for the kernels
// (onc_host_register, ABI 7). BatchDecoder given one decodes the bytes where
// they lie — no copy into the stage; only the 16-byte granules of the headers
// it parses cross PCIe (call_body.rs:53-59: payloads are slices, never read).
// Registration pins the pages (a server maps its socket buffers once);
// unpinned on destruction, so it must outlive the decodes using it.
// ----------------------------------------------------------------------------
class HostRegistration {
public:
    HostRegistration(Codec& codec, const uint8_t* buf, size_t len) : codec_(codec), host_(buf), len_(len) {
        void* d = nullptr;
        codec.check(onc_host_register(codec.get(), const_cast<uint8_t*>(buf), len ? len : 1, &d),
                    "onc_host_register");
        dev_ = static_cast<const uint8_t*>(d);
    }
    ~HostRegistration() { (void)onc_host_unregister(codec_.get(), const_cast<uint8_t*>(host_)); }
    HostRegistration(const HostRegistration&) = delete;
    HostRegistration& operator=(const HostRegistration&) = delete;
    const uint8_t* host() const { return host_; }
    const uint8_t* dev() const { return dev_; }
    size_t size() const { return len_; }

private:
    Codec& codec_;
    const uint8_t* host_;
    const uint8_t* dev_ = nullptr;
    size_t len_;
};

// ----------------------------------------------------------------------------
// BatchDecoder: try_from of many records (one buffer per record)
// ----------------------------------------------------------------------------
class BatchDecoder {
public:
    // Decode records wire[off_i, off_i + rec_len[i]) back to back (host
    // buffer). Decoded messages borrow `wire` (zero-copy, like the
    // reference's &[u8] instantiation), so it must outlive the results.
    std::vector<Decoded> try_from(Codec& codec, const uint8_t* wire, size_t wire_len,
                                  const std::vector<uint32_t>& rec_len, DecodeMode mode = DecodeMode::Slice);

    // A socket read buffer of back-to-back records: frame it on the device
    // (the caller's expected_message_len loop, rpc_message.rs:343-367), then
    // decode every complete record. `consumed` receives the bytes used;
    // `stop` why framing stopped before the end (nullopt when the buffer
    // ended on a record boundary): an incomplete trailing record means
    // "read more", as with the reference.
    std::vector<Decoded> try_from_stream(Codec& codec, const uint8_t* wire, size_t wire_len,
                                         DecodeMode mode = DecodeMode::Slice, size_t* consumed = nullptr,
                                         std::optional<Error>* stop = nullptr);

    // The same over a registered (mapped) buffer, decoded in place.
    std::vector<Decoded> try_from(Codec& codec, const HostRegistration& wire, const std::vector<uint32_t>& rec_len,
                                  DecodeMode mode = DecodeMode::Slice) {
        return lengths_at(codec, wire.host(), wire.dev(), wire.size(), rec_len, mode);
    }
    std::vector<Decoded> try_from_stream(Codec& codec, const HostRegistration& wire,
                                         DecodeMode mode = DecodeMode::Slice, size_t* consumed = nullptr,
                                         std::optional<Error>* stop = nullptr) {
        return stream_at(codec, wire.host(), wire.dev(), wire.size(), mode, consumed, stop);
    }

private:
    // dev_wire: the kernels' address of `wire` (a registration), or null:
    // the wire is copied into the stage first
    std::vector<Decoded> lengths_at(Codec& codec, const uint8_t* wire, const uint8_t* dev_wire, size_t wire_len,
                                    const std::vector<uint32_t>& rec_len, DecodeMode mode);
    std::vector<Decoded> stream_at(Codec& codec, const uint8_t* wire, const uint8_t* dev_wire, size_t wire_len,
                                   DecodeMode mode, size_t* consumed, std::optional<Error>* stop);
    // the decode outputs in staging regions, read after the synchronisation
    struct Out {
        detail::Region<onc_msg> msgs;
        detail::Region<onc_unix_params> unix;
        detail::Region<int32_t> status;
        detail::Region<uint32_t> aux0, aux1;
        onc_decoded dev() const { return onc_decoded{msgs.dev, unix.dev, status.dev, aux0.dev, aux1.dev}; }
    };
    static size_t out_bytes(size_t n);
    static Out take_out(detail::Carve& c, size_t n);
    static std::vector<Decoded> results(const Out& o, size_t n, const uint8_t* wire);
};

// expected_message_len (rpc_message.rs:343-367); throws Error.
inline uint32_t expected_message_len(Bytes data) {
    uint32_t n = 0;
    const int32_t st = onc_expected_message_len(data.ptr, data.len, &n);
    if (st != ONC_OK) throw Error(st);
    return n;
}

// ----------------------------------------------------------------------------
// BatchEncoder implementation
// ----------------------------------------------------------------------------
inline void BatchEncoder::put_auth(const AuthFlavor& a, onc_auth& d) {
    d.id = a.id();
    switch (a.kind()) {
        case AuthFlavor::Kind::AuthUnix: {
            const AuthUnixParams& p = a.unix_params();
            onc_unix_params u{};
            u.stamp = p.stamp();
            u.uid = p.uid();
            u.gid = p.gid();
            u.ngids = uint32_t(p.gids_vec().size());
            for (size_t i = 0; i < p.gids_vec().size(); ++i) u.gids[i] = p.gids_vec()[i];
            u.name_off = auth_.size();
            u.name_len = uint32_t(p.machine_name().len);
            auth_.insert(auth_.end(), p.machine_name().ptr, p.machine_name().ptr + p.machine_name().len);
            // ABI 6: declare serialised_len (unix_params.rs:219-230) so that the
            // encoder's length pass reads no parameter block; a block that
            // would panic is left undeclared (0: every check up front)
            const uint32_t ng = u.ngids, nl = u.name_len;
            d.kind_len = ONC_AUTH_PACK(ONC_KIND_UNIX, nl <= ONC_MAX_MACHINE_NAME_LEN && ng <= ONC_MAX_GIDS
                                                          ? 20u + 4u * ((nl + 3u) / 4u) + 4u * ng
                                                          : 0u);
            d.ref = unix_.size();
            unix_.push_back(u);
            return;
        }
        case AuthFlavor::Kind::AuthNone:
        case AuthFlavor::Kind::AuthShort:
        case AuthFlavor::Kind::Unknown: {
            const uint32_t kind = a.kind() == AuthFlavor::Kind::AuthNone    ? ONC_KIND_NONE
                                  : a.kind() == AuthFlavor::Kind::AuthShort ? ONC_KIND_SHORT
                                                                            : ONC_KIND_UNKNOWN;
            const Bytes b = a.data().value_or(Bytes());
            // Bodies longer than the 24-bit descriptor field cannot be
            // described; the reference would panic on them (> 200 bytes).
            if (b.len > 0xFFFFFFu) throw std::logic_error("auth associated data longer than 200 bytes");
            d.kind_len = ONC_AUTH_PACK(kind, b.len);
            d.ref = auth_.size();
            auth_.insert(auth_.end(), b.ptr, b.ptr + b.len);
            return;
        }
    }
}

inline void BatchEncoder::set_root(int root) {
    if (root_ >= 0 && root_ != root) throw std::logic_error("BatchEncoder: values of different types in one batch");
    root_ = root;
}

inline void BatchEncoder::put_payload(Bytes p, onc_msg& d) {
    if (p.len > 0xFFFFFFFFull) throw std::runtime_error("message length exceeds maximum");
    d.payload_len = uint32_t(p.len);
    d.payload_off = payload_.size();
    payload_.insert(payload_.end(), p.ptr, p.ptr + p.len);
}

inline void BatchEncoder::put_call(const CallBody& c, onc_msg& d) {
    d.msg_type = ONC_MSG_CALL;
    d.u.call.program = c.program();
    d.u.call.program_version = c.program_version();
    d.u.call.procedure = c.procedure();
    put_auth(c.auth_credentials(), d.cred);
    put_auth(c.auth_verifier(), d.verf);
    put_payload(c.payload(), d);
}

inline void BatchEncoder::put_status(const AcceptedStatus& s, onc_msg& d) {
    d.msg_type = ONC_MSG_REPLY;
    d.reply_stat = ONC_REPLY_ACCEPTED;
    d.stat = uint8_t(s.kind());
    if (s.kind() == AcceptedStatus::Kind::Success) {
        put_payload(s.payload(), d);
    } else if (s.kind() == AcceptedStatus::Kind::ProgramMismatch) {
        d.u.mismatch.low = s.mismatch().first;
        d.u.mismatch.high = s.mismatch().second;
    }
}

inline void BatchEncoder::put_accepted(const AcceptedReply& a, onc_msg& d) {
    put_auth(a.auth_verifier(), d.verf);
    put_status(a.status(), d);
}

inline void BatchEncoder::put_rejected(const RejectedReply& j, onc_msg& d) {
    d.msg_type = ONC_MSG_REPLY;
    d.reply_stat = ONC_REPLY_DENIED;
    if (j.kind() == RejectedReply::Kind::RpcVersionMismatch) {
        d.stat = ONC_REJECT_RPC_MISMATCH;
        d.u.mismatch.low = j.mismatch().first;
        d.u.mismatch.high = j.mismatch().second;
    } else {
        d.stat = ONC_REJECT_AUTH_ERROR;
        d.auth_stat = uint8_t(j.auth_error());
    }
}

inline void BatchEncoder::put_reply(const ReplyBody& r, onc_msg& d) {
    if (const AcceptedReply* a = r.accepted()) put_accepted(*a, d);
    else put_rejected(*r.denied(), d);
}

inline void BatchEncoder::push(const RpcMessage& m) {
    set_root(ONC_ROOT_RPC_MESSAGE);
    onc_msg d{};
    d.xid = m.xid();
    if (const CallBody* c = m.call_body()) put_call(*c, d);
    else put_reply(*m.reply_body(), d);
    msgs_.push_back(d);
}

inline void BatchEncoder::push(const MessageType& m) {
    set_root(ONC_ROOT_MESSAGE_TYPE);
    onc_msg d{};
    if (const CallBody* c = m.call_body()) put_call(*c, d);
    else put_reply(*m.reply_body(), d);
    msgs_.push_back(d);
}

inline void BatchEncoder::push(const CallBody& c) {
    set_root(ONC_ROOT_CALL_BODY);
    onc_msg d{};
    put_call(c, d);
    msgs_.push_back(d);
}

inline void BatchEncoder::push(const ReplyBody& r) {
    set_root(ONC_ROOT_REPLY_BODY);
    onc_msg d{};
    put_reply(r, d);
    msgs_.push_back(d);
}

inline void BatchEncoder::push(const AcceptedReply& r) {
    set_root(ONC_ROOT_ACCEPTED_REPLY);
    onc_msg d{};
    put_accepted(r, d);
    msgs_.push_back(d);
}

inline void BatchEncoder::push(const AcceptedStatus& s) {
    set_root(ONC_ROOT_ACCEPTED_STATUS);
    onc_msg d{};
    put_status(s, d);
    msgs_.push_back(d);
}

inline void BatchEncoder::push(const RejectedReply& r) {
    set_root(ONC_ROOT_REJECTED_REPLY);
    onc_msg d{};
    put_rejected(r, d);
    msgs_.push_back(d);
}

inline void BatchEncoder::push(AuthError e) {
    set_root(ONC_ROOT_AUTH_ERROR);
    onc_msg d{};
    put_rejected(RejectedReply::auth_error(e), d);
    msgs_.push_back(d);
}

inline void BatchEncoder::push(const AuthFlavor& a) {
    set_root(ONC_ROOT_AUTH_FLAVOR);
    onc_msg d{};
    d.msg_type = ONC_MSG_CALL;
    put_auth(a, d.cred);
    msgs_.push_back(d);
}

inline void BatchEncoder::push(const AuthUnixParams& p) {
    set_root(ONC_ROOT_AUTH_UNIX_PARAMS);
    onc_msg d{};
    d.msg_type = ONC_MSG_CALL;
    put_auth(AuthFlavor::unix(p), d.cred);
    msgs_.push_back(d);
}

inline size_t BatchEncoder::staged_bytes() const {
    using detail::need;
    return need<onc_msg>(msgs_.size()) + need<onc_unix_params>(unix_.size()) + need<uint8_t>(auth_.size()) +
           need<uint8_t>(payload_.size());
}

inline onc_batch BatchEncoder::stage_batch(detail::Carve& c) const {
    const size_t n = msgs_.size();
    const auto m = c.take<onc_msg>(n);
    const auto u = c.take<onc_unix_params>(unix_.size());
    const auto a = c.take<uint8_t>(auth_.size());
    const auto p = c.take<uint8_t>(payload_.size());
    if (n) std::memcpy(m.host, msgs_.data(), n * sizeof(onc_msg));
    if (!unix_.empty()) std::memcpy(u.host, unix_.data(), unix_.size() * sizeof(onc_unix_params));
    if (!auth_.empty()) std::memcpy(a.host, auth_.data(), auth_.size());
    if (!payload_.empty()) std::memcpy(p.host, payload_.data(), payload_.size());
    onc_batch b{};
    b.n = n;
    b.msgs = m.dev;
    b.unix_params = u.dev;
    b.auth_arena = a.dev;
    b.payload_arena = p.dev;
    b.unix_count = unix_.size();
    b.auth_len = auth_.size();
    b.payload_len = payload_.size();
    return b;
}

inline std::vector<uint32_t> BatchEncoder::serialised_lens(Codec& codec, std::vector<int32_t>* status) {
    using detail::need;
    const size_t n = msgs_.size();
    std::vector<uint32_t> lens(n);
    std::vector<int32_t> st(n);
    if (n) {
        detail::Carve c{codec.stage(staged_bytes() + need<uint32_t>(n) + need<int32_t>(n))};
        const onc_batch b = stage_batch(c);
        const auto dl = c.take<uint32_t>(n);
        const auto ds = c.take<int32_t>(n);
        codec.check(onc_encode_body_lengths(codec.get(), root(), &b, dl.dev, ds.dev), "onc_encode_body_lengths");
        codec.sync();
        std::memcpy(lens.data(), dl.host, n * 4);
        std::memcpy(st.data(), ds.host, n * 4);
    }
    if (status) *status = std::move(st);
    return lens;
}

// One encode pass: the output goes into the stage with a capacity no record
// can reach (a header is at most 460 bytes — 7 words and two auths of 54 —
// and a record keeping a declared extent at most 28 + 2 x 348 bytes before
// its payload), so no separate length pass is needed to size it; the bytes
// are then appended to `out`.
inline std::vector<int32_t> BatchEncoder::serialise_into(Codec& codec, std::vector<uint8_t>& out,
                                                         std::vector<uint64_t>* rec_off) {
    using detail::need;
    const size_t n = msgs_.size();
    std::vector<int32_t> st(n);
    std::vector<uint64_t> off(n + 1, 0);
    if (n) {
        const size_t cap = 1024 * n + payload_.size();
        detail::Carve c{codec.stage(staged_bytes() + need<uint8_t>(cap) + need<uint64_t>(n + 1) + need<int32_t>(n))};
        const onc_batch b = stage_batch(c);
        const auto dout = c.take<uint8_t>(cap);
        const auto doff = c.take<uint64_t>(n + 1);
        const auto ds = c.take<int32_t>(n);
        codec.check(onc_encode_body(codec.get(), root(), &b, dout.dev, cap, doff.dev, ds.dev, nullptr),
                    "onc_encode_body");
        codec.sync();
        std::memcpy(st.data(), ds.host, n * 4);
        // a failing message writes nothing (the reference panics or returns
        // before its first write): placeholder extents dropped (ABI 8)
        for (size_t i = 0; i < n; ++i) {
            if (st[i] != ONC_OK) {
                uint64_t kept = 0;
                codec.check(onc_compact(codec.get(), dout.dev, doff.dev, ds.dev, n, &kept), "onc_compact");
                break;
            }
        }
        std::memcpy(off.data(), doff.host, (n + 1) * 8);
        const uint64_t total = off[n];
        out.insert(out.end(), dout.host, dout.host + total);
    }
    if (rec_off) *rec_off = std::move(off);
    return st;
}

// ----------------------------------------------------------------------------
// BatchDecoder implementation: descriptors -> RpcMessage views over `wire`
// ----------------------------------------------------------------------------
namespace detail {

inline AuthFlavor auth_view(const onc_auth& a, const onc_unix_params* unix, const uint8_t* wire) {
    const uint32_t kind = ONC_AUTH_KIND(a);
    const uint32_t len = ONC_AUTH_LEN(a);
    switch (kind) {
        case ONC_KIND_NONE:
            // AuthNone with an empty body decodes to None (flavor.rs:71-78)
            return len == 0 ? AuthFlavor::none() : AuthFlavor::none(Bytes(wire + a.ref, len));
        case ONC_KIND_UNIX: {
            const onc_unix_params& u = unix[a.ref];
            return AuthFlavor::unix(AuthUnixParams(u.stamp, Bytes(wire + u.name_off, u.name_len), u.uid, u.gid,
                                                   std::vector<uint32_t>(u.gids, u.gids + u.ngids)));
        }
        case ONC_KIND_SHORT: return AuthFlavor::short_(Bytes(wire + a.ref, len));
        default: return AuthFlavor::unknown(a.id, Bytes(wire + a.ref, len));
    }
}

inline RpcMessage message_view(const onc_msg& d, const onc_unix_params* unix, const uint8_t* wire) {
    if (d.msg_type == ONC_MSG_CALL) {
        return RpcMessage(d.xid, MessageType::call(CallBody(d.u.call.program, d.u.call.program_version,
                                                            d.u.call.procedure, auth_view(d.cred, unix, wire),
                                                            auth_view(d.verf, unix, wire),
                                                            Bytes(wire + d.payload_off, d.payload_len))));
    }
    if (d.reply_stat == ONC_REPLY_ACCEPTED) {
        AcceptedStatus s = AcceptedStatus::of(AcceptedStatus::Kind(d.stat));
        if (d.stat == ONC_ACCEPT_SUCCESS) s = AcceptedStatus::success(Bytes(wire + d.payload_off, d.payload_len));
        if (d.stat == ONC_ACCEPT_PROG_MISMATCH) s = AcceptedStatus::program_mismatch(d.u.mismatch.low, d.u.mismatch.high);
        return RpcMessage(d.xid, MessageType::reply(ReplyBody::accepted(
                                     AcceptedReply(auth_view(d.verf, unix, wire), std::move(s)))));
    }
    RejectedReply j = d.stat == ONC_REJECT_RPC_MISMATCH
                          ? RejectedReply::rpc_version_mismatch(d.u.mismatch.low, d.u.mismatch.high)
                          : RejectedReply::auth_error(AuthError(d.auth_stat));
    return RpcMessage(d.xid, MessageType::reply(ReplyBody::denied(j)));
}

}  // namespace detail

inline size_t BatchDecoder::out_bytes(size_t n) {
    using detail::need;
    return need<onc_msg>(n) + need<onc_unix_params>(2 * n) + need<int32_t>(n) + 2 * need<uint32_t>(n);
}

inline BatchDecoder::Out BatchDecoder::take_out(detail::Carve& c, size_t n) {
    Out o;
    o.msgs = c.take<onc_msg>(n);
    o.unix = c.take<onc_unix_params>(2 * n);
    o.status = c.take<int32_t>(n);
    o.aux0 = c.take<uint32_t>(n);
    o.aux1 = c.take<uint32_t>(n);
    return o;
}

// Descriptors -> RpcMessage views over the caller's `wire` (offsets in the
// descriptors are relative to the decoded buffer, the same bytes).
inline std::vector<Decoded> BatchDecoder::results(const Out& o, size_t n, const uint8_t* wire) {
    std::vector<Decoded> res(n);
    for (size_t i = 0; i < n; ++i) {
        res[i].status = o.status.host[i];
        res[i].aux0 = o.aux0.host[i];
        res[i].aux1 = o.aux1.host[i];
        if (res[i].status == ONC_OK) res[i].message = detail::message_view(o.msgs.host[i], o.unix.host, wire);
    }
    return res;
}

// The wire is copied into the stage (the caller's buffer is not pinned) and
// decoded there in place by onc_decode_lengths (offsets inside the decode:
// one pass); the outputs land in the stage.
inline std::vector<Decoded> BatchDecoder::try_from(Codec& codec, const uint8_t* wire, size_t wire_len,
                                                   const std::vector<uint32_t>& rec_len, DecodeMode mode) {
    return lengths_at(codec, wire, nullptr, wire_len, rec_len, mode);
}

inline std::vector<Decoded> BatchDecoder::lengths_at(Codec& codec, const uint8_t* wire, const uint8_t* dev_wire,
                                                     size_t wire_len, const std::vector<uint32_t>& rec_len,
                                                     DecodeMode mode) {
    using detail::need;
    const size_t n = rec_len.size();
    if (!n) return {};
    detail::Carve c{codec.stage((dev_wire ? 0 : need<uint8_t>(wire_len)) + need<uint32_t>(n) + out_bytes(n))};
    const uint8_t* wd = dev_wire;
    if (!dev_wire) {
        const auto w = c.take<uint8_t>(wire_len);
        if (wire_len) std::memcpy(w.host, wire, wire_len);
        wd = w.dev;
    }
    const auto l = c.take<uint32_t>(n);
    std::memcpy(l.host, rec_len.data(), n * 4);
    const Out o = take_out(c, n);
    const onc_decoded d = o.dev();
    codec.check(onc_decode_lengths(codec.get(), wd, l.dev, n, 0, int(mode), nullptr, &d), "onc_decode_lengths");
    codec.sync();
    return results(o, n, wire);
}

inline std::vector<Decoded> BatchDecoder::try_from_stream(Codec& codec, const uint8_t* wire, size_t wire_len,
                                                          DecodeMode mode, size_t* consumed,
                                                          std::optional<Error>* stop) {
    return stream_at(codec, wire, nullptr, wire_len, mode, consumed, stop);
}

inline std::vector<Decoded> BatchDecoder::stream_at(Codec& codec, const uint8_t* wire, const uint8_t* dev_wire,
                                                    size_t wire_len, DecodeMode mode, size_t* consumed,
                                                    std::optional<Error>* stop) {
    using detail::need;
    // framed first with only the wire, the offsets (every record is at least
    // 4 bytes) and the result words staged; the decode outputs are carved
    // for the framed count afterwards (sized for max_records they would be
    // ~67 bytes of pinned memory per wire byte)
    const size_t max_records = wire_len / 4 + 1;
    detail::Carve c{codec.stage((dev_wire ? 0 : need<uint8_t>(wire_len)) + need<uint64_t>(max_records + 1) +
                                need<uint64_t>(5))};
    const uint8_t* wd = dev_wire;
    if (!dev_wire) {
        const auto w = c.take<uint8_t>(wire_len);
        if (wire_len) std::memcpy(w.host, wire, wire_len);
        wd = w.dev;
    }
    const size_t off_at = c.off;
    const auto off = c.take<uint64_t>(max_records + 1);
    const auto res = c.take<uint64_t>(5);
    codec.check(onc_frame_stream(codec.get(), wd, wire_len, off.dev, max_records, res.dev), "onc_frame_stream");
    codec.sync();
    uint64_t r[5];
    std::memcpy(r, res.host, sizeof(r));
    if (consumed) *consumed = size_t(r[1]);
    if (stop) {
        if (int32_t(r[2]) == ONC_OK) *stop = std::nullopt;
        else *stop = Error(int32_t(r[2]), uint32_t(r[3]), uint32_t(r[4]));
    }
    const size_t n = size_t(r[0]);
    if (!n) return {};
    // the outputs after what is staged (a stage that grows keeps the staged
    // wire and offsets; their device addresses move with it)
    const size_t mark = c.off;
    c.s = codec.stage(mark + out_bytes(n), mark);
    if (!dev_wire) wd = c.s.dev;
    const uint64_t* offd = reinterpret_cast<const uint64_t*>(c.s.dev + off_at);
    const Out o = take_out(c, n);
    const onc_decoded d = o.dev();
    codec.check(onc_decode(codec.get(), wd, offd, n, int(mode), &d), "onc_decode");
    codec.sync();
    return results(o, n, wire);
}

// ----------------------------------------------------------------------------
// RpcMessage single-message forms (batches of one)
// ----------------------------------------------------------------------------
inline uint32_t RpcMessage::serialised_len(Codec& codec) const {
    BatchEncoder e;
    e.push(*this);
    std::vector<int32_t> st;
    const uint32_t n = e.serialised_lens(codec, &st)[0];
    raise_encode_status(st[0]);
    return n;
}

inline void RpcMessage::serialise_into(Codec& codec, std::vector<uint8_t>& buf) const {
    BatchEncoder e;
    e.push(*this);
    raise_encode_status(e.serialise_into(codec, buf)[0]);
}

inline std::vector<uint8_t> RpcMessage::serialise(Codec& codec) const {
    std::vector<uint8_t> v;
    serialise_into(codec, v);
    return v;
}

inline RpcMessage RpcMessage::try_from(Codec& codec, Bytes buf, DecodeMode mode) {
    BatchDecoder d;
    std::vector<Decoded> r = d.try_from(codec, buf.ptr, buf.len, {uint32_t(buf.len)}, mode);
    if (!r[0].ok()) throw r[0].error();
    return std::move(*r[0].message);
}

// ----------------------------------------------------------------------------
// Body-level types (ONC_ROOT_*): TryFrom / serialise_into / serialised_len of
// one type of the message tree, on the GPU (onc_decode_body /
// onc_encode_body, batches of one like RpcMessage's single forms).
// ----------------------------------------------------------------------------
namespace detail {

// One record decoded as `root`; throws the reference's Error on failure.
struct BodyView {
    onc_msg d{};
    onc_unix_params unix[2]{};
};

inline BodyView decode_root(Codec& codec, int root, Bytes buf, DecodeMode mode, uint32_t param) {
    Carve c{codec.stage(need<uint8_t>(buf.len) + need<uint64_t>(2) + need<uint32_t>(1) + need<onc_msg>(1) +
                        need<onc_unix_params>(2) + 3 * need<uint32_t>(1))};
    const auto w = c.take<uint8_t>(buf.len);
    const auto o = c.take<uint64_t>(2);
    const auto p = c.take<uint32_t>(1);
    const auto m = c.take<onc_msg>(1);
    const auto u = c.take<onc_unix_params>(2);
    const auto s = c.take<int32_t>(1);
    const auto a0 = c.take<uint32_t>(1);
    const auto a1 = c.take<uint32_t>(1);
    if (buf.len) std::memcpy(w.host, buf.ptr, buf.len);
    o.host[0] = 0;
    o.host[1] = buf.len;
    p.host[0] = param;
    onc_decoded out{m.dev, u.dev, s.dev, a0.dev, a1.dev};
    codec.check(onc_decode_body(codec.get(), root, w.dev, o.dev, 1, int(mode), p.dev, &out, nullptr), "onc_decode_body");
    codec.sync();
    if (s.host[0] != ONC_OK) throw Error(s.host[0], a0.host[0], a1.host[0]);
    BodyView v;
    v.d = m.host[0];
    std::memcpy(v.unix, u.host, sizeof(v.unix));
    return v;
}

inline AcceptedStatus status_view(const onc_msg& d, const uint8_t* wire) {
    if (d.stat == ONC_ACCEPT_SUCCESS) return AcceptedStatus::success(Bytes(wire + d.payload_off, d.payload_len));
    if (d.stat == ONC_ACCEPT_PROG_MISMATCH) return AcceptedStatus::program_mismatch(d.u.mismatch.low, d.u.mismatch.high);
    return AcceptedStatus::of(AcceptedStatus::Kind(d.stat));
}

inline RejectedReply rejected_view(const onc_msg& d) {
    return d.stat == ONC_REJECT_RPC_MISMATCH ? RejectedReply::rpc_version_mismatch(d.u.mismatch.low, d.u.mismatch.high)
                                             : RejectedReply::auth_error(AuthError(d.auth_stat));
}

// serialised_len / serialise_into of one value pushed into a BatchEncoder.
template <class T>
inline uint32_t root_len(Codec& codec, const T& v) {
    BatchEncoder e;
    e.push(v);
    std::vector<int32_t> st;
    const uint32_t n = e.serialised_lens(codec, &st)[0];
    RpcMessage::raise_encode_status(st[0]);
    return n;
}

template <class T>
inline void root_into(Codec& codec, const T& v, std::vector<uint8_t>& buf) {
    BatchEncoder e;
    e.push(v);
    RpcMessage::raise_encode_status(e.serialise_into(codec, buf)[0]);
}

}  // namespace detail

inline MessageType MessageType::try_from(Codec& codec, Bytes buf, DecodeMode mode) {
    const detail::BodyView v = detail::decode_root(codec, ONC_ROOT_MESSAGE_TYPE, buf, mode, 0);
    return detail::message_view(v.d, v.unix, buf.ptr).message();
}
inline void MessageType::serialise_into(Codec& codec, std::vector<uint8_t>& buf) const { detail::root_into(codec, *this, buf); }
inline uint32_t MessageType::serialised_len(Codec& codec) const { return detail::root_len(codec, *this); }

inline CallBody CallBody::try_from(Codec& codec, Bytes buf, DecodeMode mode) {
    const detail::BodyView v = detail::decode_root(codec, ONC_ROOT_CALL_BODY, buf, mode, 0);
    return *detail::message_view(v.d, v.unix, buf.ptr).call_body();
}
inline void CallBody::serialise_into(Codec& codec, std::vector<uint8_t>& buf) const { detail::root_into(codec, *this, buf); }
inline uint32_t CallBody::serialised_len(Codec& codec) const { return detail::root_len(codec, *this); }

inline ReplyBody ReplyBody::try_from(Codec& codec, Bytes buf, DecodeMode mode) {
    const detail::BodyView v = detail::decode_root(codec, ONC_ROOT_REPLY_BODY, buf, mode, 0);
    return *detail::message_view(v.d, v.unix, buf.ptr).reply_body();
}
inline void ReplyBody::serialise_into(Codec& codec, std::vector<uint8_t>& buf) const { detail::root_into(codec, *this, buf); }
inline uint32_t ReplyBody::serialised_len(Codec& codec) const { return detail::root_len(codec, *this); }

inline AcceptedReply AcceptedReply::try_from(Codec& codec, Bytes buf, DecodeMode mode) {
    const detail::BodyView v = detail::decode_root(codec, ONC_ROOT_ACCEPTED_REPLY, buf, mode, 0);
    return AcceptedReply(detail::auth_view(v.d.verf, v.unix, buf.ptr), detail::status_view(v.d, buf.ptr));
}
inline void AcceptedReply::serialise_into(Codec& codec, std::vector<uint8_t>& buf) const { detail::root_into(codec, *this, buf); }
inline uint32_t AcceptedReply::serialised_len(Codec& codec) const { return detail::root_len(codec, *this); }

inline AcceptedStatus AcceptedStatus::try_from(Codec& codec, Bytes buf, DecodeMode mode) {
    const detail::BodyView v = detail::decode_root(codec, ONC_ROOT_ACCEPTED_STATUS, buf, mode, 0);
    return detail::status_view(v.d, buf.ptr);
}
inline void AcceptedStatus::serialise_into(Codec& codec, std::vector<uint8_t>& buf) const { detail::root_into(codec, *this, buf); }
inline uint32_t AcceptedStatus::serialised_len(Codec& codec) const { return detail::root_len(codec, *this); }

inline RejectedReply RejectedReply::try_from(Codec& codec, Bytes buf, DecodeMode mode) {
    return detail::rejected_view(detail::decode_root(codec, ONC_ROOT_REJECTED_REPLY, buf, mode, 0).d);
}
inline void RejectedReply::serialise_into(Codec& codec, std::vector<uint8_t>& buf) const { detail::root_into(codec, *this, buf); }
inline uint32_t RejectedReply::serialised_len(Codec& codec) const { return detail::root_len(codec, *this); }

inline AuthError auth_error_try_from(Codec& codec, Bytes buf, DecodeMode mode) {
    return AuthError(detail::decode_root(codec, ONC_ROOT_AUTH_ERROR, buf, mode, 0).d.auth_stat);
}
inline void serialise_into(Codec& codec, AuthError e, std::vector<uint8_t>& buf) { detail::root_into(codec, e, buf); }

inline AuthFlavor AuthFlavor::try_from(Codec& codec, Bytes buf, DecodeMode mode) {
    const detail::BodyView v = detail::decode_root(codec, ONC_ROOT_AUTH_FLAVOR, buf, mode, 0);
    return detail::auth_view(v.d.cred, v.unix, buf.ptr);
}
inline void AuthFlavor::serialise_into(Codec& codec, std::vector<uint8_t>& buf) const { detail::root_into(codec, *this, buf); }
inline uint32_t AuthFlavor::serialised_len(Codec& codec) const { return detail::root_len(codec, *this); }

inline AuthUnixParams AuthUnixParams::from_cursor(Codec& codec, Bytes buf, uint32_t expected_len) {
    const detail::BodyView v =
        detail::decode_root(codec, ONC_ROOT_AUTH_UNIX_PARAMS, buf, DecodeMode::Slice, expected_len);
    return detail::auth_view(v.d.cred, v.unix, buf.ptr).unix_params();
}
inline AuthUnixParams AuthUnixParams::try_from(Codec& codec, Bytes buf) {
    const detail::BodyView v = detail::decode_root(codec, ONC_ROOT_AUTH_UNIX_PARAMS, buf, DecodeMode::Bytes, 0);
    return detail::auth_view(v.d.cred, v.unix, buf.ptr).unix_params();
}
inline void AuthUnixParams::serialise_into(Codec& codec, std::vector<uint8_t>& buf) const { detail::root_into(codec, *this, buf); }
inline uint32_t AuthUnixParams::serialised_len(Codec& codec) const { return detail::root_len(codec, *this); }

}  // namespace onc_rpc
