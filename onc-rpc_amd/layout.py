"""Host-side mirror of the C ABI descriptors (include/onc_rpc.h) as numpy
structured dtypes, plus builders/describers between the reference's value
model and descriptor batches.

The value model ("message dicts") mirrors the reference's Rust types:

  RpcMessage { xid, MessageType }                 src/rpc_message.rs:97-105
  MessageType::Call(CallBody) / Reply(ReplyBody)  src/rpc_message.rs:22-32
  CallBody { program, program_version, procedure, auth_credentials,
             auth_verifier, payload }             src/call_body.rs:17-30
  AuthFlavor::{AuthNone(Option<T>), AuthUnix(AuthUnixParams), AuthShort(T),
               Unknown{id, data}}                 src/auth/flavor.rs:18-49
  AcceptedStatus / RejectedReply / AuthError      src/reply/*.rs

as plain dicts, e.g.
  {"xid": 1, "type": "call", "program": 100003, "program_version": 4,
   "procedure": 1, "cred": {"kind": "unix", "stamp": 0, "machine_name": "",
   "uid": 501, "gid": 20, "gids": [...]}, "verf": {"kind": "none",
   "data": None}, "payload": "<hex>"}
Byte strings are hex. This module is pure host logic (no codec work).
"""
from __future__ import annotations

import numpy as np

# --- constants (include/onc_rpc.h) -----------------------------------------
MSG_CALL, MSG_REPLY = 0, 1
REPLY_ACCEPTED, REPLY_DENIED = 0, 1
KIND_NONE, KIND_UNIX, KIND_SHORT, KIND_UNKNOWN = 0, 1, 2, 3
DECODE_SLICE, DECODE_BYTES = 0, 1
# body-level roots (include/onc_rpc.h ONC_ROOT_*): the reference type a
# record is decoded / serialised as
(ROOT_RPC_MESSAGE, ROOT_MESSAGE_TYPE, ROOT_CALL_BODY, ROOT_REPLY_BODY, ROOT_ACCEPTED_REPLY, ROOT_ACCEPTED_STATUS,
 ROOT_REJECTED_REPLY, ROOT_AUTH_ERROR, ROOT_AUTH_FLAVOR, ROOT_AUTH_UNIX_PARAMS, ROOT_OPAQUE) = range(11)
ROOT_NAMES = ["RpcMessage", "MessageType", "CallBody", "ReplyBody", "AcceptedReply", "AcceptedStatus",
              "RejectedReply", "AuthError", "AuthFlavor", "AuthUnixParams", "Opaque"]
OPAQUE_ENCODE_MAX = 255
OPAQUE_MAX_LEN = 0xFFFFFF

ACCEPT = {"success": 0, "prog_unavail": 1, "prog_mismatch": 2, "proc_unavail": 3,
          "garbage_args": 4, "system_err": 5}
ACCEPT_NAME = {v: k for k, v in ACCEPT.items()}
REJECT = {"rpc_mismatch": 0, "auth_error": 1}
REJECT_NAME = {v: k for k, v in REJECT.items()}
KIND = {"none": KIND_NONE, "unix": KIND_UNIX, "short": KIND_SHORT, "unknown": KIND_UNKNOWN}
KIND_NAME = {v: k for k, v in KIND.items()}

STATUS = {
    0: "Ok", 1: "IncompleteMessage", 2: "IncompleteHeader", 3: "Fragmented",
    4: "InvalidMessageType", 5: "InvalidReplyType", 6: "InvalidReplyStatus",
    7: "InvalidAuthData", 8: "InvalidAuthError", 9: "InvalidRejectedReplyType",
    10: "InvalidLength", 11: "InvalidRpcVersion", 12: "InvalidMachineName",
    13: "IOError(UnexpectedEof)",
    100: "EncTooLong", 101: "EncAuthGt200", 102: "EncNameGt255", 103: "EncGidsGt16",
    104: "EncBadDescriptor", 105: "EncWriteZero",
}

# --- dtypes ------------------------------------------------------------------
MSG_DTYPE = np.dtype({
    "names": ["xid", "msg_type", "reply_stat", "stat", "auth_stat", "f0", "f1", "f2",
              "payload_len", "payload_off",
              "cred_id", "cred_kind_len", "cred_ref", "verf_id", "verf_kind_len", "verf_ref"],
    "formats": ["<u4", "u1", "u1", "u1", "u1", "<u4", "<u4", "<u4", "<u4", "<u8",
                "<u4", "<u4", "<u8", "<u4", "<u4", "<u8"],
    "offsets": [0, 4, 5, 6, 7, 8, 12, 16, 20, 24, 32, 36, 40, 48, 52, 56],
    "itemsize": 64,
})
UNIX_DTYPE = np.dtype({
    "names": ["stamp", "uid", "gid", "ngids", "name_off", "name_len", "reserved", "gids"],
    "formats": ["<u4", "<u4", "<u4", "<u4", "<u8", "<u4", "<u4", ("<u4", (16,))],
    "offsets": [0, 4, 8, 12, 16, 24, 28, 32],
    "itemsize": 96,
})
IOV_DTYPE = np.dtype({
    "names": ["hdr_off", "payload_off", "wire_off", "hdr_len", "payload_len"],
    "formats": ["<u8", "<u8", "<u8", "<u4", "<u4"],
    "offsets": [0, 8, 16, 24, 28],
    "itemsize": 32,
})
assert MSG_DTYPE.itemsize == 64 and UNIX_DTYPE.itemsize == 96 and IOV_DTYPE.itemsize == 32


def pack_kind_len(kind, length):
    return (np.uint32(kind) << np.uint32(24)) | (np.uint32(length) & np.uint32(0xFFFFFF))


def kind_of(kind_len):
    return int(kind_len) >> 24


def len_of(kind_len):
    return int(kind_len) & 0xFFFFFF


# --- builder -----------------------------------------------------------------
class HostBatch:
    """A batch of messages in descriptor form (host numpy arrays)."""

    def __init__(self, msgs, unix, auth_arena, payload_arena):
        self.msgs = msgs
        self.unix = unix
        self.auth_arena = auth_arena
        self.payload_arena = payload_arena

    @property
    def n(self):
        return len(self.msgs)


def unix_body_len(name_len, ngids):
    """AuthUnixParams::serialised_len (unix_params.rs:219-230)."""
    return 20 + 4 * ((name_len + 3) // 4) + 4 * ngids


def build_batch(messages, declare=True):
    """message dicts -> HostBatch (construction of the reference values;
    limits are NOT enforced here so that the codec's panic statuses can be
    exercised). declare: AUTH_UNIX auths within the limits carry their
    serialised length in onc_auth.len (ABI 6; the encoder's length pass then
    reads no parameter block); False leaves every one 0 (undeclared)."""
    n = len(messages)
    msgs = np.zeros(n, MSG_DTYPE)
    unix_rows = []
    auth = bytearray()
    payload = bytearray()

    def put_auth(prefix, i, a):
        kind = KIND[a["kind"]]
        msgs[prefix + "_id"][i] = {KIND_NONE: 0, KIND_UNIX: 1, KIND_SHORT: 2}.get(kind, a.get("id", 0))
        if kind == KIND_UNIX:
            name = bytes.fromhex(a["machine_name"])
            row = np.zeros(1, UNIX_DTYPE)[0]
            row["stamp"], row["uid"], row["gid"] = a["stamp"], a["uid"], a["gid"]
            row["ngids"] = len(a["gids"])
            row["name_off"] = len(auth)
            row["name_len"] = len(name)
            g = list(a["gids"])[:16]
            row["gids"][: len(g)] = g
            auth.extend(name)
            ok = len(name) <= 255 and len(a["gids"]) <= 16
            msgs[prefix + "_kind_len"][i] = pack_kind_len(
                KIND_UNIX, unix_body_len(len(name), len(a["gids"])) if declare and ok else 0)
            msgs[prefix + "_ref"][i] = len(unix_rows)
            unix_rows.append(row)
        else:
            data = bytes.fromhex(a["data"]) if a.get("data") else b""
            msgs[prefix + "_kind_len"][i] = pack_kind_len(kind, len(data))
            msgs[prefix + "_ref"][i] = len(auth)
            auth.extend(data)

    for i, m in enumerate(messages):
        msgs["xid"][i] = m["xid"]
        if m["type"] == "call":
            msgs["msg_type"][i] = MSG_CALL
            msgs["f0"][i], msgs["f1"][i], msgs["f2"][i] = (m["program"], m["program_version"],
                                                          m["procedure"])
            put_auth("cred", i, m["cred"])
            put_auth("verf", i, m["verf"])
            p = bytes.fromhex(m.get("payload", ""))
            msgs["payload_off"][i] = len(payload)
            msgs["payload_len"][i] = len(p)
            payload.extend(p)
        else:
            msgs["msg_type"][i] = MSG_REPLY
            if m["reply"] == "accepted":
                msgs["reply_stat"][i] = REPLY_ACCEPTED
                msgs["stat"][i] = ACCEPT[m["accept_status"]]
                put_auth("verf", i, m["verf"])
                if m["accept_status"] == "prog_mismatch":
                    msgs["f0"][i], msgs["f1"][i] = m["low"], m["high"]
                if m["accept_status"] == "success":
                    p = bytes.fromhex(m.get("payload", ""))
                    msgs["payload_off"][i] = len(payload)
                    msgs["payload_len"][i] = len(p)
                    payload.extend(p)
            else:
                msgs["reply_stat"][i] = REPLY_DENIED
                msgs["stat"][i] = REJECT[m["rejected"]]
                if m["rejected"] == "rpc_mismatch":
                    msgs["f0"][i], msgs["f1"][i] = m["low"], m["high"]
                else:
                    msgs["auth_stat"][i] = m["auth_error"]
    unix = np.array(unix_rows, dtype=UNIX_DTYPE) if unix_rows else np.zeros(1, UNIX_DTYPE)
    return HostBatch(msgs, unix, np.frombuffer(bytes(auth) + b"\0", np.uint8).copy(),
                     np.frombuffer(bytes(payload) + b"\0", np.uint8).copy())


# --- describer -----------------------------------------------------------------
def describe_auth(m, prefix, unix, arena):
    kl = int(m[prefix + "_kind_len"])
    kind, ln = kind_of(kl), len_of(kl)
    ref = int(m[prefix + "_ref"])
    if kind == KIND_UNIX:
        u = unix[ref]
        no, nl = int(u["name_off"]), int(u["name_len"])
        ng = int(u["ngids"])
        return {"kind": "unix", "stamp": int(u["stamp"]),
                "machine_name": bytes(arena[no:no + nl]).hex(), "uid": int(u["uid"]),
                "gid": int(u["gid"]), "gids": [int(x) for x in u["gids"][:ng]]}
    data = bytes(arena[ref:ref + ln]).hex()
    if kind == KIND_NONE:
        return {"kind": "none", "data": data if ln else None}
    if kind == KIND_SHORT:
        return {"kind": "short", "data": data}
    return {"kind": "unknown", "id": int(m[prefix + "_id"]), "data": data}


def describe(m, unix, auth_arena, payload_arena=None):
    """One descriptor (numpy record) -> message dict (inverse of build_batch)."""
    if payload_arena is None:
        payload_arena = auth_arena
    po, pl = int(m["payload_off"]), int(m["payload_len"])
    d = {"xid": int(m["xid"])}
    if int(m["msg_type"]) == MSG_CALL:
        d.update({"type": "call", "program": int(m["f0"]), "program_version": int(m["f1"]),
                  "procedure": int(m["f2"]),
                  "cred": describe_auth(m, "cred", unix, auth_arena),
                  "verf": describe_auth(m, "verf", unix, auth_arena),
                  "payload": bytes(payload_arena[po:po + pl]).hex()})
        return d
    d["type"] = "reply"
    if int(m["reply_stat"]) == REPLY_ACCEPTED:
        st = ACCEPT_NAME[int(m["stat"])]
        d.update({"reply": "accepted", "verf": describe_auth(m, "verf", unix, auth_arena),
                  "accept_status": st})
        if st == "prog_mismatch":
            d.update({"low": int(m["f0"]), "high": int(m["f1"])})
        if st == "success":
            d["payload"] = bytes(payload_arena[po:po + pl]).hex()
        return d
    rj = REJECT_NAME[int(m["stat"])]
    d.update({"reply": "denied", "rejected": rj})
    if rj == "rpc_mismatch":
        d.update({"low": int(m["f0"]), "high": int(m["f1"])})
    else:
        d["auth_error"] = int(m["auth_stat"])
    return d


def unix_used(msgs, status):
    """(cred, verf) masks of the auths whose AUTH_UNIX parameters a decode
    defines: OK records, kind UNIX, a credential of a call / a verifier of a
    call or accepted reply."""
    ok = status == 0
    cred = ok & (msgs["msg_type"] == MSG_CALL) & ((msgs["cred_kind_len"] >> 24) == KIND_UNIX)
    verf = ok & ((msgs["msg_type"] == MSG_CALL) | (msgs["reply_stat"] == REPLY_ACCEPTED)) & \
        ((msgs["verf_kind_len"] >> 24) == KIND_UNIX)
    return cred, verf


def resolve_unix(msgs, unix, status):
    """A decoded batch with its AUTH_UNIX slots resolved: (descriptors with
    the unix refs zeroed, (n, 2, 96) bytes of each record's credential /
    verifier parameters, zero where none). Two decodes that place the slots
    differently (per-group packing of different batch partitions) agree on
    this form exactly when they decoded the same messages."""
    m = msgs.copy()
    params = np.zeros((len(msgs), 2, UNIX_DTYPE.itemsize), np.uint8)
    ub = unix.view(np.uint8).reshape(-1, UNIX_DTYPE.itemsize)
    for k, (f, mask) in enumerate(zip(("cred", "verf"), unix_used(msgs, status))):
        idx = np.nonzero(mask)[0]
        params[idx, k] = ub[m[f + "_ref"][idx].astype(np.int64)]
        m[f + "_ref"][idx] = 0
    return m, params


def records_from_wire(wire_list):
    """list of per-record byte strings -> (packed wire uint8 array, rec_off u64[n+1])."""
    lens = np.array([len(w) for w in wire_list], dtype=np.uint64)
    off = np.zeros(len(wire_list) + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    wire = np.frombuffer(b"".join(wire_list) + b"\0" * 16, np.uint8).copy()
    return wire, off
