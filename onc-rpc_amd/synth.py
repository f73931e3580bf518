"""Synthetic record batches for the BASELINE.json configs (host numpy,
vectorised). Seeds are fixed; every generator returns a layout.HostBatch.

  configs[0]  cpu_roundtrip   benches/bench.rs:86-101 message + 64 B payload
  configs[1]  call_none       1M Call(AuthNone x2), fixed 256 B payload
  configs[2]  mixed           1M mixed Call/Reply, payloads 64..4096 B
  configs[3]  call_unix16     4M Call(AuthUnix 16 gids) + 1 KiB payload
  configs[4]  call_none       64M x 256 B, sharded over GPUs
"""
from __future__ import annotations

import numpy as np

from . import layout as L

GIDS16 = np.array([501, 12, 20, 61, 79, 80, 81, 98, 701, 33, 100, 204, 250, 395, 398, 399],
                  dtype=np.uint32)

NONE_NONE = int(L.pack_kind_len(L.KIND_NONE, 0))


def _rng_bytes(rng, n):
    return np.frombuffer(rng.bytes(int(n)), dtype=np.uint8).copy() if n else np.zeros(1, np.uint8)


def call_none(n, payload_len=256, seed=1, first_xid=0):
    """configs[1]/[4]: Call(prog 100003, vers 4, proc 1, AuthNone(None) x2) + payload."""
    rng = np.random.default_rng(seed)
    msgs = np.zeros(n, L.MSG_DTYPE)
    msgs["xid"] = (np.arange(n, dtype=np.uint64) + first_xid).astype(np.uint32)
    msgs["msg_type"] = L.MSG_CALL
    msgs["f0"], msgs["f1"], msgs["f2"] = 100003, 4, 1
    msgs["payload_len"] = payload_len
    msgs["payload_off"] = np.arange(n, dtype=np.uint64) * np.uint64(payload_len)
    msgs["cred_kind_len"] = NONE_NONE
    msgs["verf_kind_len"] = NONE_NONE
    payload = _rng_bytes(rng, n * payload_len + 16)
    return L.HostBatch(msgs, np.zeros(1, L.UNIX_DTYPE), np.zeros(16, np.uint8), payload)


def call_unix16(n, payload_len=1024, seed=3, stamp_from_index=True, xid=None, prog=100003, vers=4,
                proc=1):
    """configs[3]: Call(AuthUnix(stamp=i, "", 501, 20, 16 gids), AuthNone) + payload.
    With stamp_from_index=False, xid=4242, prog=100000, vers=42, proc=13,
    payload_len=64 it is the benches/bench.rs:86-101 message (configs[0])."""
    rng = np.random.default_rng(seed)
    msgs = np.zeros(n, L.MSG_DTYPE)
    msgs["xid"] = np.arange(n, dtype=np.uint32) if xid is None else xid
    msgs["msg_type"] = L.MSG_CALL
    msgs["f0"], msgs["f1"], msgs["f2"] = prog, vers, proc
    msgs["payload_len"] = payload_len
    msgs["payload_off"] = np.arange(n, dtype=np.uint64) * np.uint64(payload_len)
    msgs["cred_id"] = 1
    msgs["cred_kind_len"] = int(L.pack_kind_len(L.KIND_UNIX, L.unix_body_len(0, 16)))   # declared (ABI 6)
    msgs["cred_ref"] = np.arange(n, dtype=np.uint64)
    msgs["verf_kind_len"] = NONE_NONE
    unix = np.zeros(n, L.UNIX_DTYPE)
    unix["stamp"] = np.arange(n, dtype=np.uint32) if stamp_from_index else 0
    unix["uid"], unix["gid"], unix["ngids"] = 501, 20, 16
    unix["gids"][:] = GIDS16
    payload = _rng_bytes(rng, n * payload_len + 16)
    return L.HostBatch(msgs, unix, np.zeros(16, np.uint8), payload)


def cpu_roundtrip(n, seed=0):
    """configs[0]: the reference bench message (benches/bench.rs:86-101) + 64 B payload."""
    return call_unix16(n, payload_len=64, seed=seed, stamp_from_index=False, xid=4242, prog=100000,
                       vers=42, proc=13)


def mixed(n, seed=2, pmin=64, pmax=4096, exotic=0.0):
    """configs[2]: 50% Call (cred AuthNone(None) 50% / AuthUnix
    50%: name 0-16 lowercase bytes, 0-16 random gids; verf AuthNone(None);
    payload U[pmin,pmax]) and 50% Reply (80% Accepted Success + payload,
    10% other AcceptedStatus, 10% Denied over RpcMismatch / AuthError 0-7).
    `exotic` > 0 additionally turns that fraction of auths into AuthShort /
    Unknown / AuthNone(Some) with 0-200 byte bodies (parity tests)."""
    rng = np.random.default_rng(seed)
    msgs = np.zeros(n, L.MSG_DTYPE)
    msgs["xid"] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    is_call = rng.random(n) < 0.5
    msgs["msg_type"] = np.where(is_call, L.MSG_CALL, L.MSG_REPLY)
    msgs["f0"] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    msgs["f1"] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    msgs["f2"] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)

    # replies
    u = rng.random(n)
    acc_success = ~is_call & (u < 0.8)
    acc_other = ~is_call & (u >= 0.8) & (u < 0.9)
    denied = ~is_call & (u >= 0.9)
    msgs["reply_stat"] = np.where(denied, L.REPLY_DENIED, L.REPLY_ACCEPTED)
    stat = np.zeros(n, np.uint8)
    stat[acc_other] = rng.integers(1, 6, int(acc_other.sum()))
    dchoice = rng.integers(0, 9, n)
    stat[denied] = np.where(dchoice[denied] == 0, 0, 1)
    msgs["stat"] = np.where(is_call, 0, stat)
    msgs["auth_stat"] = np.where(denied & (dchoice > 0), dchoice - 1, 0)
    msgs["f2"] = np.where(is_call, msgs["f2"], 0)

    has_payload = is_call | acc_success
    plen = rng.integers(pmin, pmax + 1, n).astype(np.uint64)
    plen[~has_payload] = 0
    poff = np.zeros(n, np.uint64)
    np.cumsum(plen[:-1], out=poff[1:])
    msgs["payload_len"] = plen.astype(np.uint32)
    msgs["payload_off"] = poff
    payload = _rng_bytes(rng, int(plen.sum()) + 16)

    # auths
    unix_cred = is_call & (rng.random(n) < 0.5)
    n_unix = int(unix_cred.sum())
    unix = np.zeros(max(n_unix, 1), L.UNIX_DTYPE)
    name_len = rng.integers(0, 17, n_unix).astype(np.uint64)
    name_off = np.zeros(n_unix, np.uint64)
    if n_unix:
        np.cumsum(name_len[:-1], out=name_off[1:])
    names = rng.integers(ord("a"), ord("z") + 1, int(name_len.sum()) + 1, dtype=np.uint8)
    unix["stamp"][:n_unix] = rng.integers(0, 2**32, n_unix, dtype=np.uint64).astype(np.uint32)
    unix["uid"][:n_unix] = rng.integers(0, 2**32, n_unix, dtype=np.uint64).astype(np.uint32)
    unix["gid"][:n_unix] = rng.integers(0, 2**32, n_unix, dtype=np.uint64).astype(np.uint32)
    ng = rng.integers(0, 17, n_unix)
    unix["ngids"][:n_unix] = ng
    g = rng.integers(0, 2**32, (n_unix, 16), dtype=np.uint64).astype(np.uint32)
    g[np.arange(16)[None, :] >= ng[:, None]] = 0
    unix["gids"][:n_unix] = g
    unix["name_off"][:n_unix] = name_off
    unix["name_len"][:n_unix] = name_len
    auth_arena = names

    msgs["cred_kind_len"] = NONE_NONE
    msgs["verf_kind_len"] = NONE_NONE
    msgs["cred_id"] = np.where(unix_cred, 1, 0)
    # three in four AUTH_UNIX credentials declare their serialised length
    # (ABI 6), the rest leave it 0: both planning paths in one batch
    decl = rng.random(n_unix) < 0.75
    blen = np.where(decl, 20 + 4 * ((name_len.astype(np.int64) + 3) // 4) + 4 * ng.astype(np.int64), 0)
    msgs["cred_kind_len"][unix_cred] = (np.uint32(L.KIND_UNIX) << np.uint32(24)) | blen.astype(np.uint32)
    msgs["cred_ref"][unix_cred] = np.arange(n_unix, dtype=np.uint64)

    if exotic > 0:
        extra = bytearray()
        base = len(auth_arena)
        for field in ("cred", "verf"):
            eligible = (is_call | (msgs["reply_stat"] == L.REPLY_ACCEPTED)) & ~unix_cred if field == "cred" \
                else (is_call | (msgs["reply_stat"] == L.REPLY_ACCEPTED))
            if field == "cred":
                eligible &= is_call
            pick = eligible & (rng.random(n) < exotic)
            idx = np.nonzero(pick)[0]
            kinds = rng.integers(0, 3, len(idx))
            lens = rng.integers(0, 201, len(idx))
            for j, i in enumerate(idx):
                k = [L.KIND_NONE, L.KIND_SHORT, L.KIND_UNKNOWN][kinds[j]]
                ln = int(lens[j]) if k != L.KIND_NONE else max(1, int(lens[j]))
                msgs[field + "_id"][i] = {L.KIND_NONE: 0, L.KIND_SHORT: 2}.get(
                    k, int(rng.integers(3, 2**32, dtype=np.uint64)))
                msgs[field + "_kind_len"][i] = int(L.pack_kind_len(k, ln))
                msgs[field + "_ref"][i] = base + len(extra)
                extra.extend(rng.bytes(ln))
        auth_arena = np.concatenate([auth_arena, np.frombuffer(bytes(extra) + b"\0", np.uint8)])
    return L.HostBatch(msgs, unix, auth_arena, payload)


def random_messages(n, seed=0, max_payload=1025):
    """Message dicts drawn like the reference's proptest strategies
    (src/rpc_message.rs:997-1124): every AuthFlavor (AuthNone Option<0..=200>,
    AuthUnix name 0..=16 B / 0..=16 gids, AuthShort 0..=200, Unknown any id),
    payloads 0..=1025 B, every AcceptedStatus / RejectedReply / AuthError."""
    rng = np.random.default_rng(seed)

    def by(k):
        return rng.bytes(int(k)).hex()

    def auth():
        c = rng.integers(0, 4)
        if c == 0:
            return {"kind": "none", "data": by(rng.integers(1, 201)) if rng.random() < 0.5 else None}
        if c == 1:
            return {"kind": "unix", "stamp": int(rng.integers(0, 2**32)), "machine_name": by(rng.integers(0, 17)),
                    "uid": int(rng.integers(0, 2**32)), "gid": int(rng.integers(0, 2**32)),
                    "gids": [int(x) for x in rng.integers(0, 2**32, rng.integers(0, 17))]}
        if c == 2:
            return {"kind": "short", "data": by(rng.integers(0, 201))}
        return {"kind": "unknown", "id": int(rng.integers(3, 2**32)), "data": by(rng.integers(0, 201))}

    out = []
    for _ in range(n):
        xid = int(rng.integers(0, 2**32))
        if rng.random() < 0.5:
            out.append({"xid": xid, "type": "call", "program": int(rng.integers(0, 2**32)),
                        "program_version": int(rng.integers(0, 2**32)),
                        "procedure": int(rng.integers(0, 2**32)), "cred": auth(), "verf": auth(),
                        "payload": by(rng.integers(0, max_payload + 1))})
        elif rng.random() < 0.5:
            st = list(L.ACCEPT)[int(rng.integers(0, 6))]
            m = {"xid": xid, "type": "reply", "reply": "accepted", "verf": auth(), "accept_status": st}
            if st == "success":
                m["payload"] = by(rng.integers(0, max_payload + 1))
            if st == "prog_mismatch":
                m["low"], m["high"] = int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32))
            out.append(m)
        else:
            if rng.random() < 0.5:
                out.append({"xid": xid, "type": "reply", "reply": "denied", "rejected": "rpc_mismatch",
                            "low": int(rng.integers(0, 2**32)), "high": int(rng.integers(0, 2**32))})
            else:
                out.append({"xid": xid, "type": "reply", "reply": "denied", "rejected": "auth_error",
                            "auth_error": int(rng.integers(0, 8))})
    return out


def corrupt(wire: np.ndarray, rec_off: np.ndarray, frac=0.05, seed=7):
    """Mutated copies of records for error-path parity (fuzz-like). Returns
    a new (wire, rec_off): each picked record gets one of: a flipped byte,
    a truncation, a few trailing bytes, or a cleared last-fragment bit."""
    rng = np.random.default_rng(seed)
    recs = [bytearray(wire[rec_off[i]:rec_off[i + 1]].tobytes()) for i in range(len(rec_off) - 1)]
    for i in np.nonzero(rng.random(len(recs)) < frac)[0]:
        r = recs[i]
        op = rng.integers(0, 5)
        if op == 0 and len(r):
            j = int(rng.integers(0, len(r)))
            r[j] ^= int(rng.integers(1, 256))
        elif op == 1 and len(r):
            del r[int(rng.integers(0, len(r))):]
        elif op == 2:
            r.extend(rng.bytes(int(rng.integers(1, 9))))
            hdr = (len(r) - 4) | 0x80000000
            r[0:4] = hdr.to_bytes(4, "big")
        elif op == 3 and len(r) >= 4:
            r[0] &= 0x7F
        elif len(r) >= 24:
            # rewrite a word in the header area with a small random value
            j = 4 * int(rng.integers(1, min(len(r) // 4, 12)))
            r[j:j + 4] = int(rng.integers(0, 300)).to_bytes(4, "big")
        recs[i] = r
    return L.records_from_wire([bytes(r) for r in recs])


def call_none_device(lo, hi, payload_len=256, seed=1, device="cuda"):
    """configs[1]/[4] records [lo, hi) generated directly in HBM (torch on the
    device; a 64M-record batch is 16.4 GB of payload, too much to build in
    host numpy and copy): the descriptors of call_none (xid = record index,
    prog 100003, vers 4, proc 1, AuthNone(None) x2, payload_len bytes at
    payload_off = (i - lo) * payload_len) and a device-RNG payload arena
    (torch.Generator seeded with (seed, lo), so every shard is reproducible
    on its own). Returns (runtime.DeviceBatch, generator seed)."""
    import torch

    from . import runtime as R
    n = hi - lo
    m = torch.zeros((max(n, 1), 16), dtype=torch.int32, device=device)
    if n:
        m[:n, 0] = (torch.arange(lo, hi, dtype=torch.int64, device=device) & 0xFFFFFFFF).to(torch.int32)
        m[:n, 2], m[:n, 3], m[:n, 4], m[:n, 5] = 100003, 4, 1, payload_len
        m.view(torch.int64)[:n, 3] = torch.arange(n, dtype=torch.int64, device=device) * payload_len
    gseed = (int(seed) * 1_000_003 + int(lo)) & 0x7FFFFFFFFFFFFFFF
    g = torch.Generator(device=device)
    g.manual_seed(gseed)
    payload = torch.randint(0, 256, (n * payload_len + 16,), dtype=torch.uint8, device=device, generator=g)
    msgs = m.view(torch.uint8).reshape(-1)
    unix = torch.zeros(96, dtype=torch.uint8, device=device)
    auth = torch.zeros(16, dtype=torch.uint8, device=device)
    return R.DeviceBatch(n, msgs, unix, auth, payload), gseed


def host_window(db, lo, hi):
    """Records [lo, hi) of a call_none_device batch as a host HostBatch
    (descriptors + their payload bytes, offsets rebased) for an oracle check."""
    import numpy as np
    msgs = db.msgs.view(-1, 64)[lo:hi].cpu().numpy().copy().view(L.MSG_DTYPE).reshape(-1)
    p0 = int(msgs["payload_off"][0]) if hi > lo else 0
    p1 = int((msgs["payload_off"].astype(np.int64) + msgs["payload_len"]).max()) if hi > lo else 0
    pay = db.payload_arena[p0:p1 + 16].cpu().numpy().copy()
    msgs["payload_off"] -= np.uint64(p0)
    return L.HostBatch(msgs, np.zeros(1, L.UNIX_DTYPE), np.zeros(16, np.uint8), pay)
