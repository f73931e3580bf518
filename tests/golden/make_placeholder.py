"""Golden fixture for the batch encode's framable placeholder (ABI 7) and its
compaction (onc_compact, ABI 8), built here with struct.pack alone — no
oracle, no library — so that both are pinned independently of the C
restatement (oracle/onc_oracle.c) that tests/test_oracle_golden.py checks
against it.

The batch (tests/test_oracle_golden.py::test_declared_extent_placeholder
builds the same descriptors): seven messages; xid 2's declared AUTH_UNIX
credential carries 17 gids (Gids::from_iter panics, unix_params.rs:47) under
a plausible declared length, so the batch encode keeps its declared extent
as a placeholder: BE32((extent - 4) | 1 << 31) (the record mark,
rpc_message.rs:156) then zeros up to the payload, then the payload. xid 3
(the same block next to a 201-byte verifier: the Gids panic comes first,
status 103, and a record failing a check besides the deferred one takes no
bytes), xid 4 (an undeclared broken block) and xid 6 (an accepted reply
whose AUTH_UNIX verifier has a 300-byte name, unix_params.rs:149) write
nothing. The compacted stream is
what a loop of serialise_into calls writes: messages 1, 5 and 7.

Usage: python tests/golden/make_placeholder.py  (writes placeholder.json)
"""
import json
import os
import struct


def u32(*v):
    return b"".join(struct.pack(">I", x) for x in v)


def opaque(b):
    return u32(len(b)) + b + b"\0" * ((4 - len(b) % 4) % 4)


def unix_body(stamp, name, uid, gid, gids):
    # AuthUnixParams::serialise_into (unix_params.rs:162-176)
    return u32(stamp) + opaque(name) + u32(uid, gid, len(gids), *gids)


def auth_unix(stamp, name, uid, gid, gids):
    body = unix_body(stamp, name, uid, gid, gids)
    return u32(1, len(body)) + body                       # flavor.rs:106-129


AUTH_NONE = u32(0, 0)


def call(xid, cred, verf, payload):
    # RpcMessage::serialise_into (rpc_message.rs:136-164) of a Call
    body = u32(xid, 0, 2, 100003, 4, 1) + cred + verf + payload
    return u32((len(body)) | 0x80000000) + body


def main():
    cred = auth_unix(7, b"host", 1, 2, [3, 4, 5])
    pay = b"\x11" * 10
    m1 = call(1, cred, AUTH_NONE, pay)
    ext = len(m1)                                         # xid 2 declares the same credential length
    m2 = u32((ext - 4) | 0x80000000) + b"\0" * (ext - 4 - len(pay)) + pay
    m5 = call(5, AUTH_NONE, AUTH_NONE, pay)
    m7 = call(7, AUTH_NONE, AUTH_NONE, pay)
    stream = [m1, m2, b"", b"", m5, b"", m7]
    off = [0]
    for r in stream:
        off.append(off[-1] + len(r))
    kept = [m1, m5, m7]
    status = [0, 103, 103, 103, 0, 102, 0]
    koff = [0]                                            # a failing record: empty, where the next one starts
    for r, st in zip(stream, status):
        koff.append(koff[-1] + (len(r) if st == 0 else 0))
    fx = {
        "source": "tests/golden/make_placeholder.py (struct.pack; no oracle): include/onc_rpc.h onc_auth (ABI 7) "
                  "placeholder, onc_compact (ABI 8); reference: rpc_message.rs:136-164,156,343-367; "
                  "unix_params.rs:47,149,162-176; flavor.rs:106-129",
        "status": status,
        "wire": b"".join(stream).hex(),
        "rec_off": off,
        "placeholder": {"index": 1, "extent": ext},
        "compacted": b"".join(kept).hex(),
        "compacted_rec_off": koff,
    }
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "placeholder.json")
    with open(path, "w") as f:
        json.dump(fx, f, indent=1)
        f.write("\n")
    print(path, len(fx["wire"]) // 2, "bytes")


if __name__ == "__main__":
    main()
