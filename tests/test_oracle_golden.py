"""Pins the CPU oracle (oracle/onc_oracle.c) to the reference's own golden
vectors (tests/golden/vectors.json, transcribed from the reference's unit
tests with citations) and to independent xdrlib-built messages.

These mirror the reference tests they cite: decode → field asserts →
serialise → byte equality.
"""
import os

import numpy as np
import pytest

import onc_rpc_amd.layout as L

MODES = {"slice": L.DECODE_SLICE, "bytes": L.DECODE_BYTES}


def _subset(expect, got, path=""):
    for k, v in expect.items():
        assert k in got, f"{path}{k} missing in {got}"
        if isinstance(v, dict):
            _subset(v, got[k], path + k + ".")
        else:
            assert got[k] == v, f"{path}{k}: got {got[k]!r} want {v!r}"


def _decoded_view(oracle, buf, mode):
    st, msg, unix, a0, a1, b = oracle.decode_message(buf, mode)
    return st, msg, unix, a0, a1, b


def _reserialise(oracle, msg, unix, b):
    hb = L.HostBatch(np.array([msg], L.MSG_DTYPE), unix, b, b)
    st, out, slen = oracle.encode_message(hb)
    assert st == 0
    return out, slen


def _extras(oracle, msg, unix, total):
    lib = oracle.load()
    ex = {"serialised_len": total}
    m = np.array([msg], L.MSG_DTYPE)
    raw_msg = m.tobytes()
    cred, verf = raw_msg[32:48], raw_msg[48:64]   # onc_msg.cred / .verf

    def slen(a):
        raw = np.frombuffer(a, np.uint8).copy()
        return lib.oracle_auth_serialised_len(raw.ctypes.data, unix.ctypes.data)

    ex["cred_serialised_len"] = slen(cred)
    ex["cred_params_serialised_len"] = ex["cred_serialised_len"] - 8
    ex["verf_serialised_len"] = slen(verf)
    ex["payload_len"] = int(msg["payload_len"])
    if int(msg["msg_type"]) == 1 and int(msg["reply_stat"]) == 0:
        st_len = 4 + (int(msg["payload_len"]) if int(msg["stat"]) == 0 else
                      8 if int(msg["stat"]) == 2 else 0)
        ex["accepted_serialised_len"] = ex["verf_serialised_len"] + st_len
    return ex


@pytest.mark.parametrize("mode", ["slice", "bytes"])
def test_reference_messages(oracle, golden, mode):
    for v in golden["messages"]:
        if mode not in v["modes"]:
            continue
        buf = bytes.fromhex(v["hex"])
        st, msg, unix, a0, a1, b = _decoded_view(oracle, buf, MODES[mode])
        assert st == v["expect"]["status"], v["name"]
        got = L.describe(msg, unix, b)
        out, slen = _reserialise(oracle, msg, unix, b)
        got.update(_extras(oracle, msg, unix, slen))
        got["status"] = st
        exp = {k: val for k, val in v["expect"].items()}
        if "machine_name" in exp.get("cred", {}):
            exp["cred"] = dict(exp["cred"], machine_name=exp["cred"]["machine_name"].encode().hex())
        _subset(exp, got, v["name"] + ":")
        if v.get("reserialise_equal"):
            assert out == buf, v["name"]
        if "expected_message_len" in v:
            w = np.zeros(1, np.uint32)
            rc = oracle.load().oracle_expected_message_len(b.ctypes.data, len(buf), w.ctypes.data)
            assert rc == 0 and int(w[0]) == v["expected_message_len"]


@pytest.mark.parametrize("mode", ["slice", "bytes"])
def test_reference_error_vectors(oracle, golden, mode):
    for v in golden["errors"]:
        buf = bytes.fromhex(v["hex"])
        st, msg, unix, a0, a1, b = _decoded_view(oracle, buf, MODES[mode])
        e = v["expect"]
        assert st == e["status"], (v["name"], st)
        if "aux0" in e:
            assert (a0, a1) == (e["aux0"], e["aux1"]), v["name"]


def test_reference_auth_vectors(oracle, golden):
    lib = oracle.load()
    for v in golden["auth"]:
        buf = bytes.fromhex(v["hex"])
        b = np.frombuffer(buf + b"\0" * 8, np.uint8).copy()
        auth = np.zeros(16, np.uint8)
        unix = np.zeros(1, L.UNIX_DTYPE)
        consumed = np.zeros(1, np.uint64)
        st = lib.oracle_auth_decode(b.ctypes.data, len(buf), L.DECODE_SLICE, auth.ctypes.data,
                                    unix.ctypes.data, consumed.ctypes.data)
        assert st == 0, v["name"]
        a = auth.view(np.dtype([("id", "<u4"), ("kind_len", "<u4"), ("ref", "<u8")]))[0]
        e = v["expect"]
        assert lib.oracle_auth_serialised_len(auth.ctypes.data, unix.ctypes.data) == e["serialised_len"]
        assert int(a["id"]) == e["id"]
        assert lib.oracle_auth_associated_data_len(auth.ctypes.data, unix.ctypes.data) == \
            e["associated_data_len"]
        assert L.KIND_NAME[L.kind_of(a["kind_len"])] == e["kind"]
        if "uid" in e:
            assert int(unix[0]["uid"]) == e["uid"]
        if "machine_name" in e:
            no, nl = int(unix[0]["name_off"]), int(unix[0]["name_len"])
            assert bytes(b[no:no + nl]).hex() == e["machine_name"]
        if "data_len" in e:
            assert L.len_of(a["kind_len"]) == e["data_len"]
        if v.get("reserialise_equal"):
            out = np.zeros(len(buf) + 8, np.uint8)
            w = np.zeros(1, np.uint64)
            st = lib.oracle_auth_encode(auth.ctypes.data, unix.ctypes.data, b.ctypes.data, out.ctypes.data,
                                        len(out), w.ctypes.data)
            assert st == 0 and bytes(out[:int(w[0])]) == buf, v["name"]


@pytest.mark.parametrize("mode", ["slice", "bytes"])
def test_reference_unix_params(oracle, golden, mode):
    lib = oracle.load()
    for v in golden["unix_params"]:
        buf = bytes.fromhex(v["hex"])
        b = np.frombuffer(buf + b"\0" * 8, np.uint8).copy()
        u = np.zeros(1, L.UNIX_DTYPE)
        consumed = np.zeros(1, np.uint64)
        st = lib.oracle_unix_params_decode(b.ctypes.data, len(buf), MODES[mode], v["expected_len"],
                                           u.ctypes.data, consumed.ctypes.data)
        assert st == 0, v["name"]
        e = v["expect"]
        ng = int(u[0]["ngids"])
        got = {"stamp": int(u[0]["stamp"]), "uid": int(u[0]["uid"]), "gid": int(u[0]["gid"]),
               "gids": [int(x) for x in u[0]["gids"][:ng]],
               "machine_name": bytes(b[int(u[0]["name_off"]):int(u[0]["name_off"]) + int(u[0]["name_len"])]).decode(),
               "serialised_len": int(consumed[0])}
        assert got == e, v["name"]
        # AuthUnixParams::new(...).serialise_into == want (unix_params.rs:292-337, :373-378)
        f = v["encode_from"]
        hb = L.build_batch([{"xid": 0, "type": "call", "program": 0, "program_version": 0, "procedure": 0,
                             "cred": {"kind": "unix", "stamp": f["stamp"], "machine_name": f["machine_name"].encode().hex(),
                                      "uid": f["uid"], "gid": f["gid"], "gids": f["gids"]},
                             "verf": {"kind": "none", "data": None}, "payload": ""}])
        out = np.zeros(len(buf) + 8, np.uint8)
        w = np.zeros(1, np.uint64)
        st = lib.oracle_unix_params_encode(hb.unix.ctypes.data, hb.auth_arena.ctypes.data, out.ctypes.data,
                                           len(out), w.ctypes.data)
        assert st == 0 and bytes(out[:int(w[0])]) == buf


def test_reference_opaque(oracle, golden):
    lib = oracle.load()
    for v in golden["opaque"]:
        buf = bytes.fromhex(v["hex"])
        b = np.frombuffer(buf + b"\0" * 8, np.uint8).copy()
        r = np.zeros(3, np.uint64)
        st = lib.oracle_opaque_from_wire(b.ctypes.data, len(buf), v["max_len"], r[0:].ctypes.data,
                                         r[1:].ctypes.data, r[2:].ctypes.data)
        e = v["expect"]
        assert st == e["status"], v["name"]
        if st == 0:
            body = bytes(b[int(r[0]):int(r[0]) + int(r[1])])
            assert body.hex() == e["body"] and int(r[2]) == e["consumed"]
            out = np.zeros(len(buf) + 8, np.uint8)
            w = np.zeros(1, np.uint64)
            src = np.frombuffer(body + b"\0", np.uint8).copy()
            assert lib.oracle_opaque_encode(src.ctypes.data, len(body), out.ctypes.data, len(out),
                                            w.ctypes.data) == 0
            assert bytes(out[:int(w[0])]) == buf


def test_pad_length(oracle):
    lib = oracle.load()
    assert [lib.oracle_pad_length(i) for i in range(9)] == [0, 3, 2, 1, 0, 3, 2, 1, 0]


@pytest.mark.parametrize("mode", ["slice", "bytes"])
def test_xdrlib_messages(oracle, golden, mode):
    for v in golden["xdrlib"]:
        buf = bytes.fromhex(v["hex"])
        st, msg, unix, a0, a1, b = _decoded_view(oracle, buf, MODES[mode])
        assert st == 0, (v["name"], st)
        assert L.describe(msg, unix, b) == v["expect_full"], v["name"]
        out, slen = _reserialise(oracle, msg, unix, b)
        assert out == buf and slen == len(buf), v["name"]
        # encode from the builder's descriptors too
        hb = L.build_batch([v["expect_full"]])
        st, out2, slen2 = oracle.encode_message(hb)
        assert st == 0 and out2 == buf, v["name"]


@pytest.mark.parametrize("mode", ["slice", "bytes"])
def test_derived_errors(oracle, golden, mode):
    for v in golden["derived_errors"]:
        buf = bytes.fromhex(v["hex"])
        st, msg, unix, a0, a1, b = _decoded_view(oracle, buf, MODES[mode])
        e = v["expect_by_mode"][mode]
        assert st == e["status"], (v["name"], mode, st)
        if "aux0" in e:
            assert a0 == e["aux0"], v["name"]
        if "aux1" in e:
            assert a1 == e["aux1"], v["name"]


def test_encode_panics_and_limits(oracle):
    """Panic contracts (unix_params.rs:474-496, flavor.rs:110) as statuses."""
    none = {"kind": "none", "data": None}

    def call(cred, verf=none):
        return {"xid": 1, "type": "call", "program": 1, "program_version": 1, "procedure": 1,
                "cred": cred, "verf": verf, "payload": ""}

    unix = lambda name_len, ngids: {"kind": "unix", "stamp": 42, "machine_name": "01" * name_len,  # noqa
                                    "uid": 42, "gid": 42, "gids": list(range(ngids))}
    cases = [
        (call(unix(255, 0)), 101),   # test_max_machine_name: constructs, but assoc 267 > 200 panics on serialise
        (call(unix(256, 0)), 102),   # test_long_machine_name_panic
        (call(unix(0, 17)), 103),    # test_long_gids_panic (17 gids)
        (call(unix(124, 16)), 0),    # assoc exactly 200: encodes
        (call(unix(125, 16)), 101),
        (call({"kind": "none", "data": "00" * 200}), 0),
        (call({"kind": "short", "data": "00" * 201}), 101),
        (call(none, {"kind": "unknown", "id": 9, "data": "00" * 201}), 101),
    ]
    for m, want in cases:
        hb = L.build_batch([m])
        hb.unix["gids"][:] = 0
        if m["cred"]["kind"] == "unix":
            hb.unix["ngids"][0] = len(m["cred"]["gids"])
        st, out, slen = oracle.encode_message(hb)
        assert st == want, (m["cred"], st)


def test_assoc_200_encodes_but_wire_208_fails_decode(oracle):
    """encode limit is on associated data, decode limit on wire length."""
    m = {"xid": 1, "type": "call", "program": 1, "program_version": 1, "procedure": 1,
         "cred": {"kind": "unix", "stamp": 0, "machine_name": "61" * 124, "uid": 0, "gid": 0,
                  "gids": list(range(16))},
         "verf": {"kind": "none", "data": None}, "payload": ""}
    st, out, _ = oracle.encode_message(L.build_batch([m]))
    assert st == 0
    for mode in (L.DECODE_SLICE, L.DECODE_BYTES):
        assert oracle.decode_message(out, mode)[0] == 10


def test_declared_extent_placeholder(oracle):
    """The library's placement rule for a declared AUTH_UNIX credential whose
    deferred block check fails (include/onc_rpc.h onc_auth, ABI 7), as the
    oracle restates it: the record keeps its declared extent and its header
    is a placeholder — the record mark of the extent (rpc_message.rs:156),
    then zeros — followed by its payload, so the serial
    expected_message_len loop (rpc_message.rs:343-367) frames every record
    and the placeholder decodes to InvalidRpcVersion(0). Records failing any
    other way (a verifier over 200 bytes next to the broken block, an
    undeclared broken credential, a broken AUTH_UNIX verifier of an accepted
    reply) take no bytes."""
    unix = {"kind": "unix", "stamp": 7, "machine_name": b"host".hex(), "uid": 1, "gid": 2, "gids": [3, 4, 5]}
    none = {"kind": "none"}

    def call(xid, cred, verf=none, payload=b"\x11" * 10):
        return {"xid": xid, "type": "call", "program": 100003, "program_version": 4, "procedure": 1,
                "cred": cred, "verf": verf, "payload": payload.hex()}
    msgs = [call(1, unix), call(2, unix), call(3, unix, {"kind": "short", "data": ("ab" * 201)}),
            call(4, unix), call(5, none),
            {"xid": 6, "type": "reply", "reply": "accepted", "verf": unix, "accept_status": "success",
             "payload": "22" * 5},
            call(7, none)]
    hb = L.build_batch(msgs, declare=True)
    m = hb.msgs
    ref = lambda i, f="cred": int(m[f + "_ref"][i])          # noqa: E731
    hb.unix["ngids"][ref(1)] = 17                             # broken block, declared: placeholder
    hb.unix["ngids"][ref(2)] = 17                             # broken block + verifier > 200: no bytes
    m["cred_kind_len"][3] = int(L.pack_kind_len(L.KIND_UNIX, 0))
    hb.unix["ngids"][ref(3)] = 17                             # undeclared broken block: no bytes
    hb.unix["name_len"][ref(5, "verf")] = 300                 # a reply's verifier is checked up front
    wire, off, st, ln = oracle.encode_batch(hb)
    assert list(st) == [0, 103, 103, 103, 0, 102, 0]          # the construction panic before the assert
    decl = L.unix_body_len(4, 3)
    ext = 4 + 4 + 4 + 16 + (8 + decl) + 8 + 10
    assert list(ln[[1, 2, 3, 5]]) == [ext, 0, 0, 0]
    w = np.frombuffer(wire, np.uint8)
    a = int(off[1])
    hole = w[a:a + ext].tobytes()
    assert hole[:4] == ((ext - 4) | 0x80000000).to_bytes(4, "big")
    assert hole[4:ext - 10] == bytes(ext - 14) and hole[ext - 10:] == b"\x11" * 10
    # framable: every record with an extent, in order
    fo, n, consumed, fst = oracle.frame_stream(wire)[:4]
    has = ln != 0
    assert (n, consumed, fst) == (int(has.sum()), len(wire), 0)
    assert np.array_equal(fo[:-1], off[:-1][has])
    ms, _, ss, a0, _ = oracle.decode_batch(np.frombuffer(wire + b"\0" * 16, np.uint8), fo, L.DECODE_SLICE)
    assert list(ss) == [0, 11, 0, 0] and int(a0[1]) == 0      # the placeholder: InvalidRpcVersion(0)
    assert list(ms["xid"][[0, 2, 3]]) == [1, 5, 7]


def _expected_message_len_loop(buf):
    """The caller's framing loop over a stream (rpc_message.rs:343-367),
    restated in Python: record starts until the buffer ends."""
    off, p = [0], 0
    while len(buf) - p >= 4:
        hdr = int.from_bytes(buf[p:p + 4], "big")
        assert hdr & 0x80000000, "Fragmented"
        p += (hdr & 0x7FFFFFFF) + 4
        assert p <= len(buf), "IncompleteMessage"
        off.append(p)
    assert p == len(buf)
    return off


def _placeholder_batch():
    """The descriptors of tests/golden/placeholder.json (make_placeholder.py)."""
    unix = {"kind": "unix", "stamp": 7, "machine_name": b"host".hex(), "uid": 1, "gid": 2, "gids": [3, 4, 5]}
    none = {"kind": "none"}

    def call(xid, cred, verf=none, payload=b"\x11" * 10):
        return {"xid": xid, "type": "call", "program": 100003, "program_version": 4, "procedure": 1,
                "cred": cred, "verf": verf, "payload": payload.hex()}
    msgs = [call(1, unix), call(2, unix), call(3, unix, {"kind": "short", "data": ("ab" * 201)}),
            call(4, unix), call(5, none),
            {"xid": 6, "type": "reply", "reply": "accepted", "verf": unix, "accept_status": "success",
             "payload": "22" * 5},
            call(7, none)]
    hb = L.build_batch(msgs, declare=True)
    m = hb.msgs
    ref = lambda i, f="cred": int(m[f + "_ref"][i])          # noqa: E731
    hb.unix["ngids"][ref(1)] = 17
    hb.unix["ngids"][ref(2)] = 17
    m["cred_kind_len"][3] = int(L.pack_kind_len(L.KIND_UNIX, 0))
    hb.unix["ngids"][ref(3)] = 17
    hb.unix["name_len"][ref(5, "verf")] = 300
    return hb


def placeholder_fixture():
    import json
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "placeholder.json")) as f:
        return json.load(f)


def test_placeholder_and_compaction_fixture(oracle):
    """tests/golden/placeholder.json (struct.pack, no oracle) pins the
    placeholder bytes of the batch encode (ABI 7) and the compacted stream
    (onc_compact, ABI 8): the oracle's encode and oracle_compact reproduce
    them byte for byte; a Python restatement of the caller's
    expected_message_len loop (rpc_message.rs:343-367) frames the encode's
    stream into the records with an extent and the compacted one into exactly
    the OK messages."""
    fx = placeholder_fixture()
    hb = _placeholder_batch()
    wire, off, st, _ = oracle.encode_batch(hb)
    assert list(st) == fx["status"]
    assert wire.hex() == fx["wire"]
    assert list(off) == fx["rec_off"]
    w = bytes.fromhex(fx["wire"])
    has = np.diff(np.asarray(fx["rec_off"])) != 0
    assert _expected_message_len_loop(w) == list(np.asarray(fx["rec_off"])[:-1][has]) + [len(w)]
    cw, coff = oracle.compact(wire, off, st)
    assert cw.hex() == fx["compacted"] and list(coff) == fx["compacted_rec_off"]
    c = bytes.fromhex(fx["compacted"])
    assert len(_expected_message_len_loop(c)) - 1 == int((np.asarray(fx["status"]) == 0).sum())
