"""Body-level roots (ONC_ROOT_*, include/onc_rpc.h): each reference type's own
TryFrom / serialise_into / serialised_len, not only RpcMessage's
("same for CallBody, AuthFlavor, ReplyBody, AcceptedReply,
AcceptedStatus, RejectedReply; TryFrom<Bytes> variants").

CPU tests pin the oracle's body entry points (oracle_decode_body /
oracle_encode_body) to the reference's body-level golden vectors
(flavor.rs:233-393, unix_params.rs:288-471, opaque.rs:133-191) and to the
message-level oracle, which the whole-message golden vectors pin. The GPU
tests run the same vectors, random bodies of every root and mutated bodies
through the kernels (onc_decode_body / onc_encode_body) against that
oracle, bit-exact, in both decode modes.
"""
import numpy as np
import pytest

import onc_rpc_amd.layout as L
import onc_rpc_amd.synth as S

MODES = {"slice": L.DECODE_SLICE, "bytes": L.DECODE_BYTES}
ROOTS = list(range(11))
# header words of the whole message before each root's bytes (record mark,
# xid, msg_type, ...): a root's serialisation is a substring of the message's
PREFIX = {L.ROOT_MESSAGE_TYPE: 8, L.ROOT_CALL_BODY: 12, L.ROOT_REPLY_BODY: 12, L.ROOT_ACCEPTED_REPLY: 16,
          L.ROOT_REJECTED_REPLY: 16, L.ROOT_AUTH_ERROR: 20, L.ROOT_AUTH_FLAVOR: 28}


def _params(root, recs, rng=None):
    """Per-record param: expected_len (AUTH_UNIX_PARAMS) = the record length,
    max_len (OPAQUE) = 255 (the machine-name bound) — or random ones."""
    if root == L.ROOT_AUTH_UNIX_PARAMS:
        p = np.array([len(r) for r in recs], np.uint32)
        if rng is not None:
            p = np.where(rng.random(len(p)) < 0.2, p + rng.integers(-8, 9, len(p)).astype(np.int64), p)
        return np.asarray(p, np.uint64).astype(np.uint32)
    if root == L.ROOT_OPAQUE:
        if rng is not None:
            return rng.choice(np.array([0, 3, 12, 15, 100, 200, 255, 0xFFFFFFFF], np.uint32), len(recs))
        return np.full(len(recs), 255, np.uint32)
    return None


def _records_of(oracle, root, hb):
    """The oracle's serialisation of every descriptor as `root` (records of
    failed descriptors dropped) -> list of bytes."""
    wire, off, st, _ = oracle.encode_body_batch(root, hb)
    return [wire[int(off[i]):int(off[i + 1])] for i in range(hb.n) if st[i] == 0]


def _valid_messages(n, seed, max_payload=300):
    msgs = S.random_messages(n, seed=seed, max_payload=max_payload)
    return msgs


# ----------------------------------------------------------------------------
# CPU: the oracle's body roots
# ----------------------------------------------------------------------------

@pytest.mark.parametrize("mode", ["slice", "bytes"])
def test_oracle_body_golden_auth(oracle, golden, mode):
    """AuthFlavor::try_from over the reference's five auth vectors
    (flavor.rs:233-393): the values the reference asserts."""
    for v in golden["auth"]:
        buf = bytes.fromhex(v["hex"])
        w, off = L.records_from_wire([buf])
        m, u, st, a0, a1, cons = oracle.decode_body_batch(L.ROOT_AUTH_FLAVOR, w, off, MODES[mode])
        e = v["expect"]
        assert st[0] == 0, v["name"]
        assert int(cons[0]) == e["serialised_len"] == len(buf), v["name"]
        assert int(m[0]["cred_id"]) == e["id"]
        assert L.KIND_NAME[L.kind_of(m[0]["cred_kind_len"])] == e["kind"]
        if "data_len" in e:
            assert L.len_of(m[0]["cred_kind_len"]) == e["data_len"]
        if "uid" in e:
            assert int(u[0]["uid"]) == e["uid"]
        if "machine_name" in e:
            no, nl = int(u[0]["name_off"]), int(u[0]["name_len"])
            assert bytes(w[no:no + nl]).hex() == e["machine_name"]


@pytest.mark.parametrize("mode", ["slice", "bytes"])
def test_oracle_body_golden_unix_params(oracle, golden, mode):
    for v in golden["unix_params"]:
        buf = bytes.fromhex(v["hex"])
        w, off = L.records_from_wire([buf])
        m, u, st, a0, a1, cons = oracle.decode_body_batch(L.ROOT_AUTH_UNIX_PARAMS, w, off, MODES[mode],
                                                          np.array([v["expected_len"]], np.uint32))
        e = v["expect"]
        assert st[0] == 0, v["name"]
        ng = int(u[0]["ngids"])
        got = {"stamp": int(u[0]["stamp"]), "uid": int(u[0]["uid"]), "gid": int(u[0]["gid"]),
               "gids": [int(x) for x in u[0]["gids"][:ng]],
               "machine_name": bytes(w[int(u[0]["name_off"]):int(u[0]["name_off"]) + int(u[0]["name_len"])]).decode(),
               "serialised_len": int(cons[0])}
        assert got == e, v["name"]


def test_oracle_body_golden_opaque(oracle, golden):
    for mode in MODES.values():
        for v in golden["opaque"]:
            buf = bytes.fromhex(v["hex"])
            w, off = L.records_from_wire([buf])
            m, u, st, a0, a1, cons = oracle.decode_body_batch(L.ROOT_OPAQUE, w, off, mode,
                                                              np.array([v["max_len"]], np.uint32))
            e = v["expect"]
            assert st[0] == e["status"], v["name"]
            if st[0] == 0:
                ref, ln = int(m[0]["cred_ref"]), L.len_of(m[0]["cred_kind_len"])
                assert bytes(w[ref:ref + ln]).hex() == e["body"] and int(cons[0]) == e["consumed"]


def test_oracle_body_roots_are_substrings_of_the_message(oracle):
    """Every root's serialisation is the matching piece of the whole
    message's (rpc_message.rs:136-164 calls each piece's serialise_into in
    turn), so the message-level oracle — pinned by the whole-message golden
    vectors — pins the body roots too."""
    hb = L.build_batch(_valid_messages(400, seed=7))
    mw, moff, mst, _ = oracle.encode_batch(hb)
    for root in ROOTS:
        bw, boff, bst, blen = oracle.encode_body_batch(root, hb)
        for i in range(hb.n):
            msg = mw[int(moff[i]):int(moff[i + 1])]
            body = bw[int(boff[i]):int(boff[i + 1])]
            m = hb.msgs[i]
            call = int(m["msg_type"]) == L.MSG_CALL
            acc = not call and int(m["reply_stat"]) == L.REPLY_ACCEPTED
            if bst[i] != 0:
                continue
            if root == L.ROOT_RPC_MESSAGE:
                assert body == msg
            elif root in (L.ROOT_MESSAGE_TYPE, L.ROOT_CALL_BODY, L.ROOT_REPLY_BODY, L.ROOT_ACCEPTED_REPLY,
                          L.ROOT_REJECTED_REPLY, L.ROOT_AUTH_ERROR):
                assert body == msg[PREFIX[root]:], (root, i)
            elif root == L.ROOT_ACCEPTED_STATUS:
                assert acc and msg.endswith(body)
            elif root == L.ROOT_AUTH_FLAVOR:
                assert body == msg[28:28 + len(body)], i
            elif root == L.ROOT_AUTH_UNIX_PARAMS:
                assert body == msg[36:36 + len(body)], i
            else:
                assert body == msg[32:32 + len(body)], i


def test_oracle_body_shape_checks(oracle):
    """A descriptor of another shape is BAD_DESCRIPTOR for a root."""
    hb = L.build_batch(_valid_messages(300, seed=8))
    for root in ROOTS:
        _, _, st, _ = oracle.encode_body_batch(root, hb)
        for i in range(hb.n):
            m = hb.msgs[i]
            call = int(m["msg_type"]) == L.MSG_CALL
            acc = not call and int(m["reply_stat"]) == L.REPLY_ACCEPTED
            den = not call and not acc
            ck, cl = L.kind_of(m["cred_kind_len"]), L.len_of(m["cred_kind_len"])
            ok = {L.ROOT_RPC_MESSAGE: True, L.ROOT_MESSAGE_TYPE: True, L.ROOT_CALL_BODY: call,
                  L.ROOT_REPLY_BODY: not call, L.ROOT_ACCEPTED_REPLY: acc, L.ROOT_ACCEPTED_STATUS: acc,
                  L.ROOT_REJECTED_REPLY: den, L.ROOT_AUTH_ERROR: den and int(m["stat"]) == 1,
                  L.ROOT_AUTH_FLAVOR: call, L.ROOT_AUTH_UNIX_PARAMS: call and ck == L.KIND_UNIX,
                  L.ROOT_OPAQUE: call and ck != L.KIND_UNIX and cl <= 255}[root]
            if not ok:
                assert st[i] == 104, (root, i)


# ----------------------------------------------------------------------------
# GPU: the kernels against the oracle
# ----------------------------------------------------------------------------

@pytest.fixture(scope="module")
def codec():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    import onc_rpc_amd.runtime as R
    c = R.Codec(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def R():
    import onc_rpc_amd.runtime as R
    return R


def _slots(msgs, status):
    ok = status == 0
    cred = ok & (msgs["msg_type"] == L.MSG_CALL) & ((msgs["cred_kind_len"] >> 24) == L.KIND_UNIX)
    verf = ok & ((msgs["msg_type"] == L.MSG_CALL) | (msgs["reply_stat"] == L.REPLY_ACCEPTED)) & \
        ((msgs["verf_kind_len"] >> 24) == L.KIND_UNIX)
    # onc_auth.ref: packed per 64-record group (include/onc_rpc.h onc_decoded)
    return np.sort(np.concatenate([msgs["cred_ref"][cred], msgs["verf_ref"][verf]]).astype(np.int64))


def _assert_same_decode(g, o, what):
    gm, gu, gs, ga0, ga1, gc = g
    om, ou, os_, oa0, oa1, oc = o
    bad = np.nonzero(gs != os_)[0]
    assert len(bad) == 0, f"{what}: status at {bad[:8]} gpu {gs[bad[:8]]} oracle {os_[bad[:8]]}"
    bad = np.nonzero((ga0 != oa0) | (ga1 != oa1))[0]
    assert len(bad) == 0, f"{what}: aux at {bad[:8]}"
    bad = np.nonzero(gc != oc)[0]
    assert len(bad) == 0, f"{what}: consumed at {bad[:8]} gpu {gc[bad[:8]]} oracle {oc[bad[:8]]}"
    gb, ob = gm.view(np.uint8).reshape(-1, 64), om.view(np.uint8).reshape(-1, 64)
    bad = np.nonzero((gb != ob).any(axis=1))[0]
    assert len(bad) == 0, f"{what}: descriptor at {bad[:8]}: {gm[bad[0]]} vs {om[bad[0]]}"
    idx = _slots(om, os_)
    if len(idx):
        gbu = gu.view(np.uint8).reshape(-1, 96)[idx]
        obu = ou.view(np.uint8).reshape(-1, 96)[idx]
        bad = np.nonzero((gbu != obu).any(axis=1))[0]
        assert len(bad) == 0, f"{what}: unix slot at {idx[bad[:8]]}"


def _decode_both(R, codec, oracle, root, recs, mode, param):
    w, off = L.records_from_wire(recs)
    g = R.decode_body_host_wire(codec, root, w, off, mode, param)
    o = oracle.decode_body_batch(root, w, off, mode, param)
    return w, off, g, o


def _reencode_from_decoded(R, codec, root, w, dec):
    """onc_encode_body of decoded descriptors (arenas = the wire)."""
    m, u, st, _, _, _ = dec
    keep = np.nonzero(st == 0)[0]
    hb = L.HostBatch(m[keep].copy(), u.copy() if len(u) else np.zeros(1, L.UNIX_DTYPE), w, w)
    # unix refs stay the decoder's slot indices (onc_auth.ref into the slot table)
    return R.encode_body_host_batch(codec, root, hb), keep


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["slice", "bytes"])
def test_gpu_body_golden_vectors(codec, R, oracle, golden, mode):
    """The reference's ten body-level vectors through the kernels: 5 AuthFlavor
    (flavor.rs:233-393), 2 AuthUnixParams (unix_params.rs:288-471), 3 Opaque
    (opaque.rs:133-191) — decoded fields as the reference asserts them, equal
    to the oracle, serialised_len (consumed), and re-encode byte-equal where
    the reference asserts it."""
    md = MODES[mode]
    # AuthFlavor
    recs = [bytes.fromhex(v["hex"]) for v in golden["auth"]]
    w, off, g, o = _decode_both(R, codec, oracle, L.ROOT_AUTH_FLAVOR, recs, md, None)
    _assert_same_decode(g, o, "auth vectors")
    gm, gu, gs, _, _, gc = g
    for i, v in enumerate(golden["auth"]):
        e = v["expect"]
        assert gs[i] == 0 and int(gc[i]) == e["serialised_len"], v["name"]
        assert int(gm[i]["cred_id"]) == e["id"] and L.KIND_NAME[L.kind_of(gm[i]["cred_kind_len"])] == e["kind"]
        if "data_len" in e:
            assert L.len_of(gm[i]["cred_kind_len"]) == e["data_len"]
        if "uid" in e:
            assert int(gu[int(gm[i]["cred_ref"])]["uid"]) == e["uid"]
        if "machine_name" in e:
            u = gu[int(gm[i]["cred_ref"])]
            no, nl = int(u["name_off"]), int(u["name_len"])
            assert bytes(w[no:no + nl]).hex() == e["machine_name"]
    (bw, boff, bst, blen), keep = _reencode_from_decoded(R, codec, L.ROOT_AUTH_FLAVOR, w, g)
    assert (bst == 0).all()
    for j, i in enumerate(keep):
        assert int(blen[j]) == golden["auth"][i]["expect"]["serialised_len"]
        if golden["auth"][i].get("reserialise_equal"):
            assert bw[int(boff[j]):int(boff[j + 1])] == recs[i], golden["auth"][i]["name"]
    # AuthUnixParams (expected_len = the reference's asserted length)
    recs = [bytes.fromhex(v["hex"]) for v in golden["unix_params"]]
    prm = np.array([v["expected_len"] for v in golden["unix_params"]], np.uint32)
    w, off, g, o = _decode_both(R, codec, oracle, L.ROOT_AUTH_UNIX_PARAMS, recs, md, prm)
    _assert_same_decode(g, o, "unix_params vectors")
    gm, gu, gs, _, _, gc = g
    for i, v in enumerate(golden["unix_params"]):
        e, u = v["expect"], gu[int(gm[i]["cred_ref"])]
        ng = int(u["ngids"])
        got = {"stamp": int(u["stamp"]), "uid": int(u["uid"]), "gid": int(u["gid"]),
               "gids": [int(x) for x in u["gids"][:ng]],
               "machine_name": bytes(w[int(u["name_off"]):int(u["name_off"]) + int(u["name_len"])]).decode(),
               "serialised_len": int(gc[i])}
        assert gs[i] == 0 and got == e, v["name"]
    (bw, boff, bst, blen), keep = _reencode_from_decoded(R, codec, L.ROOT_AUTH_UNIX_PARAMS, w, g)
    assert (bst == 0).all() and [bw[int(boff[j]):int(boff[j + 1])] for j in range(len(keep))] == recs
    # the unix_params vectors are also AuthUnixParams::new(...).serialise_into targets (unix_params.rs:292-337)
    built = L.build_batch([{"xid": 0, "type": "call", "program": 0, "program_version": 0, "procedure": 0,
                            "cred": dict(v["encode_from"], kind="unix",
                                         machine_name=v["encode_from"]["machine_name"].encode().hex()),
                            "verf": {"kind": "none", "data": None}, "payload": ""}
                           for v in golden["unix_params"]])
    bw, boff, bst, _ = R.encode_body_host_batch(codec, L.ROOT_AUTH_UNIX_PARAMS, built)
    assert (bst == 0).all() and [bw[int(boff[j]):int(boff[j + 1])] for j in range(len(recs))] == recs
    # Opaque (max_len = the reference test's 100)
    recs = [bytes.fromhex(v["hex"]) for v in golden["opaque"]]
    prm = np.array([v["max_len"] for v in golden["opaque"]], np.uint32)
    w, off, g, o = _decode_both(R, codec, oracle, L.ROOT_OPAQUE, recs, md, prm)
    _assert_same_decode(g, o, "opaque vectors")
    gm, gu, gs, _, _, gc = g
    for i, v in enumerate(golden["opaque"]):
        e = v["expect"]
        assert gs[i] == e["status"], v["name"]
        if e["status"] == 0:
            ref, ln = int(gm[i]["cred_ref"]), L.len_of(gm[i]["cred_kind_len"])
            assert bytes(w[ref:ref + ln]).hex() == e["body"] and int(gc[i]) == e["consumed"]
    (bw, boff, bst, blen), keep = _reencode_from_decoded(R, codec, L.ROOT_OPAQUE, w, g)
    assert (bst == 0).all()
    for j, i in enumerate(keep):
        if golden["opaque"][i].get("reserialise_equal"):
            assert bw[int(boff[j]):int(boff[j + 1])] == recs[i], golden["opaque"][i]["name"]


@pytest.mark.gpu
@pytest.mark.parametrize("root", ROOTS)
def test_gpu_body_encode_matches_oracle(codec, R, oracle, root):
    """onc_encode_body of random messages (every shape, so every root also
    sees descriptors it must refuse) == the oracle: bytes, offsets, statuses."""
    hb = L.build_batch(_valid_messages(3000, seed=100 + root))
    g = R.encode_body_host_batch(codec, root, hb)
    o = oracle.encode_body_batch(root, hb)
    assert np.array_equal(g[2], o[2]), L.ROOT_NAMES[root]
    assert np.array_equal(g[3], o[3]) and np.array_equal(g[1], o[1])
    assert g[0] == o[0], L.ROOT_NAMES[root]
    assert (g[2] == 0).any()


@pytest.mark.gpu
@pytest.mark.parametrize("root", ROOTS)
def test_gpu_body_decode_random_and_round_trip(codec, R, oracle, root):
    """Records of every root (the oracle's serialisations of random messages)
    decoded on the GPU in both modes == the oracle; re-encoding the decoded
    descriptors gives the records back (serialise(try_from(buf)) == buf)."""
    hb = L.build_batch(_valid_messages(2500, seed=200 + root))
    recs = _records_of(oracle, root, hb)
    assert len(recs) > 50
    for mode in MODES.values():
        w, off, g, o = _decode_both(R, codec, oracle, root, recs, mode, _params(root, recs))
        _assert_same_decode(g, o, f"{L.ROOT_NAMES[root]} mode {mode}")
        assert (g[2] == 0).all(), L.ROOT_NAMES[root]
        (bw, boff, bst, _), keep = _reencode_from_decoded(R, codec, root, w, g)
        assert (bst == 0).all() and bw == b"".join(recs), L.ROOT_NAMES[root]


def _mutants(recs, rng):
    out = []
    for r in recs:
        b = bytearray(r)
        k = rng.integers(0, 5)
        if k == 0 and len(b):
            b = b[:int(rng.integers(0, len(b)))]                       # short
        elif k == 1 and len(b) >= 4:
            p = 4 * int(rng.integers(0, len(b) // 4))
            b[p:p + 4] = int(rng.choice([0, 1, 2, 3, 7, 8, 16, 17, 200, 201, 255, 256, 0xFFFFFFFF])).to_bytes(4, "big")
        elif k == 2:
            b += rng.bytes(int(rng.integers(1, 12)))                     # trailing bytes (ignored by bodies)
        elif k == 3 and len(b):
            p = int(rng.integers(0, len(b)))
            b[p] ^= 1 << int(rng.integers(0, 8))
        out.append(bytes(b))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("root", ROOTS)
def test_gpu_body_decode_mutants_first_error(codec, R, oracle, root):
    """Truncated, word-replaced, bit-flipped and over-long records of every
    root: the first error (status, aux) and every value == the oracle, in both
    modes, with random expected_len / max_len params."""
    rng = np.random.default_rng(300 + root)
    hb = L.build_batch(_valid_messages(2000, seed=300 + root))
    recs = _mutants(_records_of(oracle, root, hb), rng)
    for mode in MODES.values():
        w, off, g, o = _decode_both(R, codec, oracle, root, recs, mode, _params(root, recs, rng))
        _assert_same_decode(g, o, f"{L.ROOT_NAMES[root]} mutants mode {mode}")
        assert (g[2] != 0).any()


@pytest.mark.gpu
def test_gpu_body_decode_requires_param(codec, R):
    import torch
    b = R.DecodeBuffers(1)
    w = torch.zeros(16, dtype=torch.uint8, device="cuda")
    off = torch.tensor([0, 8], dtype=torch.int64, device="cuda")
    for root, mode in [(L.ROOT_OPAQUE, L.DECODE_SLICE), (L.ROOT_OPAQUE, L.DECODE_BYTES),
                       (L.ROOT_AUTH_UNIX_PARAMS, L.DECODE_SLICE)]:
        with pytest.raises(R.CodecError):
            codec.decode_body(root, w, off, 1, mode, b.msgs, b.unix, b.status, b.aux0, b.aux1)
    with pytest.raises(R.CodecError):
        codec.decode_body(11, w, off, 1, 0, b.msgs, b.unix, b.status, b.aux0, b.aux1)
    # AuthUnixParams::try_from(Bytes) takes no length
    codec.decode_body(L.ROOT_AUTH_UNIX_PARAMS, w, off, 1, L.DECODE_BYTES, b.msgs, b.unix, b.status, b.aux0, b.aux1)
    codec.sync()


@pytest.mark.gpu
@pytest.mark.parametrize("root", [L.ROOT_ACCEPTED_STATUS, L.ROOT_ACCEPTED_REPLY, L.ROOT_REPLY_BODY,
                                  L.ROOT_MESSAGE_TYPE, L.ROOT_AUTH_ERROR])
def test_gpu_body_short_headers_every_alignment(codec, R, oracle, root):
    """Roots whose header is shorter than a 16-byte chunk (AcceptedStatus: 4
    bytes, AcceptedReply with AuthNone: 12) put payload bytes into the chunk
    the record starts in, which the record before owns: every record start
    offset 0..15 and payload lengths 0..48 (and some long ones), bit-exact."""
    msgs = []
    rng = np.random.default_rng(root)
    for i in range(1200):
        if i % 11 == 3:
            msgs.append({"xid": i, "type": "reply", "reply": "denied", "rejected": "auth_error", "auth_error": i % 8})
            continue
        plen = int(i % 49) if i % 7 else int(rng.integers(49, 700))
        msgs.append({"xid": i, "type": "reply", "reply": "accepted",
                     "verf": {"kind": "none", "data": None} if i % 5 else {"kind": "short", "data": "ab" * (i % 9)},
                     "accept_status": "success" if i % 13 else "prog_mismatch", "low": 1, "high": 2,
                     "payload": rng.bytes(plen).hex()})
    hb = L.build_batch(msgs)
    for shift in (0, 1, 2, 3, 5, 13):
        # `shift` bytes of writer position change every record's chunk offset
        import torch
        o_wire, o_off, o_st, o_len = oracle.encode_body_batch(root, hb)
        db = R.DeviceBatch.from_host(hb)
        total = len(o_wire)
        buf = torch.full((total + shift + 48,), 0xA5, dtype=torch.uint8, device="cuda")
        off = torch.empty(hb.n + 1, dtype=torch.int64, device="cuda")
        st = torch.empty(hb.n, dtype=torch.int32, device="cuda")
        codec.encode_body(root, db, buf[shift:], off, st, out_cap=total)
        codec.sync()
        b = buf.cpu().numpy()
        assert np.array_equal(st.cpu().numpy(), o_st)
        assert np.array_equal(off.cpu().numpy().view(np.uint64), o_off)
        assert b[shift:shift + total].tobytes() == o_wire, (L.ROOT_NAMES[root], shift)
        assert (b[:shift] == 0xA5).all() and (b[shift + total:] == 0xA5).all()


def _too_long_batch():
    """CallBody / RpcMessage records around the 2^31 limit: a Call with
    AuthNone(None) credential and verifier has a 32-byte CallBody header
    (call_body.rs:111-119) and a 44-byte RpcMessage (+ mark, xid, type);
    payload lengths put each root's total at 2^31 - 1 and 2^31. Lengths only:
    the payload is never read (a 16-byte arena declared as 4 GiB)."""
    msgs = np.zeros(4, L.MSG_DTYPE)
    msgs["msg_type"] = L.MSG_CALL
    msgs["payload_len"] = [(1 << 31) - 33, (1 << 31) - 32, (1 << 31) - 45, (1 << 31) - 44]
    return L.HostBatch(msgs, np.zeros(1, L.UNIX_DTYPE), np.zeros(16, np.uint8), np.zeros(16, np.uint8))


def test_oracle_too_long_boundary(oracle):
    """The 2^31 limit at its boundary. RpcMessage::serialise_into refuses a
    record of 2^31 bytes or more (rpc_message.rs:146-151: the record mark's
    length field). The body roots apply the same limit: a deliberate
    deviation — the reference's CallBody::serialise_into has no
    limit and its serialised_len is a u32 — so that any body also frames as a
    message; parity unpinned, no reference test covers it."""
    import ctypes as C
    hb = _too_long_batch()
    lib = oracle.load()
    for root, ok, bad in ((L.ROOT_CALL_BODY, 0, 1), (L.ROOT_RPC_MESSAGE, 2, 3)):
        off = np.zeros(5, np.uint64)
        st = np.zeros(4, np.int32)
        ln = np.zeros(4, np.uint32)
        lib.oracle_encode_body_batch(root, 4, C.c_void_p(hb.msgs.ctypes.data), C.c_void_p(hb.unix.ctypes.data),
                                     C.c_void_p(hb.auth_arena.ctypes.data), C.c_void_p(hb.payload_arena.ctypes.data),
                                     None, 0, C.c_void_p(off.ctypes.data), C.c_void_p(st.ctypes.data),
                                     C.c_void_p(ln.ctypes.data))
        assert st[ok] == 105 and ln[ok] == (1 << 31) - 1          # fits (WRITE_ZERO: no capacity given)
        assert st[bad] == 100 and ln[bad] == 0                    # ONC_ENC_TOO_LONG


@pytest.mark.gpu
def test_gpu_too_long_boundary(codec, R):
    """onc_encode_body_lengths / onc_encode_lengths at the same boundary as
    the oracle test: 2^31 - 1 fits, 2^31 is ONC_ENC_TOO_LONG, for the
    CallBody root and for RpcMessage."""
    import torch
    hb = _too_long_batch()
    db = R.DeviceBatch.from_host(hb)
    db.payload_len = 1 << 32
    rl = torch.empty(4, dtype=torch.int32, device="cuda")
    st = torch.empty(4, dtype=torch.int32, device="cuda")
    for root, ok, bad in ((L.ROOT_CALL_BODY, 0, 1), (L.ROOT_RPC_MESSAGE, 2, 3)):
        codec.encode_body_lengths(root, db, rl, st)
        codec.sync()
        s, n = st.cpu().numpy(), rl.cpu().numpy().view(np.uint32)
        assert s[ok] == 0 and n[ok] == (1 << 31) - 1
        assert s[bad] == 100 and n[bad] == 0
