"""GPU parity: the gfx950 kernels (through the C ABI) against the CPU oracle,
the reference's golden vectors and round-trip invariants.

Bit-exact for everything (integer/byte work): wire bytes, record offsets,
per-record status + aux, decoded descriptors and AUTH_UNIX slots.
"""
import numpy as np
import pytest

import onc_rpc_amd.layout as L
import onc_rpc_amd.synth as S

pytestmark = pytest.mark.gpu

MODES = [L.DECODE_SLICE, L.DECODE_BYTES]


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


def unix_slots_used(msgs, status):
    """Indices of the AUTH_UNIX slots defined for OK records (onc_auth.ref;
    packed per 64-record group, include/onc_rpc.h onc_decoded)."""
    ok = status == 0
    cred = ok & (msgs["msg_type"] == L.MSG_CALL) & ((msgs["cred_kind_len"] >> 24) == L.KIND_UNIX)
    verf = ok & ((msgs["msg_type"] == L.MSG_CALL) | (msgs["reply_stat"] == L.REPLY_ACCEPTED)) & \
        ((msgs["verf_kind_len"] >> 24) == L.KIND_UNIX)
    idx = np.concatenate([msgs["cred_ref"][cred], msgs["verf_ref"][verf]]).astype(np.int64)
    return np.sort(idx)


def assert_decoded_equal(gpu, ora, what=""):
    gm, gu, gs, ga0, ga1 = gpu
    om, ou, os_, oa0, oa1 = ora
    bad = np.nonzero(gs != os_)[0]
    assert len(bad) == 0, f"{what} status mismatch at {bad[:10]}: gpu {gs[bad[:10]]} oracle {os_[bad[:10]]}"
    bad = np.nonzero((ga0 != oa0) | (ga1 != oa1))[0]
    assert len(bad) == 0, f"{what} aux mismatch at {bad[:10]}"
    gb = gm.view(np.uint8).reshape(-1, 64)
    ob = om.view(np.uint8).reshape(-1, 64)
    bad = np.nonzero((gb != ob).any(axis=1))[0]
    assert len(bad) == 0, f"{what} descriptor mismatch at {bad[:10]}: {gm[bad[0]]} vs {om[bad[0]]}"
    idx = unix_slots_used(om, os_)
    if len(idx):
        gbu = gu.view(np.uint8).reshape(-1, 96)[idx]
        obu = ou.view(np.uint8).reshape(-1, 96)[idx]
        bad = np.nonzero((gbu != obu).any(axis=1))[0]
        assert len(bad) == 0, f"{what} unix slot mismatch at {idx[bad[:10]]}"


def gpu_vs_oracle_encode(R, codec, oracle, hb, out_cap=None):
    g_wire, g_off, g_st, g_len = R.encode_host_batch(codec, hb, out_cap=out_cap)
    o_wire, o_off, o_st, o_len = oracle.encode_batch(hb, out_cap=out_cap)
    assert np.array_equal(g_st, o_st), f"status {np.nonzero(g_st != o_st)[0][:10]}"
    assert np.array_equal(g_off, o_off), f"rec_off {np.nonzero(g_off != o_off)[0][:10]}"
    assert np.array_equal(g_len, o_len)
    if g_wire != o_wire:
        a = np.frombuffer(g_wire, np.uint8)
        b = np.frombuffer(o_wire, np.uint8)
        n = min(len(a), len(b))
        first = int(np.nonzero(a[:n] != b[:n])[0][0]) if (a[:n] != b[:n]).any() else n
        rec = int(np.searchsorted(o_off, first, side="right") - 1)
        raise AssertionError(f"wire differs first at byte {first} (record {rec}); len {len(a)} vs {len(b)}")
    return o_wire, o_off, o_st


def all_golden_records(golden):
    recs, names = [], []
    for sect in ("messages", "errors", "xdrlib", "derived_errors"):
        for v in golden[sect]:
            recs.append(bytes.fromhex(v["hex"]))
            names.append((sect, v))
    return recs, names


# ---------------------------------------------------------------------------
def test_golden_decode_both_modes(codec, R, oracle, golden):
    recs, names = all_golden_records(golden)
    # each record in a batch twice: at an aligned and a misaligned start
    recs = recs + [r for r in recs]
    wire, off = L.records_from_wire(recs)
    for mode in MODES:
        g = R.decode_host_wire(codec, wire, off, mode)
        o = oracle.decode_batch(wire, off, mode)
        assert_decoded_equal(g, o, f"mode {mode}")
        gm, gu, gs, ga0, ga1 = g
        mode_name = "bytes" if mode == L.DECODE_BYTES else "slice"
        for i, (sect, v) in enumerate(names):
            if sect in ("messages", "xdrlib"):
                assert gs[i] == 0, v["name"]
            elif sect == "errors":
                assert gs[i] == v["expect"]["status"], v["name"]
                if "aux0" in v["expect"]:
                    assert (ga0[i], ga1[i]) == (v["expect"]["aux0"], v["expect"]["aux1"])
            else:
                e = v["expect_by_mode"][mode_name]
                assert gs[i] == e["status"], (v["name"], mode_name, gs[i])
                if "aux0" in e:
                    assert ga0[i] == e["aux0"]
            if sect == "xdrlib":
                assert L.describe(gm[i], gu, wire) == v["expect_full"], v["name"]


def test_golden_reencode_from_decoded(codec, R, oracle, golden):
    """serialise(try_from(buf)) == buf on the GPU for every golden message
    (rpc_message.rs:578-579, :826-827, :877-878; fuzz parse_serialise)."""
    recs = [bytes.fromhex(v["hex"]) for s in ("messages", "xdrlib") for v in golden[s]]
    wire, off = L.records_from_wire(recs)
    gm, gu, gs, _, _ = R.decode_host_wire(codec, wire, off, L.DECODE_SLICE)
    assert (gs == 0).all()
    hb = L.HostBatch(gm.copy(), gu.copy(), wire, wire)
    g_wire, g_off, g_st, _ = R.encode_host_batch(codec, hb)
    assert (g_st == 0).all()
    assert np.array_equal(g_off, off)
    assert g_wire == b"".join(recs)


def test_golden_encode_from_builder(codec, R, oracle, golden):
    msgs = [v["expect_full"] for v in golden["xdrlib"]]
    hb = L.build_batch(msgs)
    wire, off, st = gpu_vs_oracle_encode(R, codec, oracle, hb)
    assert wire == b"".join(bytes.fromhex(v["hex"]) for v in golden["xdrlib"])


@pytest.mark.parametrize("gen", ["call_none", "call_unix16", "cpu_roundtrip", "mixed", "mixed_exotic"])
def test_encode_configs_bit_exact(codec, R, oracle, gen):
    hb = {"call_none": lambda: S.call_none(5000, 256),
          "call_unix16": lambda: S.call_unix16(3000, 1024),
          "cpu_roundtrip": lambda: S.cpu_roundtrip(2000),
          "mixed": lambda: S.mixed(4000, seed=5),
          "mixed_exotic": lambda: S.mixed(4000, seed=6, pmin=0, pmax=300, exotic=0.3)}[gen]()
    wire, off, st = gpu_vs_oracle_encode(R, codec, oracle, hb)
    assert (st == 0).all()
    # and decode the result back on the GPU, both modes, against the oracle
    w = np.frombuffer(wire + b"\0" * 16, np.uint8).copy()
    for mode in MODES:
        g = R.decode_host_wire(codec, w, off, mode)
        o = oracle.decode_batch(w, off, mode)
        assert_decoded_equal(g, o, gen)
        assert (g[2] == 0).all()


@pytest.mark.parametrize("seed", [11, 12])
def test_random_messages_round_trip(codec, R, oracle, seed):
    """prop_round_trip (rpc_message.rs:1128-1154) over the reference's
    strategies: serialise == oracle, serialised_len == bytes written,
    expected_message_len == len, and decode -> describe == original."""
    ms = S.random_messages(1500, seed=seed)
    hb = L.build_batch(ms)
    wire, off, st = gpu_vs_oracle_encode(R, codec, oracle, hb)
    assert (st == 0).all()
    w = np.frombuffer(wire + b"\0" * 16, np.uint8).copy()
    lens = np.diff(off)
    hdr = w[off[:-1, None].astype(np.int64) + np.arange(4)[None, :]]
    explen = ((hdr[:, 0].astype(np.uint64) & 0x7F) << 24 | hdr[:, 1].astype(np.uint64) << 16 |
              hdr[:, 2].astype(np.uint64) << 8 | hdr[:, 3].astype(np.uint64)) + 4
    assert np.array_equal(explen, lens)
    for mode in MODES:
        g = R.decode_host_wire(codec, w, off, mode)
        assert_decoded_equal(g, oracle.decode_batch(w, off, mode))
        gm, gu, gs, _, _ = g
        assert (gs == 0).all()
        for i in range(len(ms)):
            want = dict(ms[i])
            for k in ("cred", "verf"):
                if k in want and want[k]["kind"] == "none" and not want[k]["data"]:
                    want[k] = {"kind": "none", "data": None}
            got = L.describe(gm[i], gu, w)
            assert got == want, i


@pytest.mark.parametrize("mode", MODES)
def test_corrupted_records_first_error(codec, R, oracle, mode):
    """Fuzz-style mutated records: first-error parity (status + aux)."""
    hb = L.build_batch(S.random_messages(1200, seed=21, max_payload=64))
    wire, off, _ = oracle.encode_batch(hb)[:3]
    w = np.frombuffer(wire + b"\0" * 16, np.uint8).copy()
    cw, coff = S.corrupt(w, off, frac=0.6, seed=int(mode) + 3)
    g = R.decode_host_wire(codec, cw, coff, mode)
    o = oracle.decode_batch(cw, coff, mode)
    assert_decoded_equal(g, o, "corrupt")
    assert (o[2] != 0).sum() > 200


def test_slice_vs_bytes_fuzz_invariant(codec, R, oracle):
    """fuzz/fuzz_targets/bytes.rs: slice and Bytes decoders agree on Ok/Err and
    the successful decodes re-serialise identically."""
    hb = L.build_batch(S.random_messages(800, seed=31, max_payload=40))
    wire, off, _ = oracle.encode_batch(hb)[:3]
    w = np.frombuffer(wire + b"\0" * 16, np.uint8).copy()
    cw, coff = S.corrupt(w, off, frac=0.7, seed=9)
    gs = R.decode_host_wire(codec, cw, coff, L.DECODE_SLICE)
    gb = R.decode_host_wire(codec, cw, coff, L.DECODE_BYTES)
    assert np.array_equal(gs[2] == 0, gb[2] == 0)
    ok = np.nonzero(gs[2] == 0)[0]
    a = R.encode_host_batch(codec, L.HostBatch(gs[0][ok].copy(), gs[1], cw, cw))[0]
    b = R.encode_host_batch(codec, L.HostBatch(gb[0][ok].copy(), gb[1], cw, cw))[0]
    assert a == b


def test_encode_panic_statuses(codec, R, oracle):
    none = {"kind": "none", "data": None}

    def call(cred, verf=none):
        return {"xid": 1, "type": "call", "program": 1, "program_version": 1, "procedure": 1,
                "cred": cred, "verf": verf, "payload": "ab"}

    def unix(nl, ng):
        return {"kind": "unix", "stamp": 42, "machine_name": "01" * nl, "uid": 42, "gid": 42, "gids": list(range(ng))}

    ms = [call(unix(255, 0)), call(unix(256, 0)), call(unix(0, 16)), call(unix(124, 16)),
          call(unix(125, 16)), call({"kind": "short", "data": "00" * 201}),
          call(none, {"kind": "unknown", "id": 7, "data": "11" * 201}), call(none)]
    hb = L.build_batch(ms)
    hb.unix["ngids"][2] = 17          # Gids::from_iter panic (> 16), unix_params.rs:47
    hb.msgs["msg_type"][7] = 5        # unrepresentable descriptor
    wire, off, st = gpu_vs_oracle_encode(R, codec, oracle, hb)
    assert list(st) == [101, 102, 103, 0, 101, 101, 101, 104]


def test_write_zero_capacity(codec, R, oracle):
    hb = S.mixed(700, seed=8, pmin=0, pmax=200)
    total = int(oracle.encode_batch(hb)[1][-1])
    for cap in (0, 37, total // 3, total - 1, total):
        gpu_vs_oracle_encode(R, codec, oracle, hb, out_cap=cap)


@pytest.mark.parametrize("plen", [1023, 1021, 1022])
def test_byte_path_with_spans(codec, R, oracle, plen):
    """AUTH_UNIX (16 gids) headers + odd payloads: every tile takes enc_emit's
    byte path and is cut into several LDS spans."""
    hb = S.call_unix16(700, plen)
    gpu_vs_oracle_encode(R, codec, oracle, hb)
    total = int(oracle.encode_batch(hb)[1][-1])
    for cap in (total // 2 + 7, total - 3):
        gpu_vs_oracle_encode(R, codec, oracle, hb, out_cap=cap)


def test_small_payload_lengths(codec, R, oracle):
    """Payloads of 0..40 bytes (those under 16 live in the LDS image), at every
    record alignment, mixed with AUTH_NONE and AUTH_UNIX headers."""
    msgs = []
    rng = np.random.default_rng(5)
    for i in range(1500):
        m = S.random_messages(1, seed=1000 + i, max_payload=1)[0]
        msgs.append(m)
    hb = L.build_batch(msgs)
    pl = rng.integers(0, 41, len(hb.msgs)).astype(np.uint32)
    is_pay = (hb.msgs["msg_type"] == L.MSG_CALL) | \
        ((hb.msgs["reply_stat"] == L.REPLY_ACCEPTED) & (hb.msgs["stat"] == 0))
    pay = rng.integers(0, 256, int(pl.sum()) + 64, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(pl)[:-1]]).astype(np.uint64)
    msgs2 = hb.msgs.copy()
    msgs2["payload_len"] = np.where(is_pay, pl, msgs2["payload_len"])
    msgs2["payload_off"] = np.where(is_pay, offs, msgs2["payload_off"])
    gpu_vs_oracle_encode(R, codec, oracle, L.HostBatch(msgs2, hb.unix, hb.auth_arena, pay))


def test_unaligned_arenas(codec, R, oracle):
    """Payload/auth bodies at every byte alignment in the arenas."""
    base = L.build_batch(S.random_messages(600, seed=41, max_payload=70))
    for shift in (1, 2, 3):
        pay = np.concatenate([np.zeros(shift, np.uint8), base.payload_arena])
        auth = np.concatenate([np.zeros(4 - shift, np.uint8), base.auth_arena])
        msgs = base.msgs.copy()
        unix = base.unix.copy()
        msgs["payload_off"] += shift
        for f in ("cred", "verf"):
            opaque = (msgs[f + "_kind_len"] >> 24) != L.KIND_UNIX
            msgs[f + "_ref"][opaque] += 4 - shift
        unix["name_off"] += 4 - shift
        gpu_vs_oracle_encode(R, codec, oracle, L.HostBatch(msgs, unix, auth, pay))


def test_empty_and_single(codec, R, oracle):
    import torch
    hb = S.call_none(1, 0)
    gpu_vs_oracle_encode(R, codec, oracle, hb)
    db = R.DeviceBatch(0, *(torch.zeros(16, dtype=torch.uint8, device="cuda") for _ in range(4)))
    out = torch.zeros(16, dtype=torch.uint8, device="cuda")
    rec_off = torch.full((1,), 7, dtype=torch.int64, device="cuda")
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    codec.encode(db, out, rec_off, st)
    codec.sync()
    assert int(rec_off[0]) == 0
    # decode of zero records is a no-op
    bufs = R.DecodeBuffers(0)
    codec.decode(out, rec_off, 0, 0, bufs.msgs, bufs.unix, bufs.status, bufs.aux0, bufs.aux1)
    codec.sync()


def test_scan_lengths(codec, R):
    import torch
    rng = np.random.default_rng(3)
    for n in (1, 255, 256, 257, 100000):
        lens = rng.integers(0, 5000, n).astype(np.uint32)
        d = torch.from_numpy(lens.view(np.int32).copy()).cuda()
        off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        codec.scan_lengths(d, n, 12345, off)
        codec.sync()
        want = np.concatenate([[0], np.cumsum(lens.astype(np.uint64))]) + 12345
        assert np.array_equal(off.cpu().numpy().view(np.uint64), want)


def test_full_size_config1_loopback(codec, R, oracle):
    """configs[1] at full size (1M x 256 B): encode -> decode on the GPU with
    size-independent checks (all OK, xids, offsets, payload bytes, lengths),
    plus a bit-exact oracle comparison of a 20k-record window."""
    import torch
    n = 1_000_000
    hb = S.call_none(n, 256)
    db = R.DeviceBatch.from_host(hb)
    out = torch.empty(n * 300 + 16, dtype=torch.uint8, device="cuda")
    rec_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    codec.encode(db, out, rec_off, st)
    bufs = R.DecodeBuffers(n)
    codec.decode(out, rec_off, n, L.DECODE_SLICE, bufs.msgs, bufs.unix, bufs.status, bufs.aux0, bufs.aux1)
    codec.sync()
    assert int((st != 0).sum()) == 0
    assert torch.equal(rec_off, torch.arange(n + 1, device="cuda", dtype=torch.int64) * 300)
    assert int((bufs.status != 0).sum()) == 0
    dm = bufs.msgs.view(-1, 64)
    xid = dm[:, 0:4].contiguous().view(torch.int32).view(-1)
    assert torch.equal(xid, torch.arange(n, device="cuda", dtype=torch.int32))
    # payload bytes of every record == payload arena (gather by offsets)
    wire_payload = out[: n * 300].view(n, 300)[:, 44:]
    assert torch.equal(wire_payload.reshape(-1), db.payload_arena[: n * 256])
    # bit-exact window vs the oracle
    lo, hi = 500_000, 520_000
    sub = L.HostBatch(hb.msgs[lo:hi].copy(), hb.unix, hb.auth_arena, hb.payload_arena)
    o_wire = oracle.encode_batch(sub)[0]
    assert out[lo * 300:hi * 300].cpu().numpy().tobytes() == o_wire


@pytest.mark.parametrize("cfg", ["c2", "c3"])
def test_full_size_loopback_idempotent(codec, R, oracle, cfg):
    """configs[2] (1M mixed Call/Reply, payloads 64..4096 B) and configs[3]
    (4M Call(AuthUnix 16 gids) + 1 KiB) at full size, with size-independent
    properties: encode OK and offsets = prefix sum of serialised_len; both
    decode modes OK with the input xids; serialise(try_from(buf)) == buf over
    the whole buffer (rpc_message.rs:1150-1153, fuzz parse_serialise.rs:5-12),
    re-encoding straight from the decoded descriptors (arenas = the wire);
    plus a 20k-record window bit-exact vs the oracle (encode and decode)."""
    import torch
    if cfg == "c2":
        n, hb = 1_000_000, S.mixed(1_000_000, seed=2)
    else:
        n, hb = 4_000_000, S.call_unix16(4_000_000, 1024, seed=3)
    db = R.DeviceBatch.from_host(hb)
    rec_len = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    codec.encode_lengths(db, rec_len, st)
    codec.sync()
    lens = rec_len.to(torch.int64)
    total = int(lens.sum())
    if cfg == "c3":
        assert torch.all(lens == 1152)
    out = torch.empty(total + 16, dtype=torch.uint8, device="cuda")
    rec_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    codec.encode(db, out, rec_off, st)
    codec.sync()
    assert int((st != 0).sum()) == 0
    assert int(rec_off[0]) == 0 and torch.equal(rec_off[1:], torch.cumsum(lens, 0))
    del db
    want_xid = torch.from_numpy(hb.msgs["xid"].view(np.int32).copy()).cuda()
    bufs = R.DecodeBuffers(n)
    for mode in MODES:
        codec.decode(out, rec_off, n, mode, bufs.msgs, bufs.unix, bufs.status, bufs.aux0, bufs.aux1)
        codec.sync()
        assert int((bufs.status != 0).sum()) == 0, f"mode {mode}"
        xid = bufs.msgs.view(-1, 64)[:, 0:4].contiguous().view(torch.int32).view(-1)
        assert torch.equal(xid, want_xid), f"mode {mode}"
    # re-encode the decoded batch: descriptors point into the wire itself
    again = R.DeviceBatch(n, bufs.msgs, bufs.unix, out, out)
    out2 = torch.empty(total + 16, dtype=torch.uint8, device="cuda")
    rec_off2 = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    codec.encode(again, out2, rec_off2, st)
    codec.sync()
    assert int((st != 0).sum()) == 0
    assert torch.equal(rec_off2, rec_off)
    assert torch.equal(out2[:total], out[:total])
    del out2, again
    # bit-exact window vs the oracle
    lo, hi = n // 2, n // 2 + 20_000
    sub = L.HostBatch(hb.msgs[lo:hi].copy(), hb.unix, hb.auth_arena, hb.payload_arena)
    o_wire, o_off, o_st, _ = oracle.encode_batch(sub)
    b0, b1 = int(rec_off[lo]), int(rec_off[hi])
    g_wire = out[b0:b1].cpu().numpy()
    assert g_wire.tobytes() == o_wire
    w = np.concatenate([g_wire, np.zeros(16, np.uint8)])
    for mode in MODES:
        g = R.decode_host_wire(codec, w, o_off, mode)
        o = oracle.decode_batch(w, o_off, mode)
        assert_decoded_equal(g, o, f"{cfg} window")


def test_block_base_scan_path(R, oracle):
    """Encode places tiles either from enc_emit's own sum of the enc_len
    workgroup totals (<= 1024 workgroups) or from the scan kernel: the
    forced-scan codec and a batch above the fused limit (1.1M records) are
    bit-exact vs the oracle as well."""
    hb = S.mixed(6000, seed=21, pmin=0, pmax=700, exotic=0.2)
    c_scan = R.Codec(0, force_scan=True)
    try:
        gpu_vs_oracle_encode(R, c_scan, oracle, hb)
    finally:
        c_scan.close()
    c = R.Codec(0)
    try:
        gpu_vs_oracle_encode(R, c, oracle, hb)
        big = S.call_none(1_100_000, 13, seed=5)       # 1075 workgroups: scan launch, byte path
        gpu_vs_oracle_encode(R, c, oracle, big)
        edge = S.call_none(1024 * 1024, 8, seed=6)     # exactly 1024 workgroups: the last fused batch
        gpu_vs_oracle_encode(R, c, oracle, edge)
    finally:
        c.close()


# ---------------------------------------------------------------------------
# Vectored encode: headers + in-place payload slices.
def iov_wire(hb, hdr, iov, st):
    """Reassemble the packed wire from an iov encode (what writev would send)."""
    parts = []
    for i in range(len(iov)):
        if st[i] != 0:
            continue
        h = iov[i]
        parts.append(hdr[int(h["hdr_off"]):int(h["hdr_off"]) + int(h["hdr_len"])].tobytes())
        po = int(h["payload_off"])
        parts.append(hb.payload_arena[po:po + int(h["payload_len"])].tobytes())
    return b"".join(parts)


def gpu_iov(R, codec, hb, hdr_cap=None):
    import torch
    db = R.DeviceBatch.from_host(hb, "cuda")
    n = hb.n
    lens = R.codec_lengths(codec, db)
    cap = int(lens.sum()) if hdr_cap is None else hdr_cap
    hdr = torch.zeros(max(16, cap + 16), dtype=torch.uint8, device="cuda")
    iov = torch.zeros(max(1, n) * 32, dtype=torch.uint8, device="cuda")
    st = torch.zeros(max(1, n), dtype=torch.int32, device="cuda")
    tot = torch.zeros(2, dtype=torch.int64, device="cuda")
    codec.encode_iov(db, hdr, iov, st, tot, hdr_cap=cap)
    codec.sync()
    return (hdr.cpu().numpy(), iov.cpu().numpy().view(L.IOV_DTYPE)[:n], st.cpu().numpy()[:n],
            tot.cpu().numpy().view(np.uint64))


@pytest.mark.parametrize("gen", ["call_none", "call_unix16", "mixed_exotic", "random"])
def test_iov_encode_matches_packed_encode(codec, R, oracle, gen):
    hb = {"call_none": lambda: S.call_none(3000, 256),
          "call_unix16": lambda: S.call_unix16(2000, 1024),
          "mixed_exotic": lambda: S.mixed(3000, seed=5, pmin=0, pmax=500, exotic=0.3),
          "random": lambda: L.build_batch(S.random_messages(1500, seed=77))}[gen]()
    o_wire, o_off, o_st, _ = oracle.encode_batch(hb)
    hdr, iov, st, tot = gpu_iov(R, codec, hb)
    assert np.array_equal(st, o_st)
    ok = st == 0
    assert np.array_equal(iov["wire_off"][ok], o_off[:-1][ok])
    assert iov_wire(hb, hdr, iov, st) == o_wire
    assert int(tot[1]) == len(o_wire)
    assert int(tot[0]) == int(iov["hdr_len"].sum())
    # headers are packed back to back
    hl = iov["hdr_len"].astype(np.uint64)
    assert np.array_equal(iov["hdr_off"][ok], (np.cumsum(hl) - hl)[ok])
    assert not iov["hdr_len"][~ok].any() and not iov["payload_len"][~ok].any()


def test_iov_encode_header_capacity(codec, R, oracle):
    hb = S.mixed(700, seed=12, pmin=0, pmax=100)
    full_hdr, full_iov, full_st, _ = gpu_iov(R, codec, hb)
    total = int(full_iov["hdr_len"].sum())
    for cap in (0, 37, total // 2, total - 1):
        hdr, iov, st, _ = gpu_iov(R, codec, hb, hdr_cap=cap)
        ends = full_iov["hdr_off"] + full_iov["hdr_len"]
        want = np.where((full_st == 0) & (ends > cap), 105, full_st)
        assert np.array_equal(st, want), cap
        fit = (full_st == 0) & (ends <= cap)
        # every record that fits has its header bytes written
        for i in np.nonzero(fit)[0][:200]:
            a, b = int(full_iov["hdr_off"][i]), int(ends[i])
            assert hdr[a:b].tobytes() == full_hdr[a:b].tobytes()
        # nothing past the last fitting header is written
        lim = int(ends[fit].max()) if fit.any() else 0
        assert not hdr[lim:cap].any()


# ---------------------------------------------------------------------------
# GPU-vs-CPU differential fuzz (fuzz/fuzz_targets/*.rs)
def _random_records(n, seed):
    """Structure-aware random records: a valid record mark, then random words
    biased toward small values and the wire discriminants, so that decoding
    gets deep into every branch before failing (or succeeding)."""
    rng = np.random.default_rng(seed)
    recs = []
    for _ in range(n):
        nw = int(rng.integers(0, 48))
        words = rng.integers(0, 2**32, nw, dtype=np.uint64)
        small = rng.random(nw) < 0.7
        words[small] = rng.choice([0, 1, 2, 3, 4, 5, 6, 7, 8, 16, 20, 24, 84, 200, 201, 255, 256],
                                  int(small.sum()))
        # words 1/2 (message type, rpcvers / reply_stat) mostly valid, so the
        # decode reaches the auth / reply parsers
        if nw > 1 and rng.random() < 0.9:
            words[1] = int(rng.integers(0, 2))
        if nw > 2 and rng.random() < 0.9:
            words[2] = 2 if words[1] == 0 else int(rng.integers(0, 2))
        body = b"".join(int(w).to_bytes(4, "big") for w in words) + rng.bytes(int(rng.integers(0, 4)))
        recs.append(((len(body)) | 0x80000000).to_bytes(4, "big") + body)
    return recs


@pytest.mark.parametrize("seed", [101, 102, 103])
def test_differential_fuzz_random_records(codec, R, oracle, seed):
    recs = _random_records(6000, seed)
    wire, off = L.records_from_wire(recs)
    for mode in MODES:
        g = R.decode_host_wire(codec, wire, off, mode)
        o = oracle.decode_batch(wire, off, mode)
        assert_decoded_equal(g, o, f"fuzz seed {seed} mode {mode}")
    # fuzz_targets/bytes.rs: the two decoders agree on Ok/Err
    gs = R.decode_host_wire(codec, wire, off, L.DECODE_SLICE)[2]
    gb = R.decode_host_wire(codec, wire, off, L.DECODE_BYTES)[2]
    assert np.array_equal(gs == 0, gb == 0)


def test_parse_serialise_fuzz_invariant(codec, R, oracle):
    """fuzz_targets/parse_serialise.rs: whatever decodes re-serialises to a
    message that decodes to the same value."""
    hb = L.build_batch(S.random_messages(1000, seed=41, max_payload=64))
    wire, off, _ = oracle.encode_batch(hb)[:3]
    w = np.frombuffer(wire + b"\0" * 16, np.uint8).copy()
    recs = [w[off[i]:off[i + 1]].tobytes() for i in range(len(off) - 1)] + _random_records(2000, 7)
    cw, coff = L.records_from_wire(recs)
    cw, coff = S.corrupt(cw, coff, frac=0.5, seed=5)
    gm, gu, gs, _, _ = R.decode_host_wire(codec, cw, coff, L.DECODE_SLICE)
    ok = np.nonzero(gs == 0)[0]
    assert len(ok) > 500
    wire2, off2, st2, _ = R.encode_host_batch(codec, L.HostBatch(gm[ok].copy(), gu, cw, cw))
    assert (st2 == 0).all()
    w2 = np.frombuffer(wire2 + b"\0" * 16, np.uint8).copy()
    hm, hu, hs, _, _ = R.decode_host_wire(codec, w2, off2, L.DECODE_SLICE)
    assert (hs == 0).all()
    for j, i in enumerate(ok):
        assert L.describe(hm[j], hu, w2) == L.describe(gm[i], gu, cw), int(i)


# ---------------------------------------------------------------------------
# Stream framing vs the caller's expected_message_len loop
def _frame_both(R, codec, oracle, buf, max_records=None):
    g = R.frame_host_stream(codec, buf, max_records)
    o = oracle.frame_stream(buf, max_records)
    assert g[1:] == o[1:], (g[1:], o[1:])
    assert np.array_equal(g[0], o[0])
    return o


@pytest.fixture(params=[None, 64, 1024, "force_scan"])
def frame_codec(request, R):
    """Codec with the default framing chunk (64 KiB) and with small chunks
    (onc_codec_options.frame_chunk), so that test streams span many chunks: guesses,
    verification and the walk across chunk boundaries; "force_scan" takes the
    three-launch count scan (onc_codec_options ONC_OPT_FORCE_SCAN) instead of the fused one."""
    if request.param == "force_scan":
        c = R.Codec(0, force_scan=True)
    elif request.param is not None:
        c = R.Codec(0, frame_chunk=request.param)
    else:
        c = R.Codec(0)
    yield c
    c.close()


def test_frame_stream_valid_streams(frame_codec, R, oracle):
    codec = frame_codec
    for hb in (S.call_none(5000, 256), S.mixed(3000, seed=3, pmin=0, pmax=5000, exotic=0.2),
               L.build_batch(S.random_messages(3000, seed=8, max_payload=300))):
        wire = oracle.encode_batch(hb)[0]
        o = _frame_both(R, codec, oracle, wire)
        assert o[1] == int((oracle.encode_batch(hb)[2] == 0).sum()) and o[3] == 0
        # every cut inside the stream: incomplete tails
        for cut in (len(wire) - 1, len(wire) - 3, len(wire) // 2, 5, 2, 0):
            _frame_both(R, codec, oracle, wire[:cut])
        for m in (1, 7, hb.n // 2, hb.n - 1, hb.n, hb.n + 5):
            _frame_both(R, codec, oracle, wire, max_records=m)


def test_frame_stream_adversarial(frame_codec, R, oracle):
    codec = frame_codec
    rng = np.random.default_rng(4)
    # payloads that are themselves RPC streams (nested records fool the guess)
    inner = oracle.encode_batch(S.mixed(400, seed=9, pmin=0, pmax=900))[0]
    msgs = []
    for i in range(600):
        k = int(rng.integers(0, len(inner) - 2000))
        msgs.append({"xid": i, "type": "call", "program": 1, "program_version": 1, "procedure": 1,
                     "cred": {"kind": "none", "data": None}, "verf": {"kind": "none", "data": None},
                     "payload": inner[k:k + int(rng.integers(0, 2000))].hex()})
    wire = oracle.encode_batch(L.build_batch(msgs))[0]
    _frame_both(R, codec, oracle, wire)
    # tiny and empty-body records (4..20 bytes), huge records spanning chunks
    parts = []
    for i in range(3000):
        kind = int(rng.integers(0, 3))
        body = rng.bytes(int(rng.integers(0, 17)) if kind < 2 else int(rng.integers(3000, 9000)))
        parts.append(((len(body)) | 0x80000000).to_bytes(4, "big") + body)
    stream = b"".join(parts)
    _frame_both(R, codec, oracle, stream)
    # a fragmented header, and random garbage after a valid prefix
    bad = bytearray(stream)
    j = len(b"".join(parts[:1500]))
    bad[j] &= 0x7F
    _frame_both(R, codec, oracle, bytes(bad))
    _frame_both(R, codec, oracle, stream[:j] + rng.bytes(50000))
    _frame_both(R, codec, oracle, rng.bytes(100000))
