"""GPU tests, round 3: the plan / emit contract (a plan is discarded by any
call that reuses the handle's scratch; emit must get the plan's status
array), and payloads at the first and last byte of a tightly sized payload
arena on both enc_emit kernels; the chunked encode at 2048-record chunks
(message and body roots), the decode line policy and the emit from the
plan's lengths. Bit-exact against the CPU oracle."""
import numpy as np
import pytest

import onc_rpc_amd.layout as L
import onc_rpc_amd.synth as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def R():
    import onc_rpc_amd.runtime as R
    return R


@pytest.fixture(scope="module")
def codec(R):
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    c = R.Codec(0)
    yield c
    c.close()


def _plan(R, codec, hb):
    import torch
    db = R.DeviceBatch.from_host(hb)
    st = torch.empty(hb.n, dtype=torch.int32, device="cuda")
    codec.encode_plan(db, st)
    return db, st


def test_plan_discarded_by_scratch_users(codec, R, oracle):
    """plan(A), then any call that writes the handle's scratch (encode
    lengths / encode / iov / decode_lengths / scan_lengths), then emit(A):
    refused (EINVAL) instead of placing A by the other call's totals; a fresh
    plan makes emit work again, bit-exact."""
    import torch
    hb = S.mixed(3000, seed=31, pmin=0, pmax=600, exotic=0.2)
    other = S.call_none(5000, 64)
    o_wire, o_off, o_st, _ = oracle.encode_batch(hb)
    total = len(o_wire)
    buf = torch.zeros(total + 64, dtype=torch.uint8, device="cuda")
    off = torch.empty(hb.n + 1, dtype=torch.int64, device="cuda")
    dbo = R.DeviceBatch.from_host(other)
    rl = torch.empty(other.n, dtype=torch.int32, device="cuda")
    sto = torch.empty(other.n, dtype=torch.int32, device="cuda")
    wire_o, off_o, _, len_o = R.encode_host_batch(codec, other)
    w_dev = R.to_device(np.frombuffer(wire_o + b"\0" * 16, np.uint8), "cuda")
    lens = torch.from_numpy(len_o.view(np.int32).copy()).cuda()
    dec = R.DecodeBuffers(other.n)
    offs = torch.empty(other.n + 1, dtype=torch.int64, device="cuda")

    def lengths():
        codec.encode_lengths(dbo, rl, sto)

    def decode_lengths():
        codec.decode_lengths(w_dev, lens, other.n, 0, L.DECODE_SLICE, dec.msgs, dec.unix, dec.status, dec.aux0,
                             dec.aux1)

    def scan():
        codec.scan_lengths(lens, other.n, 0, offs)

    def iov():
        hdr = torch.empty(other.n * 64, dtype=torch.uint8, device="cuda")
        iv = torch.empty(other.n * 32, dtype=torch.uint8, device="cuda")
        codec.encode_iov(dbo, hdr, iv, sto)

    def encode_other():
        R.encode_host_batch(codec, other)

    for between in (lengths, decode_lengths, scan, iov, encode_other):
        db, st = _plan(R, codec, hb)
        between()
        with pytest.raises(R.CodecError):
            codec.encode_emit(db, buf, off, st, out_cap=total)
    db, st = _plan(R, codec, hb)
    codec.encode_emit(db, buf, off, st, out_cap=total)
    codec.sync()
    assert buf.cpu().numpy()[:total].tobytes() == o_wire
    assert np.array_equal(off.cpu().numpy().view(np.uint64), o_off)
    assert np.array_equal(st.cpu().numpy(), o_st)


def test_emit_needs_the_plans_status_array(codec, R, oracle):
    """emit only adds WRITE_ZERO to the plan's statuses, so it must be handed
    the array the plan filled (onc_rpc.h onc_encode_emit)."""
    import torch
    hb = S.call_none(700, 100)
    db, st = _plan(R, codec, hb)
    other_st = torch.empty_like(st)
    buf = torch.zeros(700 * 160, dtype=torch.uint8, device="cuda")
    off = torch.empty(hb.n + 1, dtype=torch.int64, device="cuda")
    with pytest.raises(R.CodecError):
        codec.encode_emit(db, buf, off, other_st)
    codec.encode_emit(db, buf, off, st)      # the plan is still there
    codec.sync()
    o_wire, o_off, _, _ = oracle.encode_batch(hb)
    assert buf.cpu().numpy()[:len(o_wire)].tobytes() == o_wire


@pytest.mark.parametrize("variant", [0x200, 0x400, 0x200 | 0x4000, 0x200 | 0x8000])
@pytest.mark.parametrize("layout", ["first_last", "reversed"])
def test_payloads_at_arena_edges(R, oracle, variant, layout):
    """Payloads starting at byte 0 and ending at the last byte of a payload
    arena declared exactly as large as its payloads (and placed at the very
    end of its tensor): the interior-span source check (encode.hip
    ws_stage_span) must keep every load inside [0, payload_len); output
    bit-exact on the wave-specialised kernel (0x200, with and without the
    interior / full-interior paths) and the wave-per-tile one (0x400)."""
    import torch
    codec = R.Codec(0, variant=variant)
    try:
        rng = np.random.default_rng(variant + (7 if layout == "reversed" else 0))
        n = 3000
        plens = rng.integers(16, 700, n)
        plens[::5] = 4 * rng.integers(4, 170, len(plens[::5]))      # word-path tiles too
        msgs = []
        for i in range(n):
            msgs.append({"xid": i, "type": "call", "program": 100003, "program_version": 4, "procedure": 1,
                         "cred": {"kind": "none", "data": None}, "verf": {"kind": "none", "data": None},
                         "payload": rng.bytes(int(plens[i])).hex()})
        hb = L.build_batch(msgs)
        total_p = int(plens.sum())
        arena = hb.payload_arena[:total_p]                     # drop the builder's spare byte: exact size
        if layout == "reversed":
            # record i's payload sits where record n-1-i's did: the first record
            # reads the arena's last bytes, the last record its first bytes
            offs = np.concatenate([[0], np.cumsum(plens[::-1])])[:-1][::-1]
            new = np.zeros(total_p, np.uint8)
            for i in range(n):
                o, src, ln = int(offs[i]), int(hb.msgs["payload_off"][i]), int(plens[i])
                new[o:o + ln] = arena[src:src + ln]
            hb.msgs["payload_off"] = offs
            arena = new
        hb = L.HostBatch(hb.msgs, hb.unix, hb.auth_arena, arena)
        o_wire, o_off, o_st, _ = oracle.encode_batch(hb)
        # the arena at the end of its tensor, declared exactly
        big = torch.full((total_p + 4096,), 0xEE, dtype=torch.uint8, device="cuda")
        pay = big[4096:]
        pay.copy_(torch.from_numpy(arena.copy()).cuda())
        db = R.DeviceBatch(n, R.to_device(hb.msgs, "cuda"), R.to_device(hb.unix, "cuda"),
                           R.to_device(hb.auth_arena, "cuda"), pay, payload_len=total_p)
        out = torch.zeros(len(o_wire) + 64, dtype=torch.uint8, device="cuda")
        off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        st = torch.empty(n, dtype=torch.int32, device="cuda")
        codec.encode(db, out, off, st, out_cap=len(o_wire))
        codec.sync()
        assert np.array_equal(st.cpu().numpy(), o_st) and (o_st == 0).all()
        assert np.array_equal(off.cpu().numpy().view(np.uint64), o_off)
        assert out.cpu().numpy()[:len(o_wire)].tobytes() == o_wire
    finally:
        codec.close()


def test_bench_two_ranks_line_has_cpu_baseline():
    """A real 2-rank bench run (both ranks on GPU 0, gloo for the control
    plane): the JSON line carries per-GPU rows, the aggregate, validated, and
    the CPU baseline rank 0 timed after both ranks' GPU legs."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["ONC_BENCH_SAME_DEVICE"] = "1"
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--records", "20000", "--c4-leg", "off", "--iov-leg", "off", "--steps", "3", "--warmup", "1",
                        "--cpu-seconds", "1", "--cpu-threads", "2", "--no-pcie"],
                       env=env, cwd=root, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert r["n_gpus"] == 2 and r["validated"] and len(r["per_gpu"]) == 2
    cb = r["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["sample_bit_exact_vs_gpu"] is True
    assert "after all 2 ranks" in cb["note"]


@pytest.mark.parametrize("shift,cap_frac", [(0, None), (7, None), (3, 0.6)])
def test_chunked_encode_bit_exact(codec, R, oracle, shift, cap_frac):
    """onc_encode beyond 1M records runs as 1M-record chunks, each planned
    right before it is emitted (codec.hip encode_batch): records across the
    chunk boundary at any writer position (byte path: odd payloads), with the
    capacity ending inside the second chunk — bytes, offsets and statuses
    equal to the oracle's whole-batch loop."""
    import torch
    hb = S.mixed(1_100_000, seed=5, pmin=0, pmax=300, exotic=0.1)
    o_wire, o_off, o_st, o_len = oracle.encode_batch(hb)
    total = len(o_wire)
    cap = total if cap_frac is None else int(total * cap_frac)
    if cap != total:
        o_wire, o_off, o_st, o_len = oracle.encode_batch(hb, out_cap=cap)
    db = R.DeviceBatch.from_host(hb)
    buf = torch.full((shift + total + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    off = torch.empty(hb.n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(hb.n, dtype=torch.int32, device="cuda")
    rl = torch.empty(hb.n, dtype=torch.int32, device="cuda")
    codec.encode(db, buf[shift:], off, st, rl, out_cap=cap)
    codec.sync()
    b = buf.cpu().numpy()
    assert np.array_equal(st.cpu().numpy(), o_st)
    assert np.array_equal(off.cpu().numpy().view(np.uint64), o_off)
    assert np.array_equal(rl.cpu().numpy().view(np.uint32), o_len)
    assert b[shift:shift + len(o_wire)].tobytes() == o_wire
    assert (b[:shift] == 0xA5).all() and (b[shift + cap:] == 0xA5).all()


def _same_decode(g, o, what):
    gm, gu, gs, ga0, ga1 = g
    om, ou, os_, oa0, oa1 = o
    bad = np.nonzero(gs != os_)[0]
    assert len(bad) == 0, f"{what}: status at {bad[:8]} gpu {gs[bad[:8]]} oracle {os_[bad[:8]]}"
    assert np.array_equal(ga0, oa0) and np.array_equal(ga1, oa1), what
    # the packed AUTH_UNIX layout is the ABI's: descriptors (refs included)
    # byte-equal, and the referenced slots equal
    bad = np.nonzero((gm.view(np.uint8).reshape(-1, 64) != om.view(np.uint8).reshape(-1, 64)).any(axis=1))[0]
    assert len(bad) == 0, f"{what}: descriptor at {bad[:8]}"
    _, gp = L.resolve_unix(gm, gu, gs)
    _, op = L.resolve_unix(om, ou, os_)
    assert np.array_equal(gp, op), what


@pytest.mark.parametrize("gen", ["mixed", "unix16"])
def test_decode_at_every_record_alignment(codec, R, oracle, gen):
    """The decode window's columns are funnelled by the record's byte offset
    once, at staging (decode.hip `Rd`): the same batch decoded at wire
    offsets 0..15 (every position in a 16-byte granule, every byte offset in
    a word), and with 1..3-byte junk records between its records so that
    neighbours start at every offset; both modes, bit-exact vs the oracle
    (descriptors, AUTH_UNIX slots at their packed refs, statuses, aux)."""
    if gen == "mixed":
        hb = S.mixed(1500, seed=31, pmin=0, pmax=200, exotic=0.2)
    else:
        hb = S.call_unix16(1500, 40, seed=32)
    wire, off, st, _ = oracle.encode_batch(hb)
    assert (st == 0).all()
    base = np.frombuffer(wire, np.uint8)
    for shift in range(16):
        w = np.concatenate([np.full(shift, 0xEE, np.uint8), base, np.zeros(16, np.uint8)])
        o2 = off.astype(np.uint64) + np.uint64(shift)
        for mode in (L.DECODE_SLICE, L.DECODE_BYTES):
            _same_decode(R.decode_host_wire(codec, w, o2, mode), oracle.decode_batch(w, o2, mode),
                         f"{gen} shift {shift} mode {mode}")
    recs = []
    for i in range(hb.n):
        recs.append(bytes(base[int(off[i]):int(off[i + 1])]))
        if i % 3 == 1:
            recs.append(b"\x80" * (1 + (i // 3) % 3))   # IncompleteHeader, shifts what follows
    w, o2 = L.records_from_wire(recs)
    starts = np.asarray(o2[:-1], np.int64) & 15
    assert len(np.unique(starts)) == 16
    for mode in (L.DECODE_SLICE, L.DECODE_BYTES):
        g = R.decode_host_wire(codec, w, o2, mode)
        _same_decode(g, oracle.decode_batch(w, o2, mode), f"{gen} interleaved mode {mode}")
        assert int((g[2] == 0).sum()) == hb.n


@pytest.mark.parametrize("policy", [0, 2, 1])
def test_decode_line_policy(R, oracle, policy):
    """The decode's two first-round policies (decode.hip kLine1Min): the line
    policy (ONC_DECODE_POLICY_LINE: round 1 takes the rest of the record's
    first 128-byte line), the standard one (_STANDARD), and the automatic
    choice from the codec's hint word (_AUTO: a unix16 batch flips it to the
    line policy for the next launch, a mixed one back). Every launch bit-exact vs the oracle in
    both modes: header-heavy and mixed batches at every record alignment,
    records cut inside their first line (truncated headers), and the
    lengths-driven decode."""
    import torch
    codec = R.Codec(0, decode_policy=policy)
    try:
        unix16 = S.call_unix16(1200, 40, seed=41)
        mixed = S.mixed(1200, seed=42, pmin=0, pmax=300, exotic=0.2)
        for hb in (unix16, unix16, mixed, mixed, unix16):
            wire, off, st, _ = oracle.encode_batch(hb)
            base = np.frombuffer(wire, np.uint8)
            for shift in (0, 3, 8, 13):
                w = np.concatenate([np.full(shift, 0xEE, np.uint8), base, np.zeros(16, np.uint8)])
                o2 = off.astype(np.uint64) + np.uint64(shift)
                for mode in (L.DECODE_SLICE, L.DECODE_BYTES):
                    _same_decode(R.decode_host_wire(codec, w, o2, mode), oracle.decode_batch(w, o2, mode),
                                 f"policy {policy} shift {shift} mode {mode}")
            # every record cut to a prefix (1..200 bytes): headers that end
            # inside the first line, inside round 1, or past the window
            rng = np.random.default_rng(policy + 1)
            recs = []
            for i in range(hb.n):
                r = bytes(base[int(off[i]):int(off[i + 1])])
                recs.append(r[:int(rng.integers(1, 200))] if i % 2 else r)
            w2, o3 = L.records_from_wire(recs)
            for mode in (L.DECODE_SLICE, L.DECODE_BYTES):
                _same_decode(R.decode_host_wire(codec, w2, o3, mode), oracle.decode_batch(w2, o3, mode),
                             f"policy {policy} truncated mode {mode}")
            # lengths-driven decode of the same wire
            n = hb.n
            lens = np.diff(off.astype(np.int64)).astype(np.uint32)
            dw = torch.from_numpy(base.copy()).cuda()
            rl = torch.from_numpy(lens.view(np.int32).copy()).cuda()
            dec = R.DecodeBuffers(n)
            ro = torch.empty(n + 1, dtype=torch.int64, device="cuda")
            codec.decode_lengths(dw, rl, n, 0, L.DECODE_SLICE, dec.msgs, dec.unix, dec.status, dec.aux0, dec.aux1,
                                 rec_off=ro)
            codec.sync()
            _same_decode(dec.to_host(), oracle.decode_batch(base, off.astype(np.uint64), L.DECODE_SLICE),
                         f"policy {policy} decode_lengths")
    finally:
        codec.close()


@pytest.mark.parametrize("variant", [0x400, 0x400 | 0x20000])
@pytest.mark.parametrize("given_len", [False, True])
def test_emit_from_plan_lengths(R, oracle, variant, given_len):
    """The wave-per-tile enc_emit reads the plan's record lengths (the
    caller's rec_len, or the codec's own array) instead of planning again
    when the batch has an AUTH_UNIX table (codec.hip use_lens; 0x20000 keeps
    the re-planning emit): AUTH_UNIX-heavy and mixed batches with failing
    records, through onc_encode and through onc_encode_plan + emit, and past
    one 1M-record plan chunk — bytes, offsets and statuses equal to the
    oracle's."""
    import torch
    codec = R.Codec(0, variant=variant)
    try:
        for hb in (S.cpu_roundtrip(3000, seed=51), S.mixed(3000, seed=52, pmin=0, pmax=90, exotic=0.3),
                   S.call_unix16(1_050_000, 20, seed=53)):
            o_wire, o_off, o_st, o_len = oracle.encode_batch(hb)
            db = R.DeviceBatch.from_host(hb)
            n = hb.n
            for plan_emit in (False, True):
                if plan_emit and n > 1_000_000:
                    continue          # plan + emit covers one plan (the chunked path is onc_encode's)
                out = torch.zeros(len(o_wire) + 64, dtype=torch.uint8, device="cuda")
                off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
                st = torch.empty(n, dtype=torch.int32, device="cuda")
                rl = torch.empty(n, dtype=torch.int32, device="cuda") if given_len else None
                if plan_emit:
                    codec.encode_plan(db, st, rl)
                    codec.encode_emit(db, out, off, st)
                else:
                    codec.encode(db, out, off, st, rl)
                codec.sync()
                what = f"variant {variant:#x} n {n} plan_emit {plan_emit}"
                assert np.array_equal(st.cpu().numpy(), o_st), what
                assert np.array_equal(off.cpu().numpy().view(np.uint64), o_off), what
                if rl is not None:
                    assert np.array_equal(rl.cpu().numpy().view(np.uint32), o_len), what
                assert out.cpu().numpy()[:len(o_wire)].tobytes() == o_wire, what
    finally:
        codec.close()


@pytest.mark.parametrize("variant", [0, 0x200, 0x400])
def test_small_encode_chunks(R, oracle, variant):
    """The chunked encode (codec.hip encode_batch) with 2048-record chunks
    (onc_codec_options.enc_chunk), so that small batches cross many chunk boundaries:
    RpcMessage batches of every shape (mixed with failing records and odd
    payloads, AUTH_UNIX-heavy with the plan's lengths read by the emit) at an
    odd writer position with the capacity ending inside a later chunk, on the
    automatic kernel choice and with each enc_emit kernel forced, and every
    body root (onc_encode_body) — bytes, offsets, statuses and lengths equal
    to the oracle's whole-batch loop."""
    import torch
    from test_body_roots import ROOTS, _valid_messages
    codec = R.Codec(0, variant=variant, enc_chunk=2048)
    try:
        for hb in (S.mixed(9001, seed=61, pmin=0, pmax=300, exotic=0.2), S.cpu_roundtrip(7000, seed=62),
                   S.call_none(5000, 256, seed=63)):
            for shift, cap_frac in ((0, None), (5, 0.7)):
                o_wire, o_off, o_st, o_len = oracle.encode_batch(hb)
                total = len(o_wire)
                cap = total if cap_frac is None else int(total * cap_frac)
                if cap != total:
                    o_wire, o_off, o_st, o_len = oracle.encode_batch(hb, out_cap=cap)
                db = R.DeviceBatch.from_host(hb)
                buf = torch.full((shift + total + 64,), 0xA5, dtype=torch.uint8, device="cuda")
                off = torch.empty(hb.n + 1, dtype=torch.int64, device="cuda")
                st = torch.empty(hb.n, dtype=torch.int32, device="cuda")
                rl = torch.empty(hb.n, dtype=torch.int32, device="cuda")
                codec.encode(db, buf[shift:], off, st, rl, out_cap=cap)
                codec.sync()
                what = f"variant {variant:#x} n {hb.n} shift {shift} cap {cap}"
                b = buf.cpu().numpy()
                assert np.array_equal(st.cpu().numpy(), o_st), what
                assert np.array_equal(off.cpu().numpy().view(np.uint64), o_off), what
                assert np.array_equal(rl.cpu().numpy().view(np.uint32), o_len), what
                assert b[shift:shift + len(o_wire)].tobytes() == o_wire, what
                assert (b[:shift] == 0xA5).all() and (b[shift + cap:] == 0xA5).all(), what
        hb = L.build_batch(_valid_messages(5000, seed=64))
        for root in ROOTS:
            g = R.encode_body_host_batch(codec, root, hb)
            o = oracle.encode_body_batch(root, hb)
            assert np.array_equal(g[2], o[2]) and np.array_equal(g[3], o[3]), L.ROOT_NAMES[root]
            assert np.array_equal(g[1], o[1]) and g[0] == o[0], L.ROOT_NAMES[root]
    finally:
        codec.close()
