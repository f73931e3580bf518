"""GPU tests, round 6 (ABI 8).

* onc_compact / onc_compact_iov: the placeholder extents of failing records
  dropped from an encoded batch in place — the stream the reference's loop
  of serialise_into calls writes (a failing message writes nothing:
  unix_params.rs:47,149, flavor.rs:110). Checked against the struct-built
  fixture (tests/golden/placeholder.json), the oracle's restatement
  (oracle_compact) and the oracle's encode of only the OK records, then
  framed (expected_message_len, rpc_message.rs:343-367) and decoded.
* Host registrations belong to the process: a registration outlives its
  codec (onc_host_unregister with a NULL codec), registrations of one range
  are counted, a range running past its pinned allocation is refused.
* The one-launch small-batch encode after the single-pass lab's removal
  (placement through LDS only).
* The decode's cooperative round 1 (decode.hip load_round1) on ragged
  waves, and its per-lane fallback for windows 2 GiB apart.
"""
import ctypes as C
import mmap

import numpy as np
import pytest

import onc_rpc_amd.layout as L
import onc_rpc_amd.synth as S
from test_gpu_parity import all_golden_records, assert_decoded_equal

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


def _device_encode(R, codec, hb, shift=0, variant_codec=None):
    """Device encode into a buffer at writer offset `shift` -> (torch out,
    torch rec_off, torch status, total)."""
    import torch
    c = variant_codec or codec
    db = R.DeviceBatch.from_host(hb)
    total = int(R.codec_lengths(c, db).sum())
    out = torch.full((shift + total + 64,), 0x5A, dtype=torch.uint8, device="cuda")
    off = torch.empty(hb.n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(max(hb.n, 1), dtype=torch.int32, device="cuda")
    c.encode(db, out[shift:], off, st, out_cap=total)
    c.sync()
    return out, off, st, total, db


@pytest.mark.parametrize("shift", [0, 3])
def test_compact_fixture(codec, R, shift):
    """The struct-built fixture: the device encode writes its placeholder
    bytes; onc_compact leaves exactly the compacted stream and offsets."""
    from test_oracle_golden import _placeholder_batch, placeholder_fixture
    fx = placeholder_fixture()
    hb = _placeholder_batch()
    out, off, st, total, _ = _device_encode(R, codec, hb, shift)
    assert list(st.cpu().numpy()[:hb.n]) == fx["status"]
    assert out[shift:shift + total].cpu().numpy().tobytes().hex() == fx["wire"]
    assert list(off.cpu().numpy()) == fx["rec_off"]
    new_total = codec.compact(out[shift:], off, st, hb.n)
    codec.sync()
    c = bytes.fromhex(fx["compacted"])
    assert new_total == len(c)
    assert out[shift:shift + len(c)].cpu().numpy().tobytes() == c
    assert list(off.cpu().numpy()) == fx["compacted_rec_off"]
    assert (out[:shift].cpu().numpy() == 0x5A).all()


@pytest.mark.parametrize("seed,n", [(101, 3000), (102, 20_000), (103, 70_001)])
def test_compact_adversarial_batch(codec, R, oracle, seed, n):
    """An adversarial batch (a quarter of the AUTH_UNIX auths broken: many
    placeholders among failing and OK records): onc_compact's bytes and
    offsets are the oracle's compaction, equal to the oracle's encode of only
    the OK records; the compacted stream frames (device and oracle) into
    exactly the OK records and each decodes to its descriptor."""
    from test_gpu_emit_paths import _adversarial
    hb = _adversarial(seed, n=n)
    o_wire, o_off, o_st, o_len = oracle.encode_batch(hb)
    assert ((o_st != 0) & (o_len != 0)).sum() > 10
    out, off, st, total, _ = _device_encode(R, codec, hb)
    assert out[:total].cpu().numpy().tobytes() == o_wire
    new_total = codec.compact(out, off, st, hb.n)
    codec.sync()
    c_wire, c_off = oracle.compact(o_wire, o_off, o_st)
    assert new_total == len(c_wire)
    assert out[:new_total].cpu().numpy().tobytes() == c_wire
    assert np.array_equal(off.cpu().numpy().view(np.uint64), c_off)
    # = the oracle's encode of the OK records alone
    keep = np.nonzero(o_st == 0)[0]
    sub = L.HostBatch(hb.msgs[keep].copy(), hb.unix, hb.auth_arena, hb.payload_arena)
    s_wire, s_off, s_st, _ = oracle.encode_batch(sub)
    assert (s_st == 0).all() and s_wire == c_wire
    fo, nf, consumed, fst, _, _ = R.frame_host_stream(codec, c_wire)
    assert (nf, consumed, fst) == (len(keep), len(c_wire), 0)
    assert np.array_equal(fo, s_off)
    gm = R.decode_host_wire(codec, np.frombuffer(c_wire + b"\0" * 16, np.uint8), fo, L.DECODE_SLICE)
    assert (gm[2] == 0).all()
    assert np.array_equal(gm[0]["xid"], hb.msgs["xid"][keep])
    assert np.array_equal(gm[0]["payload_len"], hb.msgs["payload_len"][keep])


@pytest.mark.parametrize("variant", [0x200, 0x400, 0x400 | 0x20000])
def test_compact_every_emit_path(R, oracle, variant):
    """Placeholders from each enc_emit kernel, compacted: the oracle's bytes."""
    from test_gpu_emit_paths import _adversarial
    hb = _adversarial(104 + variant % 5, n=5000)
    o_wire, o_off, o_st, _ = oracle.encode_batch(hb)
    c = R.Codec(0, variant=variant)
    try:
        out, off, st, total, _ = _device_encode(R, None, hb, variant_codec=c)
        new_total = c.compact(out, off, st, hb.n)
        c.sync()
        c_wire, c_off = oracle.compact(o_wire, o_off, o_st)
        assert out[:new_total].cpu().numpy().tobytes() == c_wire
        assert np.array_equal(off.cpu().numpy().view(np.uint64), c_off)
    finally:
        c.close()


def test_compact_nothing_to_drop(codec, R, oracle):
    """No placeholder (failing records without an extent only, or none):
    nothing moves, the offsets stay, the total is rec_off[n]; n = 0 returns
    rec_off[0]."""
    import torch
    hb = S.call_none(4000, 100, seed=105)
    hb = L.HostBatch(hb.msgs, hb.unix, np.zeros(256, np.uint8), hb.payload_arena)
    bad = np.arange(7, hb.n, 97)
    hb.msgs["verf_kind_len"][bad] = int(L.pack_kind_len(L.KIND_SHORT, 201))   # assert > 200: no bytes
    o_wire, o_off, o_st, o_len = oracle.encode_batch(hb)
    assert (o_st[bad] == 101).all() and not ((o_st != 0) & (o_len != 0)).any()
    out, off, st, total, _ = _device_encode(R, codec, hb)
    before = out.clone()
    off0 = off.clone()
    assert codec.compact(out, off, st, hb.n) == total
    codec.sync()
    assert torch.equal(out, before) and torch.equal(off, off0)
    z = torch.tensor([7], dtype=torch.int64, device="cuda")
    assert codec.compact(out, z, st, 0) == 7


def test_compact_large_c1_shape(codec, R, oracle):
    """A configs[1]-shaped batch of 1M records with 1 in 4096 credentials
    declared AUTH_UNIX and broken (placeholders spread over the whole
    output): the compacted buffer is the oracle's compaction, byte for byte."""
    import torch
    hb = S.call_none(1_000_000, 256, seed=106)
    # a few records get a declared AUTH_UNIX credential whose block is broken
    rng = np.random.default_rng(106)
    idx = np.sort(rng.choice(hb.n, hb.n // 4096, replace=False))
    unix = np.zeros(len(idx), L.UNIX_DTYPE)
    unix["ngids"] = 17
    m = hb.msgs
    m["cred_kind_len"][idx] = int(L.pack_kind_len(L.KIND_UNIX, 20))
    m["cred_id"][idx] = 1
    m["cred_ref"][idx] = np.arange(len(idx))
    hb = L.HostBatch(m, unix, np.zeros(16, np.uint8), hb.payload_arena)
    o_wire, o_off, o_st, o_len = oracle.encode_batch(hb)
    assert int(((o_st != 0) & (o_len != 0)).sum()) == len(idx)
    out, off, st, total, _ = _device_encode(R, codec, hb)
    new_total = codec.compact(out, off, st, hb.n)
    codec.sync()
    c_wire, c_off = oracle.compact(o_wire, o_off, o_st)
    assert new_total == len(c_wire)
    got = out[:new_total].cpu().numpy()
    assert np.array_equal(got, np.frombuffer(c_wire, np.uint8))
    assert np.array_equal(off.cpu().numpy().view(np.uint64), c_off)
    del out
    torch.cuda.empty_cache()


def test_compact_mapped_output(codec, R, oracle):
    """The encode's output in mapped host memory (a send buffer), compacted
    in place there."""
    from test_gpu_emit_paths import _adversarial
    hb = _adversarial(107, n=4000)
    o_wire, o_off, o_st, _ = oracle.encode_batch(hb)
    db = R.DeviceBatch.from_host(hb)
    out = R.HostMapped(codec, len(o_wire) + 64)
    off = R.HostMapped(codec, 8 * (hb.n + 1))
    st = R.HostMapped(codec, 4 * hb.n)
    try:
        codec.encode(db, out, off, st, out_cap=len(o_wire))
        codec.sync()
        assert out.host[:len(o_wire)].tobytes() == o_wire
        t = codec.compact(out, off, st, hb.n)
        c_wire, c_off = oracle.compact(o_wire, o_off, o_st)
        assert t == len(c_wire) and out.host[:t].tobytes() == c_wire
        assert np.array_equal(off.view(np.uint64)[:hb.n + 1], c_off)
    finally:
        for b in (out, off, st):
            b.close()


def test_compact_iov(codec, R, oracle):
    """onc_compact_iov: the failing records' iovecs emptied and wire_off
    re-placed; the gathered iovecs are the compacted contiguous stream."""
    import torch
    from test_gpu_emit_paths import _adversarial
    from test_gpu_iov import gpu_iov
    from test_gpu_r05 import gather_iov
    hb = _adversarial(108, n=3000)
    o_wire, o_off, o_st, _ = oracle.encode_batch(hb)
    c_wire, c_off = oracle.compact(o_wire, o_off, o_st)
    db = R.DeviceBatch.from_host(hb)
    n = hb.n
    hdr = torch.zeros(len(o_wire) + 64, dtype=torch.uint8, device="cuda")
    iov = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    tot = torch.zeros(2, dtype=torch.int64, device="cuda")
    codec.encode_iov(db, hdr, iov, st, tot, hdr_cap=len(o_wire))
    codec.compact_iov(iov, st, n, tot)
    codec.sync()
    e = iov.cpu().numpy().view(L.IOV_DTYPE)[:n]
    assert np.array_equal(e["wire_off"], c_off[:-1])
    bad = o_st != 0
    assert (e["hdr_len"][bad] == 0).all() and (e["payload_len"][bad] == 0).all()
    assert gather_iov(hb, hdr.cpu().numpy(), e) == c_wire
    t = tot.cpu().numpy()
    assert int(t[1]) == len(c_wire) and int(t[0]) == int(e["hdr_len"].astype(np.int64).sum())


# ---------------------------------------------------------------------------
# host registrations (ABI 8)
# ---------------------------------------------------------------------------
_libc = C.CDLL(None, use_errno=True)
_libc.mmap.restype = C.c_void_p
_libc.mmap.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_long]
_libc.munmap.argtypes = [C.c_void_p, C.c_size_t]
PROT_RW, MAP_PRIV_ANON, MAP_FIXED = 0x3, 0x22, 0x10


def _pinned(addr):
    """hipPointerGetAttributes: whether the runtime holds `addr` pinned."""
    hip = C.CDLL("libamdhip64.so")
    attr = (C.c_uint8 * 128)()
    rc = hip.hipPointerGetAttributes(C.byref(attr), C.c_void_p(addr))
    if rc != 0:
        hip.hipGetLastError()
        return False
    return C.cast(attr, C.POINTER(C.c_int))[0] != 0          # hipMemoryType: 0 = unregistered


def _decode_golden_at(R, codec, addr, dev, golden):
    """Golden records written at `addr` (mapped, device address `dev`),
    decoded in place: the oracle's outputs."""
    recs, _ = all_golden_records(golden)
    wire, off = L.records_from_wire(recs)
    C.memmove(addr, wire.tobytes(), len(wire))

    class _P:
        def data_ptr(self):
            return dev
    import torch
    n = len(off) - 1
    d = R.DecodeBuffers(n)
    o = torch.from_numpy(off.astype(np.uint64).view(np.int64).copy()).cuda()
    codec.decode(_P(), o, n, L.DECODE_SLICE, d.msgs, d.unix, d.status, d.aux0, d.aux1)
    codec.sync()
    return d.to_host(), wire, off


def test_registration_outlives_codec(R, oracle, golden):
    """A range registered by a codec that is then destroyed is unregistered
    with a NULL codec (before its pages are freed); new pages mapped at the
    same address and registered by another codec are read in place — not
    the old mapping's stale pages (HostMapped.close after its
    codec's close left the range pinned)."""
    size = 1 << 20
    a = _libc.mmap(None, size, PROT_RW, MAP_PRIV_ANON, -1, 0)
    assert a and a != C.c_void_p(-1).value
    try:
        c1 = R.Codec(0)
        dev = C.c_void_p()
        assert c1.lib.onc_host_register(c1.h, C.c_void_p(a), size, C.byref(dev)) == 0
        assert _pinned(a)
        C.memset(a, 0x77, size)
        c1.close()
        assert _pinned(a)                                   # the codec's end does not unpin it
        assert c1.lib.onc_host_unregister(None, C.c_void_p(a)) == 0
        assert not _pinned(a)
        # fresh pages at the same address
        assert _libc.munmap(C.c_void_p(a), size) == 0
        b = _libc.mmap(C.c_void_p(a), size, PROT_RW, MAP_PRIV_ANON | MAP_FIXED, -1, 0)
        assert b == a
        c2 = R.Codec(0)
        try:
            dev2 = C.c_void_p()
            assert c2.lib.onc_host_register(c2.h, C.c_void_p(a), size, C.byref(dev2)) == 0
            got, wire, off = _decode_golden_at(R, c2, a, dev2.value, golden)
            assert_decoded_equal(got, oracle.decode_batch(np.concatenate([wire, np.zeros(16, np.uint8)]), off,
                                                          L.DECODE_SLICE), "fresh pages")
            assert c2.lib.onc_host_unregister(c2.h, C.c_void_p(a)) == 0
        finally:
            c2.close()
    finally:
        _libc.munmap(C.c_void_p(a), size)


def test_hostmapped_close_after_codec_close(R):
    """runtime.HostMapped closed after its codec: unregistered all the same."""
    c = R.Codec(0)
    m = R.HostMapped(c, 1 << 16)
    addr = m._addr
    assert _pinned(addr)
    c.close()
    m.close()
    assert not _pinned(addr)


def test_registrations_are_counted(R):
    """Two codecs map one range: the first unregister leaves it pinned (the
    other codec still decodes from it), the second unpins it; an address
    inside the range finds it."""
    size = 1 << 18
    mm = mmap.mmap(-1, size)
    addr = np.frombuffer(mm, np.uint8).ctypes.data
    a, b = R.Codec(0), R.Codec(0)
    try:
        da, db_ = C.c_void_p(), C.c_void_p()
        assert a.lib.onc_host_register(a.h, C.c_void_p(addr), size, C.byref(da)) == 0
        assert b.lib.onc_host_register(b.h, C.c_void_p(addr + 4096), 4096, C.byref(db_)) == 0
        assert db_.value == da.value + 4096
        assert a.lib.onc_host_unregister(a.h, C.c_void_p(addr)) == 0
        assert _pinned(addr)
        assert b.lib.onc_host_unregister(b.h, C.c_void_p(addr + 4096)) == 0
        assert not _pinned(addr)
        assert a.lib.onc_host_unregister(a.h, C.c_void_p(addr)) == 0      # no longer recorded: a no-op
    finally:
        a.close()
        b.close()


def test_register_past_pinned_allocation(codec, R):
    """A range starting in pinned memory but running past its allocation
    (torch pin_memory, or a range this library pinned) is ONC_RC_EINVAL,
    not a mapping a kernel would read past."""
    import torch
    t = torch.zeros(8192, dtype=torch.uint8).pin_memory()
    dev = C.c_void_p()
    lib = codec.lib
    assert lib.onc_host_register(codec.h, C.c_void_p(t.data_ptr()), 8192, C.byref(dev)) == 0
    assert lib.onc_host_register(codec.h, C.c_void_p(t.data_ptr() + 4096), 1 << 20, C.byref(dev)) == -1
    m = R.HostMapped(codec, 1 << 16)
    try:
        assert lib.onc_host_register(codec.h, C.c_void_p(m._addr + 100), 1 << 16, C.byref(dev)) == -1
        assert lib.onc_host_register(codec.h, C.c_void_p(m._addr + 100), 1000, C.byref(dev)) == 0
        assert dev.value == m.data_ptr() + 100
        assert lib.onc_host_unregister(codec.h, C.c_void_p(m._addr + 100)) == 0
        assert _pinned(m._addr)
    finally:
        m.close()


# ---------------------------------------------------------------------------
# small batches: one launch, placement through LDS only
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("n", [1, 63, 64, 65, 300, 511, 512])
def test_small_batch_lds_placement(codec, R, oracle, n):
    """Batches of at most 512 records (enc_emit_single_kernel: one
    workgroup, its waves' tile totals exchanged through LDS): the oracle's
    bytes, offsets and statuses, placeholders included, at an odd writer
    position; twice in a row on one stream (the LDS flags are per launch)."""
    from test_gpu_emit_paths import _adversarial
    hb = _adversarial(109 + n, n=n) if n >= 64 else L.build_batch(S.random_messages(n, seed=110 + n))
    o_wire, o_off, o_st, _ = oracle.encode_batch(hb)
    for _ in range(2):
        out, off, st, total, _ = _device_encode(R, codec, hb, shift=5)
        assert out[5:5 + total].cpu().numpy().tobytes() == o_wire
        assert np.array_equal(off.cpu().numpy().view(np.uint64), o_off)
        assert np.array_equal(st.cpu().numpy()[:hb.n], o_st)


# ---------------------------------------------------------------------------
# the decode's round 1 (decode.hip load_round1): cooperative buffer loads,
# and the per-lane fallback when a wave's windows lie 2 GiB or more apart
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("policy", ["standard", "line"])
@pytest.mark.parametrize("mode", [L.DECODE_SLICE, L.DECODE_BYTES])
def test_decode_far_windows_fallback(R, oracle, policy, mode):
    """Record 0 is a valid Call whose payload makes it 2 GiB - 200 bytes
    long, so records 1-63 of its wave lie past the cooperative loader's
    2 GiB resource and the wave takes the per-lane path: the oracle's
    results, in both modes and policies. Records of the next waves (the
    cooperative path) check the same way."""
    import torch
    big = (1 << 31) - 200
    hb = S.mixed(200, seed=121, pmin=0, pmax=300, exotic=0.1)
    ws, offs, st, _ = oracle.encode_batch(hb)
    assert not st.any()
    h0, _, _, _ = oracle.encode_batch(S.call_none(1, 0, seed=122))     # a Call with no payload
    h0 = bytearray(h0)
    h0[0:4] = ((big - 4) | 0x80000000).to_bytes(4, "big")             # its payload: the rest of 2 GiB
    wire = np.zeros(big + len(ws) + 16, np.uint8)                      # zero pages: not touched
    wire[:len(h0)] = np.frombuffer(bytes(h0), np.uint8)
    wire[big:big + len(ws)] = np.frombuffer(ws, np.uint8)
    off = np.concatenate([[0], big + offs.astype(np.uint64)]).astype(np.uint64)
    pol = R.DECODE_POLICY_LINE if policy == "line" else R.DECODE_POLICY_STANDARD
    c = R.Codec(0, decode_policy=pol)
    try:
        got = R.decode_host_wire(c, wire, off, mode)
    finally:
        c.close()
    ora = oracle.decode_batch(wire, off, mode)
    assert ora[2][0] == 0 and int(ora[0]["payload_len"][0]) == big - len(h0)
    assert_decoded_equal(got, ora, f"far windows {policy}")
    del wire
    torch.cuda.empty_cache()


@pytest.mark.parametrize("policy", ["standard", "line"])
def test_decode_coop_short_and_empty_records(R, oracle, policy):
    """Waves mixing empty records, records shorter than one granule,
    records ending inside their first round and long headers, at odd
    starts: the cooperative loader hands every lane its own granules (none
    for an empty record), bit-exact against the oracle in both modes."""
    recs = []
    rng = np.random.default_rng(123)
    hb = S.mixed(400, seed=124, pmin=0, pmax=64, exotic=0.3)
    ws, offs, _, _ = oracle.encode_batch(hb)
    full = [bytes(ws[int(offs[i]):int(offs[i + 1])]) for i in range(hb.n)]
    for i in range(600):
        k = rng.integers(0, 5)
        r = full[i % hb.n]
        recs.append(b"" if k == 0 else r[:int(rng.integers(1, 16))] if k == 1 else
                    r[:int(rng.integers(16, 64))] if k == 2 else r)
    wire, off = L.records_from_wire(recs)
    w = np.concatenate([np.zeros(5, np.uint8), wire, np.zeros(16, np.uint8)])
    off = off.astype(np.uint64) + 5                                    # every record start shifted by 5
    pol = R.DECODE_POLICY_LINE if policy == "line" else R.DECODE_POLICY_STANDARD
    c = R.Codec(0, decode_policy=pol)
    try:
        for mode in (L.DECODE_SLICE, L.DECODE_BYTES):
            assert_decoded_equal(R.decode_host_wire(c, w, off, mode), oracle.decode_batch(w, off, mode),
                                 f"coop {policy} mode {mode}")
    finally:
        c.close()
