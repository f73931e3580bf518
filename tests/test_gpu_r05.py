"""GPU tests, round 5 (ABI 7).

* Host-mapped buffers (onc_host_register): a wire that lives in host memory —
  a socket buffer — decoded in place, the kernels fetching only the header
  granules they parse over PCIe (the zero-copy decode of call_body.rs:53-59,
  opaque.rs:92-97), with the outputs in device or in mapped host memory; the
  encode reading its descriptors and arenas in place. Every result equal to
  the oracle's and to the device-resident call's, in both decode modes, on
  the reference's golden vectors, corrupted records and configs[2]-shaped
  batches.
* The framable placeholder of a declared AUTH_UNIX record failing its
  deferred block check: the encoded stream frames record by record
  (expected_message_len, rpc_message.rs:343-367 — onc_frame_stream and the
  oracle's serial loop) and every OK record after such a record decodes; the
  vectored encode gathers to the same bytes.
* onc_encode_plan of more records than one plan chunk inside a capture
  (onc_codec_reserve sizes the plan's lengths for it).
* configs[4]'s device byte check (bench.c4_wire_bytes_ok) across its chunk
  boundaries at 9M records, and that it catches a wrong byte.
"""
import ctypes as C
import os
import sys

import numpy as np
import pytest

import onc_rpc_amd.layout as L
import onc_rpc_amd.synth as S
from test_gpu_parity import all_golden_records, assert_decoded_equal

pytestmark = pytest.mark.gpu

MODES = [L.DECODE_SLICE, L.DECODE_BYTES]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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


class _MappedOut:
    """Decode outputs in mapped host memory (the kernels write them there)."""

    def __init__(self, R, codec, n):
        m = max(n, 1)
        self.n = n
        self.msgs = R.HostMapped(codec, 64 * m)
        self.unix = R.HostMapped(codec, 2 * 96 * m)
        self.status = R.HostMapped(codec, 4 * m)
        self.aux0 = R.HostMapped(codec, 4 * m)
        self.aux1 = R.HostMapped(codec, 4 * m)
        for b in (self.msgs, self.unix, self.status, self.aux0, self.aux1):
            b.host[:] = 0xEE                       # everything the decode defines is overwritten

    def to_host(self):
        n = self.n
        return (self.msgs.view(L.MSG_DTYPE)[:n].copy(), self.unix.view(L.UNIX_DTYPE)[:2 * n].copy(),
                self.status.view(np.int32)[:n].copy(), self.aux0.view(np.uint32)[:n].copy(),
                self.aux1.view(np.uint32)[:n].copy())

    def close(self):
        for b in (self.msgs, self.unix, self.status, self.aux0, self.aux1):
            b.close()


def mapped_decode(R, codec, wire, off, mode, out_mapped=True, lengths=False):
    """Decode `wire` (numpy bytes, records at off) from mapped host memory in
    place: onc_decode from offsets or onc_decode_lengths from lengths (also
    in mapped memory), outputs mapped or in device memory."""
    n = len(off) - 1
    w = R.HostMapped.from_array(codec, np.concatenate([np.asarray(wire, np.uint8), np.zeros(16, np.uint8)]))
    out = _MappedOut(R, codec, n) if out_mapped else R.DecodeBuffers(n)
    d = out
    try:
        if lengths:
            rl = R.HostMapped.from_array(codec, np.diff(off.astype(np.int64)).astype(np.uint32))
            ro = R.HostMapped(codec, 8 * (n + 1))
            codec.decode_lengths(w, rl, n, 0, mode, d.msgs, d.unix, d.status, d.aux0, d.aux1, rec_off=ro)
            codec.sync()
            assert np.array_equal(ro.view(np.uint64)[:n + 1], off.astype(np.uint64))
            rl.close()
            ro.close()
        else:
            o = R.HostMapped.from_array(codec, off.astype(np.uint64))
            codec.decode(w, o, n, mode, d.msgs, d.unix, d.status, d.aux0, d.aux1)
            codec.sync()
            o.close()
        return out.to_host()
    finally:
        w.close()
        if out_mapped:
            out.close()


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("out_mapped,lengths", [(True, False), (False, False), (True, True)])
def test_mapped_wire_decode_golden_and_corrupted(codec, R, oracle, golden, mode, out_mapped, lengths):
    """Every golden record (aligned and misaligned) and a corrupted-record
    batch, decoded from mapped host memory: the oracle's statuses, aux words,
    descriptors and AUTH_UNIX slots."""
    recs, _ = all_golden_records(golden)
    wire, off = L.records_from_wire(recs + recs)
    assert_decoded_equal(mapped_decode(R, codec, wire, off, mode, out_mapped, lengths),
                         oracle.decode_batch(wire, off, mode), "golden")
    hb = L.build_batch(S.random_messages(3000, seed=61, max_payload=300))
    w, o, _, _ = oracle.encode_batch(hb)
    cw, coff = S.corrupt(np.frombuffer(w + b"\0" * 16, np.uint8), o, frac=0.6, seed=62 + mode)
    assert_decoded_equal(mapped_decode(R, codec, cw, coff, mode, out_mapped, lengths),
                         oracle.decode_batch(cw, coff, mode), "corrupted")


@pytest.mark.parametrize("mode", MODES)
def test_mapped_wire_decode_configs2(codec, R, oracle, mode):
    """A configs[2]-shaped batch (mixed Call/Reply, payloads 64..4096 B) in
    mapped host memory, decoded in place with onc_decode_lengths into mapped
    outputs: equal to the device-resident decode of the same bytes and to the
    oracle."""
    hb = S.mixed(40_000, seed=63)
    w, off, st, _ = oracle.encode_batch(hb)
    assert (st == 0).all()
    wire = np.frombuffer(w, np.uint8)
    g_map = mapped_decode(R, codec, wire, off, mode, out_mapped=True, lengths=True)
    g_dev = R.decode_host_wire(codec, np.concatenate([wire, np.zeros(16, np.uint8)]), off, mode)
    assert_decoded_equal(g_map, g_dev, "mapped vs device")
    assert_decoded_equal(g_map, oracle.decode_batch(np.concatenate([wire, np.zeros(16, np.uint8)]), off, mode),
                         "mapped vs oracle")


def test_mapped_pinned_torch_tensor(codec, R, oracle):
    """A wire in torch pinned memory (hipHostMalloc): onc_host_register maps
    it without registering it again (unregister is then a no-op) and the
    decode reads it in place."""
    import torch
    hb = S.call_unix16(5000, 100, seed=64)
    w, off, _, _ = oracle.encode_batch(hb)
    raw = np.frombuffer(w + b"\0" * 16, np.uint8)
    t = torch.from_numpy(raw.copy()).pin_memory()
    dptr = R.host_device_pointer(codec, t)
    assert codec.lib.onc_host_unregister(codec.h, C.c_void_p(t.data_ptr())) == 0

    class _P:                                   # a device address for the binding
        def data_ptr(self):
            return dptr
    n = hb.n
    d = R.DecodeBuffers(n)
    o = torch.from_numpy(off.astype(np.uint64).view(np.int64).copy()).cuda()
    codec.decode(_P(), o, n, L.DECODE_SLICE, d.msgs, d.unix, d.status, d.aux0, d.aux1)
    codec.sync()
    assert_decoded_equal(d.to_host(), oracle.decode_batch(raw, off, L.DECODE_SLICE), "pinned")


def test_mapped_encode_inputs_and_outputs(codec, R, oracle):
    """The encode with its descriptors, AUTH_UNIX table and arenas read in
    place from mapped host memory, writing the wire straight into a mapped
    send buffer at an odd writer position; and the vectored encode with
    mapped inputs and outputs: the oracle's bytes."""
    hb = L.build_batch(S.random_messages(6000, seed=65, max_payload=700))
    o_wire, o_off, o_st, o_len = oracle.encode_batch(hb)
    mb = R.MappedHostBatch(codec, hb)
    total = len(o_wire)
    out = R.HostMapped(codec, total + 64)
    out.host[:] = 0x5A
    rec_off = R.HostMapped(codec, 8 * (hb.n + 1))
    st = R.HostMapped(codec, 4 * hb.n)

    class _At:                                  # out + 3: any writer position
        def __init__(self, m, k):
            self.m, self.k = m, k

        def data_ptr(self):
            return self.m.data_ptr() + self.k

        def numel(self):
            return self.m.numel() - self.k
    try:
        codec.encode(mb, _At(out, 3), rec_off, st, out_cap=total)
        codec.sync()
        assert np.array_equal(st.view(np.int32)[:hb.n], o_st)
        assert np.array_equal(rec_off.view(np.uint64)[:hb.n + 1], o_off)
        b = out.host
        assert b[3:3 + total].tobytes() == o_wire
        assert (b[:3] == 0x5A).all() and (b[3 + total:] == 0x5A).all()
        # vectored: headers + iovecs + statuses into mapped memory
        hdr = R.HostMapped(codec, total + 16)
        iov = R.HostMapped(codec, 32 * hb.n)
        ist = R.HostMapped(codec, 4 * hb.n)
        tot = R.HostMapped(codec, 16)
        codec.encode_iov(mb, hdr, iov, ist, tot, hdr_cap=total)
        codec.sync()
        e = iov.view(L.IOV_DTYPE)[:hb.n]
        assert np.array_equal(ist.view(np.int32)[:hb.n], o_st)
        assert np.array_equal(e["wire_off"], o_off[:-1])
        assert gather_iov(hb, hdr.host, e) == o_wire
        for m in (hdr, iov, ist, tot):
            m.close()
    finally:
        for m in (out, rec_off, st):
            m.close()
        mb.close()


def gather_iov(hb, hdr, e):
    """The bytes a writev of every iovec pair sends (record order)."""
    parts = []
    for i in range(len(e)):
        h0, hl = int(e["hdr_off"][i]), int(e["hdr_len"][i])
        p0, pl = int(e["payload_off"][i]), int(e["payload_len"][i])
        parts.append(bytes(hdr[h0:h0 + hl]))
        parts.append(hb.payload_arena[p0:p0 + pl].tobytes())
    return b"".join(parts)


def test_host_register_contract(codec, R):
    """EINVAL for a NULL pointer or length; unregister of a range it did not
    pin is a no-op; a registered range unpins once."""
    lib = codec.lib
    dev = C.c_void_p()
    assert lib.onc_host_register(codec.h, None, 64, C.byref(dev)) == -1
    buf = np.zeros(8192, np.uint8)
    assert lib.onc_host_register(codec.h, C.c_void_p(buf.ctypes.data), 0, C.byref(dev)) == -1
    assert lib.onc_host_unregister(codec.h, C.c_void_p(buf.ctypes.data)) == 0       # never registered
    m = R.HostMapped(codec, 1 << 20)
    assert m.data_ptr()
    m.close()
    m.close()                                   # idempotent


# ---------------------------------------------------------------------------
# framable placeholders (ABI 7)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("variant,frame_chunk", [(0, 0), (0x200, 1024), (0x400, 0), (0x400 | 0x20000, 64)])
def test_placeholder_keeps_stream_framable(R, oracle, variant, frame_chunk):
    """An encode output with records whose declared credentials fail their
    deferred checks (every emit path: ws, wave-per-tile reading the plan's
    lengths, wave-per-tile re-planning): the oracle's bytes; framed on the
    device (onc_frame_stream, 64 B / 1 KiB / 64 KiB chunks) and by the
    oracle's serial expected_message_len loop into exactly the records with
    an extent; every OK record decodes to its descriptor's values and every
    placeholder to InvalidRpcVersion(0)."""
    import torch
    from test_gpu_emit_paths import _adversarial
    hb = _adversarial(81 + variant % 7, n=3000)
    o_wire, o_off, o_st, o_len = oracle.encode_batch(hb)
    holes = (o_st != 0) & (o_len != 0)
    assert holes.sum() > 50
    c = R.Codec(0, variant=variant, frame_chunk=frame_chunk)
    try:
        db = R.DeviceBatch.from_host(hb)
        total = len(o_wire)
        out = torch.zeros(total + 64, dtype=torch.uint8, device="cuda")
        off = torch.empty(hb.n + 1, dtype=torch.int64, device="cuda")
        st = torch.empty(hb.n, dtype=torch.int32, device="cuda")
        c.encode(db, out, off, st, out_cap=total)
        c.sync()
        assert np.array_equal(st.cpu().numpy(), o_st)
        assert out[:total].cpu().numpy().tobytes() == o_wire
        has = o_len != 0
        want = np.concatenate([o_off[:-1][has], [total]]).astype(np.uint64)
        fo, n, consumed, fst, _, _ = R.frame_host_stream(c, o_wire)
        assert (n, consumed, fst) == (int(has.sum()), total, 0)
        assert np.array_equal(fo, want)
        ofo, on_, ocons, ost = oracle.frame_stream(o_wire)[:4]
        assert (on_, ocons, ost) == (n, total, 0) and np.array_equal(np.asarray(ofo)[:n + 1], want)
        # decode of the framed records
        w = np.frombuffer(o_wire + b"\0" * 16, np.uint8)
        gm, gu, gs, ga0, ga1 = R.decode_host_wire(c, w, fo, L.DECODE_SLICE)
        kept = np.nonzero(has)[0]
        assert np.array_equal(gs == 0, o_st[kept] == 0)
        bad = o_st[kept] != 0
        assert (gs[bad] == 11).all() and (ga0[bad] == 0).all()      # InvalidRpcVersion(0)
        assert np.array_equal(gm["xid"][~bad], hb.msgs["xid"][kept][~bad])
        assert np.array_equal(gm["payload_len"][~bad], hb.msgs["payload_len"][kept][~bad])
    finally:
        c.close()


def test_iov_placeholder_gathers_encode_bytes(codec, R, oracle):
    """The vectored encode of the same adversarial batch: its iovecs gather
    to onc_encode's bytes for every record with an extent, placeholders
    included (header iovec = the placeholder, payload slice in place)."""
    from test_gpu_emit_paths import _adversarial
    from test_gpu_iov import gpu_iov
    hb = _adversarial(86, n=2500)
    o_wire, o_off, o_st, o_len = oracle.encode_batch(hb)
    hdr, iov, st, tot = gpu_iov(R, codec, hb)
    assert np.array_equal(st, o_st)
    assert np.array_equal(iov["wire_off"], o_off[:-1])
    assert int(tot[1]) == int(o_off[-1])
    assert np.array_equal(iov["hdr_len"].astype(np.int64) + iov["payload_len"], o_len)
    assert gather_iov(hb, hdr, iov) == o_wire


# ---------------------------------------------------------------------------
def test_plan_past_a_chunk_inside_a_capture(R, oracle):
    """onc_encode_plan plans the whole batch at once: after onc_codec_reserve
    a plan of more records than one plan chunk (enc_chunk 2048, 5000
    records, AUTH_UNIX: the emit reads the plan's lengths) is captured and
    replayed without ONC_RC_ECAPTURE, bit-exact vs the oracle."""
    import torch
    hb = S.call_unix16(5000, 40, seed=66)
    o_wire, o_off, o_st, _ = oracle.encode_batch(hb)
    s = torch.cuda.Stream()
    c = R.Codec(0, stream=s.cuda_stream, enc_chunk=2048, variant=0x400)
    try:
        c.reserve(hb.n)
        db = R.DeviceBatch.from_host(hb)
        out = torch.full((len(o_wire) + 64,), 0xA5, dtype=torch.uint8, device="cuda")
        off = torch.zeros(hb.n + 1, dtype=torch.int64, device="cuda")
        st = torch.zeros(hb.n, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            c.encode_plan(db, st)
            c.encode_emit(db, out, off, st)
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(st.cpu().numpy(), o_st)
        assert np.array_equal(off.cpu().numpy().view(np.uint64), o_off)
        assert out[:len(o_wire)].cpu().numpy().tobytes() == o_wire
    finally:
        c.close()


def test_c4_device_byte_check_across_chunks(R):
    """bench.py's configs[4] device check (c4_wire_bytes_ok) over a 9M-record
    shard (two 4M-record comparison chunks and a ragged third, the encode's
    1M-record plan chunks) after a real encode, starting at a nonzero first
    xid; and it reports a single wrong byte in the last chunk."""
    import torch
    sys.path.insert(0, ROOT)
    import bench
    lo, n = 3_000_000, 9_000_000
    db, _ = S.call_none_device(lo, lo + n, 256, seed=4, device=torch.device("cuda", 0))
    c = R.Codec(0)
    try:
        c.reserve(n)
        out = torch.empty(n * 300 + 16, dtype=torch.uint8, device="cuda")
        off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        st = torch.empty(n, dtype=torch.int32, device="cuda")
        c.encode(db, out, off, st)
        c.sync()
        assert int((st != 0).sum()) == 0 and int(off[n]) == n * 300
        assert bench.c4_wire_bytes_ok(torch, out, db, lo, n)
        out[(n - 5) * 300 + 7] ^= 1                 # an xid byte of a record in the last chunk
        assert not bench.c4_wire_bytes_ok(torch, out, db, lo, n)
        out[(n - 5) * 300 + 7] ^= 1
        out[(n - 2) * 300 + 100] ^= 0x80            # a payload byte
        assert not bench.c4_wire_bytes_ok(torch, out, db, lo, n)
    finally:
        c.close()
        del db
        torch.cuda.empty_cache()


# ---------------------------------------------------------------------------
# small batches (<= 512 records): one enc_emit_single_kernel launch, no
# length pass (codec.hip small_batch) — the default path, every content kind
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 300, 511, 512, 513])
def test_small_batch_one_launch_bit_exact(R, oracle, n):
    """Batches up to 512 records encode in one launch (the workgroup's waves
    place their tiles through LDS); at and around the tile and workgroup
    boundaries they give the oracle's bytes, offsets, statuses and lengths for
    adversarial content (failing and declared AUTH_UNIX records, placeholders)
    and for configs[0]'s message, at two writer positions and with a capacity
    inside the batch; 513 records take the two-pass path."""
    from test_gpu_emit_paths import _enc_oracle_sized, _adversarial
    c = R.Codec(0)
    try:
        for hb in (_adversarial(97 + n, n=n), S.cpu_roundtrip(n)):
            o_st, o_len = _enc_oracle_sized(R, c, hb, oracle)
            _enc_oracle_sized(R, c, hb, oracle, shift=7)
            total = int(o_len.astype(np.int64).sum())
            if total > 8:
                _enc_oracle_sized(R, c, hb, oracle, shift=1, cap=total // 2 + 3)
    finally:
        c.close()


@pytest.mark.parametrize("n", [3, 200, 512, 600])
def test_small_batch_capacity_zero_and_tiny(R, oracle, n):
    """onc_encode with no output room (out_cap 0) and with room for a few
    bytes: every record that does not fit gets ONC_ENC_WRITE_ZERO and the
    offsets still place every record — on the one-launch path (n <= 512) as
    on the two-pass one, against the oracle."""
    import torch
    hb = S.cpu_roundtrip(n)
    db = R.DeviceBatch.from_host(hb)
    c = R.Codec(0)
    try:
        for cap in (0, 5, 200):
            o_wire, o_off, o_st, o_len = oracle.encode_batch(hb, out_cap=cap)
            buf = torch.full((cap + 64,), 0x5A, dtype=torch.uint8, device="cuda")
            off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
            st = torch.empty(n, dtype=torch.int32, device="cuda")
            c.encode(db, buf, off, st, out_cap=cap)
            c.sync()
            assert np.array_equal(st.cpu().numpy(), o_st)
            assert np.array_equal(off.cpu().numpy().view(np.uint64), o_off)
            b = buf.cpu().numpy()
            assert b[:len(o_wire)].tobytes() == o_wire and (b[cap:] == 0x5A).all()
    finally:
        c.close()
