"""GPU tests, round 4: onc_encode + onc_decode captured into a hipGraph
(torch.cuda.CUDAGraph) after onc_codec_reserve and replayed on new inputs,
including the chunked encode and the lengths-driven decode; a call that would
grow the scratch inside a capture is refused (ONC_RC_ECAPTURE); codec
options instead of environment variables. Bit-exact against the CPU oracle."""
import numpy as np
import pytest

import onc_rpc_amd.layout as L
import onc_rpc_amd.synth as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def R():
    import onc_rpc_amd.runtime as R
    return R


class _Slots:
    """Fixed device buffers a captured graph reads: every new batch is copied
    into their prefixes (the rest zero), so the pointers and the declared
    arena sizes of the captured onc_batch stay valid."""

    def __init__(self, R, n, unix_cap, auth_cap, pay_cap, out_cap):
        import torch
        self.n = n
        self.msgs = torch.zeros(64 * n, dtype=torch.uint8, device="cuda")
        self.unix = torch.zeros(96 * max(unix_cap, 1), dtype=torch.uint8, device="cuda")
        self.auth = torch.zeros(max(auth_cap, 16), dtype=torch.uint8, device="cuda")
        self.pay = torch.zeros(max(pay_cap, 16), dtype=torch.uint8, device="cuda")
        self.db = R.DeviceBatch(n, self.msgs, self.unix, self.auth, self.pay)
        self.out = torch.zeros(out_cap, dtype=torch.uint8, device="cuda")
        self.off = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
        self.st = torch.zeros(n, dtype=torch.int32, device="cuda")
        self.rl = torch.zeros(n, dtype=torch.int32, device="cuda")
        self.doff = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
        self.dec = R.DecodeBuffers(n)

    def load(self, hb):
        import torch
        for dst, arr in ((self.msgs, hb.msgs), (self.unix, hb.unix), (self.auth, hb.auth_arena),
                         (self.pay, hb.payload_arena)):
            raw = torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8).reshape(-1).copy())
            assert raw.numel() <= dst.numel()
            dst.zero_()
            dst[:raw.numel()].copy_(raw)
        self.out.fill_(0xA5)
        torch.cuda.synchronize()


def _batches(kind, n, seeds):
    if kind == "call_none":
        return [S.call_none(n, 256, seed=s, first_xid=1000 * s) for s in seeds]
    if kind == "unix16":
        return [S.call_unix16(n, 40 + 8 * (s % 3), seed=s) for s in seeds]
    return [S.mixed(n, seed=s, pmin=0, pmax=300, exotic=0.2) for s in seeds]


def _caps(hbs, oracle):
    tot = max(len(oracle.encode_batch(hb)[0]) for hb in hbs)
    return (max(len(hb.unix) for hb in hbs), max(hb.auth_arena.nbytes for hb in hbs),
            max(hb.payload_arena.nbytes for hb in hbs), tot + 64)


@pytest.mark.parametrize("kind,n,opts,lengths", [
    ("call_none", 20_000, {}, False),
    ("call_none", 1_100_000, {}, True),                  # above one 1M-record plan chunk
    ("mixed", 9_001, {"enc_chunk": 2048}, True),          # the chunked encode: chunk k+1 reads k's end
    ("unix16", 5_000, {"enc_chunk": 2048, "variant": 0x400}, True),   # the emit reads the plan's lengths
    ("mixed", 6_000, {"decode_policy": 2}, False),
])
def test_graph_capture_replay_new_inputs(R, oracle, kind, n, opts, lengths):
    """Capture encode -> decode (or encode -> decode_lengths from the plan's
    record lengths) on the codec's stream after onc_codec_reserve, then
    replay the graph on four batches copied into the same buffers: every
    replay bit-exact vs the oracle (wire bytes, offsets, statuses, decoded
    descriptors, AUTH_UNIX slots, aux words)."""
    import torch
    hbs = _batches(kind, n, [11, 12, 13] if n > 100_000 else [11, 12, 13, 14, 15])
    slots = _Slots(R, n, *_caps(hbs, oracle))
    s = torch.cuda.Stream()
    codec = R.Codec(0, stream=s.cuda_stream, **opts)
    try:
        codec.reserve(n)
        if "decode_policy" not in opts:
            codec.set_decode_policy(R.DECODE_POLICY_LINE if kind == "unix16" else R.DECODE_POLICY_STANDARD)
        mode = L.DECODE_BYTES if lengths else L.DECODE_SLICE
        d = slots.dec

        def work():
            codec.encode(slots.db, slots.out, slots.off, slots.st, slots.rl)
            if lengths:
                codec.decode_lengths(slots.out, slots.rl, n, 0, mode, d.msgs, d.unix, d.status, d.aux0, d.aux1,
                                     rec_off=slots.doff)
            else:
                codec.decode(slots.out, slots.off, n, mode, d.msgs, d.unix, d.status, d.aux0, d.aux1)

        slots.load(hbs[0])
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            work()                                   # warm-up outside the capture
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            work()
        torch.cuda.synchronize()
        for hb in hbs[1:]:
            slots.load(hb)
            g.replay()
            torch.cuda.synchronize()
            o_wire, o_off, o_st, o_len = oracle.encode_batch(hb)
            total = len(o_wire)
            assert np.array_equal(slots.st.cpu().numpy(), o_st)
            assert np.array_equal(slots.off.cpu().numpy().view(np.uint64), o_off)
            assert np.array_equal(slots.rl.cpu().numpy().view(np.uint32), o_len)
            ob = slots.out.cpu().numpy()
            assert ob[:total].tobytes() == o_wire and (ob[total:] == 0xA5).all()
            w = np.concatenate([np.frombuffer(o_wire, np.uint8), np.zeros(16, np.uint8)])
            om, ou, os_, oa0, oa1 = oracle.decode_batch(w, o_off, mode)
            gm, gu, gs, ga0, ga1 = d.to_host()
            assert np.array_equal(gs, os_) and np.array_equal(ga0, oa0) and np.array_equal(ga1, oa1)
            assert np.array_equal(gm.view(np.uint8), om.view(np.uint8))
            _, gp = L.resolve_unix(gm, gu, gs)
            _, op = L.resolve_unix(om, ou, os_)
            assert np.array_equal(gp, op)
            if lengths:
                assert np.array_equal(slots.doff.cpu().numpy().view(np.uint64), o_off)
    finally:
        codec.close()


def test_growth_inside_a_capture_is_refused(R):
    """Without onc_codec_reserve the first encode would allocate scratch: in
    a capture it returns ONC_RC_ECAPTURE (no allocation, no synchronisation
    inside the capture), and the same call works after reserve."""
    import torch
    hb = S.call_none(3000, 64, seed=3)
    db = R.DeviceBatch.from_host(hb)
    out = torch.zeros(3000 * 128, dtype=torch.uint8, device="cuda")
    off = torch.zeros(3001, dtype=torch.int64, device="cuda")
    st = torch.zeros(3000, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    codec = R.Codec(0, stream=s.cuda_stream)
    try:
        g = torch.cuda.CUDAGraph()
        err = None
        with torch.cuda.graph(g, stream=s):
            try:
                codec.encode(db, out, off, st)
            except R.CodecError as e:
                err = str(e)
        assert err is not None and "rc=-5" in err, err
        codec.reserve(3000)
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2, stream=s):
            codec.encode(db, out, off, st)
        g2.replay()
        torch.cuda.synchronize()
        assert (st.cpu().numpy() == 0).all()
        assert int(off[3000]) == int(R.codec_lengths(codec, db).sum())
    finally:
        codec.close()


def test_codec_options_validated(R):
    """onc_codec_create_ex refuses an unknown flag, a decode policy out of
    range and a framing chunk under 64 bytes; set_decode_policy likewise."""
    with pytest.raises(R.CodecError):
        R.Codec(0, decode_policy=3)
    with pytest.raises(R.CodecError):
        R.Codec(0, frame_chunk=32)
    c = R.Codec(0)
    try:
        with pytest.raises(R.CodecError):
            c.set_decode_policy(7)
        c.set_decode_policy(R.DECODE_POLICY_LINE)
    finally:
        c.close()


def test_two_codecs_on_two_streams_concurrently(R, oracle):
    """Two codecs, each on its own stream, encode and decode different
    batches with their work interleaved on the device: a configs[1]-shaped
    batch (the wave-specialised kernel, a persistent grid of 1024
    workgroups — two such grids cannot both be resident, and neither waits
    on the other's workgroups) and a configs[0]-shaped one (the
    wave-per-tile kernel). Each codec's scratch and decode policy are its
    own (include/onc_rpc.h: one handle per stream); every output bit-exact
    vs the oracle."""
    import torch
    batches = [S.call_none(150_000, 256, seed=71), S.cpu_roundtrip(60_000, seed=72)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    codecs = [R.Codec(0, stream=s.cuda_stream) for s in streams]
    try:
        bufs = []
        for hb, c in zip(batches, codecs):
            db = R.DeviceBatch.from_host(hb)
            o_wire = oracle.encode_batch(hb)[0]
            out = torch.zeros(len(o_wire) + 64, dtype=torch.uint8, device="cuda")
            off = torch.zeros(hb.n + 1, dtype=torch.int64, device="cuda")
            st = torch.zeros(hb.n, dtype=torch.int32, device="cuda")
            c.reserve(hb.n)
            bufs.append((hb, db, out, off, st, R.DecodeBuffers(hb.n)))
        torch.cuda.synchronize()
        for _ in range(3):
            for k in (0, 1):                       # enqueue both encodes, then both decodes
                hb, db, out, off, st, d = bufs[k]
                codecs[k].encode(db, out, off, st)
            for k in (0, 1):
                hb, db, out, off, st, d = bufs[k]
                codecs[k].decode(out, off, hb.n, L.DECODE_SLICE, d.msgs, d.unix, d.status, d.aux0, d.aux1)
        torch.cuda.synchronize()
        for hb, db, out, off, st, d in bufs:
            o_wire, o_off, o_st, _ = oracle.encode_batch(hb)
            assert np.array_equal(st.cpu().numpy(), o_st)
            assert np.array_equal(off.cpu().numpy().view(np.uint64), o_off)
            assert out[:len(o_wire)].cpu().numpy().tobytes() == o_wire
            w = np.concatenate([np.frombuffer(o_wire, np.uint8), np.zeros(16, np.uint8)])
            om, ou, os_, oa0, oa1 = oracle.decode_batch(w, o_off, L.DECODE_SLICE)
            gm, gu, gs, ga0, ga1 = d.to_host()
            assert np.array_equal(gs, os_) and np.array_equal(ga0, oa0) and np.array_equal(ga1, oa1)
            assert np.array_equal(gm.view(np.uint8), om.view(np.uint8))
            _, gp = L.resolve_unix(gm, gu, gs)
            _, op = L.resolve_unix(om, ou, os_)
            assert np.array_equal(gp, op)
    finally:
        for c in codecs:
            c.close()
