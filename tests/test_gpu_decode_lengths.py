"""onc_decode_lengths — the caller's length-delimited slices decoded in one
pass, offsets computed inside the decode (TryFrom<&[u8]> / TryFrom<Bytes>,
rpc_message.rs:235-314, over the rpc_message.rs:238-242 slicing contract) —
bit-exact against the CPU oracle and identical to onc_scan_lengths +
onc_decode, in both modes, with the block totals summed in the kernel
(<= 2M records) and scanned by a separate launch (forced here with
ONC_OPT_FORCE_SCAN), at a non-zero base offset, on corrupted records and at
workgroup / block boundaries."""
import numpy as np
import pytest

import _onc_pkg  # noqa: F401

_onc_pkg.load()
import onc_rpc_amd.layout as L  # noqa: E402
import onc_rpc_amd.synth as S  # noqa: E402

pytestmark = pytest.mark.gpu
MODES = [L.DECODE_SLICE, L.DECODE_BYTES]


@pytest.fixture(scope="module")
def R():
    import onc_rpc_amd.runtime as R
    return R


@pytest.fixture(scope="module", params=["fused", "scan"])
def codec(request, R):
    import os
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    c = R.Codec(0, force_scan=request.param == "scan")
    yield c
    c.close()


def _decode_lengths(R, codec, wire, lens, base, mode):
    import torch
    n = len(lens)
    w = R.to_device(np.frombuffer(bytes(wire) + b"\0" * 16, np.uint8), "cuda")
    rl = torch.from_numpy(np.asarray(lens, np.uint32).view(np.int32).copy()).to("cuda")
    off = torch.full((n + 1,), -1, dtype=torch.int64, device="cuda")
    bufs = R.DecodeBuffers(n)
    codec.decode_lengths(w, rl, n, base, mode, bufs.msgs, bufs.unix, bufs.status, bufs.aux0, bufs.aux1, rec_off=off)
    codec.sync()
    return bufs.to_host(), off.cpu().numpy().view(np.uint64)


def _batches():
    out = []
    hb = S.mixed(9000, seed=51, pmin=0, pmax=700, exotic=0.2)
    out.append(("mixed", hb))
    out.append(("random", L.build_batch(S.random_messages(3000, seed=52, max_payload=300))))
    out.append(("unix16", S.call_unix16(4100, 64, seed=53)))
    return out


@pytest.mark.parametrize("base", [0, 7])
def test_decode_lengths_matches_oracle(codec, R, oracle, base):
    for name, hb in _batches():
        o_wire, o_off, o_st, _ = oracle.encode_batch(hb)
        w, off = S.corrupt(np.frombuffer(o_wire, np.uint8), o_off, frac=0.05, seed=54)
        wire = bytes(base) + w.tobytes()
        lens = np.diff(off.astype(np.int64)).astype(np.uint32)
        for mode in MODES:
            g, g_off = _decode_lengths(R, codec, wire, lens, base, mode)
            ow = np.frombuffer(wire + b"\0" * 16, np.uint8).copy()
            o = oracle.decode_batch(ow, off.astype(np.uint64) + np.uint64(base), mode)
            assert np.array_equal(g_off, off.astype(np.uint64) + np.uint64(base)), name
            assert np.array_equal(g[2], o[2]), name
            assert np.array_equal(g[3], o[3]) and np.array_equal(g[4], o[4]), name
            assert np.array_equal(g[0].view(np.uint8), o[0].view(np.uint8)), name
            # AUTH_UNIX parameters at their packed refs (descriptors equal above)
            _, gp = L.resolve_unix(g[0], g[1], g[2])
            _, op = L.resolve_unix(o[0], o[1], o[2])
            assert np.array_equal(gp, op), name


@pytest.mark.parametrize("n", [1, 63, 64, 65, 4095, 4096, 4097, 12345])
def test_decode_lengths_same_as_scan_then_decode(codec, R, oracle, n):
    """Workgroup (64) and block (4096) boundaries: identical outputs to
    onc_scan_lengths + onc_decode."""
    import torch
    hb = S.mixed(n, seed=55 + n, pmin=0, pmax=200, exotic=0.1)
    o_wire, o_off, _, _ = oracle.encode_batch(hb)
    lens = np.diff(o_off.astype(np.int64)).astype(np.uint32)
    for mode in MODES:
        g, g_off = _decode_lengths(R, codec, o_wire, lens, 0, mode)
        rl = torch.from_numpy(lens.view(np.int32).copy()).to("cuda")
        off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        codec.scan_lengths(rl, n, 0, off)
        codec.sync()
        h = R.decode_host_wire(codec, np.frombuffer(o_wire + b"\0" * 16, np.uint8), off.cpu().numpy().view(np.uint64),
                               mode)
        assert np.array_equal(g_off, o_off)
        for k in (0, 2, 3, 4):          # unix slots are defined only for AUTH_UNIX records
            assert np.array_equal(np.asarray(g[k]).view(np.uint8), np.asarray(h[k]).view(np.uint8)), k


@pytest.mark.parametrize("n", [1, 2, 33, 64])
def test_decode_lengths_one_workgroup(codec, R, oracle, n):
    """One decode workgroup (n <= 64) launches the decode alone (no
    dlen_tiles): offsets from its own scan, at a non-zero base, corrupted
    records included, equal to the oracle in both modes."""
    hb = S.mixed(n, seed=70 + n, pmin=0, pmax=300, exotic=0.3)
    o_wire, o_off, _, _ = oracle.encode_batch(hb)
    w, off = S.corrupt(np.frombuffer(o_wire, np.uint8), o_off, frac=0.2, seed=71 + n)
    base = 5
    wire = bytes(base) + w.tobytes()
    lens = np.diff(off.astype(np.int64)).astype(np.uint32)
    for mode in MODES:
        g, g_off = _decode_lengths(R, codec, wire, lens, base, mode)
        o = oracle.decode_batch(np.frombuffer(wire + b"\0" * 16, np.uint8).copy(), off.astype(np.uint64) + np.uint64(base),
                                mode)
        assert np.array_equal(g_off, off.astype(np.uint64) + np.uint64(base))
        assert np.array_equal(g[2], o[2]) and np.array_equal(g[3], o[3]) and np.array_equal(g[4], o[4])
        assert np.array_equal(g[0].view(np.uint8), o[0].view(np.uint8))
        _, gp = L.resolve_unix(g[0], g[1], g[2])
        _, op = L.resolve_unix(o[0], o[1], o[2])
        assert np.array_equal(gp, op)
