"""Vectored encode (onc_encode_iov) at iov_len
workgroup boundaries and beyond the fused-base limit (> 1024 workgroups of
1024 records: the two scan launches place the workgroups), bit-exact against
the oracle's contiguous wire (rpc_message.rs:136-164 per record)."""
import numpy as np
import pytest

import _onc_pkg

_onc_pkg.load()
import onc_rpc_amd.layout as L  # noqa: E402
import onc_rpc_amd.synth as S  # noqa: E402

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


def gpu_iov(R, codec, hb):
    import torch
    db = R.DeviceBatch.from_host(hb, "cuda")
    n = hb.n
    cap = int(R.codec_lengths(codec, db).sum())
    hdr = torch.zeros(cap + 16, dtype=torch.uint8, device="cuda")
    iov = torch.zeros(max(1, n) * 32, dtype=torch.uint8, device="cuda")
    st = torch.full((max(1, n),), -1, dtype=torch.int32, device="cuda")
    tot = torch.zeros(2, dtype=torch.int64, device="cuda")
    codec.encode_iov(db, hdr, iov, st, tot, hdr_cap=cap)
    codec.sync()
    return (hdr.cpu().numpy(), iov.cpu().numpy().view(L.IOV_DTYPE)[:n], st.cpu().numpy()[:n],
            tot.cpu().numpy().view(np.uint64))


def reassemble(hb, hdr, iov, st):
    """The wire writev would send: every accepted record's header slice then
    its payload slice, vectorised (record order = wire order)."""
    ok = st == 0
    e = iov[ok]
    hl = e["hdr_len"].astype(np.int64)
    pl = e["payload_len"].astype(np.int64)
    ho = e["hdr_off"].astype(np.int64)
    po = e["payload_off"].astype(np.int64)
    rl = hl + pl
    start = np.cumsum(rl) - rl
    out = np.zeros(int(rl.sum()), dtype=np.uint8)
    # header bytes
    rh = np.repeat(np.arange(len(e)), hl)
    k = np.arange(int(hl.sum())) - np.repeat(np.cumsum(hl) - hl, hl)
    out[start[rh] + k] = hdr[ho[rh] + k]
    # payload bytes, in place in the caller's arena
    rp = np.repeat(np.arange(len(e)), pl)
    j = np.arange(int(pl.sum())) - np.repeat(np.cumsum(pl) - pl, pl)
    out[start[rp] + hl[rp] + j] = hb.payload_arena[po[rp] + j]
    return out, start


def check(hb, oracle, hdr, iov, st, tot):
    o_wire, o_off, o_st, _ = oracle.encode_batch(hb)
    assert np.array_equal(st, o_st)
    ok = st == 0
    got, start = reassemble(hb, hdr, iov, st)
    assert got.tobytes() == bytes(o_wire)
    assert np.array_equal(iov["wire_off"][ok], o_off[:-1][ok])
    assert np.array_equal(start, o_off[:-1][ok].astype(np.int64))
    hl = iov["hdr_len"].astype(np.uint64)
    assert np.array_equal(iov["hdr_off"][ok], (np.cumsum(hl) - hl)[ok])
    assert int(tot[0]) == int(hl.sum()) and int(tot[1]) == len(o_wire)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1023, 1024, 1025, 4095, 4097, 16385, 70001])
def test_iov_workgroup_boundaries(codec, R, oracle, n):
    hb = S.mixed(n, seed=100 + n % 97, pmin=0, pmax=300, exotic=0.2)
    check(hb, oracle, *gpu_iov(R, codec, hb))


def test_iov_auth_unix_tiles(codec, R, oracle):
    # 32-word headers (the padded LDS staging) and odd payloads
    hb = S.call_unix16(5000, 1023)
    check(hb, oracle, *gpu_iov(R, codec, hb))


def test_iov_beyond_fused_blocks(codec, R, oracle):
    # 1075 iov_len workgroups > kFusedBlocks (1024): the scan-launch placement
    n = 1_100_000
    hb = S.mixed(n, seed=9, pmin=0, pmax=64, exotic=0.1)
    check(hb, oracle, *gpu_iov(R, codec, hb))


def _max_unix(name_len, ngids, rng):
    return {"kind": "unix", "stamp": int(rng.integers(0, 2**32)), "machine_name": rng.bytes(name_len).hex(),
            "uid": int(rng.integers(0, 2**32)), "gid": int(rng.integers(0, 2**32)),
            "gids": [int(x) for x in rng.integers(0, 2**32, ngids)]}


def test_iov_maximal_headers(codec, R, oracle):
    """Tiles of 460-byte headers (credential and verifier both AUTH_UNIX at
    the associated-data limit, flavor.rs:110): 29 KiB of headers per tile,
    past the LDS staging budget, so those records write their own words;
    interleaved with ordinary tiles staged in LDS."""
    rng = np.random.default_rng(5)
    msgs = []
    for i in range(64 * 12):
        big = (i // 64) % 2 == 0
        if big:
            c = [(124, 16), (188, 0)][int(rng.integers(0, 2))]
            v = [(124, 16), (188, 0)][int(rng.integers(0, 2))]
            cred, verf = _max_unix(*c, rng), _max_unix(*v, rng)
        else:
            cred, verf = {"kind": "none"}, {"kind": "none"}
        msgs.append({"xid": i, "type": "call", "program": 1, "program_version": 2, "procedure": 3,
                     "cred": cred, "verf": verf, "payload": rng.bytes(int(rng.integers(0, 40))).hex()})
    hb = L.build_batch(msgs)
    check(hb, oracle, *gpu_iov(R, codec, hb))


def test_iov_declared_extents(codec, R, oracle):
    """Declared AUTH_UNIX credentials whose blocks fail the deferred checks
    (tests/test_gpu_emit_paths.py::_adversarial): the vectored encode places
    records as onc_encode does (wire_off = the oracle's offsets for every
    record, a failing record's declared extent included; totals[1] = the
    packed total), the statuses are the oracle's, a record that fails without
    an extent has zero lengths, and every record with an extent — a failing
    declared one's placeholder header (ABI 7) included — gathers to the
    oracle's bytes: its header slice, then its payload slice."""
    from test_gpu_emit_paths import _adversarial
    hb = _adversarial(75, n=2500)
    o_wire, o_off, o_st, o_len = oracle.encode_batch(hb)
    assert ((o_st != 0) & (o_len != 0)).any()
    hdr, iov, st, tot = gpu_iov(R, codec, hb)
    assert np.array_equal(st, o_st)
    assert np.array_equal(iov["wire_off"], o_off[:-1])
    assert int(tot[1]) == int(o_off[-1])
    gone = o_len == 0
    assert (iov["hdr_len"][gone] == 0).all() and (iov["payload_len"][gone] == 0).all()
    w = np.frombuffer(o_wire, np.uint8)
    for i in np.nonzero(~gone)[0]:
        e = iov[i]
        a, hl, pl = int(o_off[i]), int(e["hdr_len"]), int(e["payload_len"])
        assert hl + pl == int(o_len[i])
        assert hdr[int(e["hdr_off"]):int(e["hdr_off"]) + hl].tobytes() == w[a:a + hl].tobytes()
        po = int(e["payload_off"])
        assert hb.payload_arena[po:po + pl].tobytes() == w[a + hl:a + hl + pl].tobytes()
