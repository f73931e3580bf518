"""Both enc_emit kernels, forced (onc_codec_options.variant 0x200: the wave-specialised
producer/consumer kernel; 0x400: the wave-per-tile kernel), bit-exact against
the CPU oracle (RpcMessage::serialise_into, rpc_message.rs:136-164) on the
batch shapes that stress placement and staging: many tiles per persistent
workgroup, multi-span tiles of maximal AUTH_UNIX headers on the byte path,
odd writer positions, capacity limits and invalid records. The codec picks
one of the two per batch (codec.hip enc_args); these tests pin both."""
import numpy as np
import pytest

import _onc_pkg  # noqa: F401  (the hyphenated package directory as onc_rpc_amd)

_onc_pkg.load()
import onc_rpc_amd.layout as L  # noqa: E402
import onc_rpc_amd.synth as S  # noqa: E402

pytestmark = pytest.mark.gpu

# ws: the wave-specialised kernel, which runs header-heavy batches as
# wave-per-tile workers (encode.hip ws_header_heavy); ws_pipeline: the same
# kernel with that fallback off (0x10000), its producer/consumer pipeline
# on every shape; tile: the wave-per-tile kernel
PATHS = {"ws": 0x200, "ws_pipeline": 0x10200, "tile": 0x400}


@pytest.fixture(scope="module")
def R():
    import onc_rpc_amd.runtime as R
    return R


@pytest.fixture(scope="module", params=sorted(PATHS))
def codec(request, R):
    import os
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    c = R.Codec(0, variant=PATHS[request.param])
    yield c
    c.close()


def _enc(R, codec, hb, shift=0, cap=None, fill=0x5A):
    import torch
    db = R.DeviceBatch.from_host(hb)
    total = int(R.codec_lengths(codec, db).sum())
    cap = total if cap is None else cap
    buf = torch.full((shift + max(cap, total) + 64,), fill, dtype=torch.uint8, device="cuda")
    rec_off = torch.empty(hb.n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(max(hb.n, 1), dtype=torch.int32, device="cuda")
    codec.encode(db, buf[shift:], rec_off, st, out_cap=cap)
    codec.sync()
    return buf.cpu().numpy(), rec_off.cpu().numpy().view(np.uint64), st.cpu().numpy()[:hb.n], total


def _check(R, codec, oracle, hb, shift=0, cap=None):
    o_wire, o_off, o_st, _ = oracle.encode_batch(hb, out_cap=cap) if cap is not None else oracle.encode_batch(hb)
    buf, off, st, total = _enc(R, codec, hb, shift, cap)
    assert np.array_equal(st, o_st)
    assert np.array_equal(off, o_off)
    assert buf[shift:shift + len(o_wire)].tobytes() == o_wire
    assert (buf[:shift] == 0x5A).all()
    end = shift + (total if cap is None else cap)
    assert (buf[end:] == 0x5A).all()


@pytest.mark.parametrize("shift", [0, 5])
def test_call_none_many_tiles(codec, R, oracle, shift):
    """configs[1]-shaped records, 200k of them: 3125 tiles, three per
    persistent workgroup of the wave-specialised kernel."""
    _check(R, codec, oracle, S.call_none(200_000, 256, seed=31), shift)


@pytest.mark.parametrize("gen", ["mixed", "random", "unix16", "odd", "big", "big_odd"])
def test_shapes(codec, R, oracle, gen):
    if gen == "mixed":
        hb = S.mixed(40_000, seed=32, pmin=0, pmax=900, exotic=0.1)
    elif gen == "random":
        hb = L.build_batch(S.random_messages(20_000, seed=33, max_payload=700))
    elif gen == "unix16":
        hb = S.call_unix16(30_000, 64, seed=34)
    elif gen == "odd":
        hb = S.call_none(50_000, 257, seed=35)       # odd payloads: the byte path in every tile
    elif gen == "big":
        hb = S.call_unix16(20_000, 1024, seed=39)    # >= 512 B mean payload: 1 KiB consumer steps
    else:
        hb = S.call_none(20_000, 1023, seed=40)
    _check(R, codec, oracle, hb)
    _check(R, codec, oracle, hb, shift=11)


def test_capacity_and_invalid(codec, R, oracle):
    """out_cap inside the batch (WRITE_ZERO parity, nothing past the cap)
    and records that fail validation mid-tile (zero-length spans)."""
    hb = S.mixed(30_000, seed=36, pmin=0, pmax=600, exotic=0.2)
    total = len(oracle.encode_batch(hb)[0])
    for cap in (total // 3 + 7, 1000, total - 1):
        _check(R, codec, oracle, hb, shift=3, cap=cap)
    # every 7th credential an AUTH_SHORT body of 300 bytes (> 200, flavor.rs:110),
    # every 11th a verifier of 201 bytes; bodies inside the auth arena
    rng = np.random.default_rng(37)
    msgs = []
    for i in range(20_000):
        cl = 300 if i % 7 == 0 else 0
        vl = 201 if i % 11 == 0 else 8
        msgs.append({"xid": i, "type": "call", "program": 100003, "program_version": 4, "procedure": 1,
                     "cred": {"kind": "short" if cl else "none", "data": rng.bytes(cl).hex() if cl else None},
                     "verf": {"kind": "short", "data": rng.bytes(vl).hex()},
                     "payload": rng.bytes(int(rng.integers(0, 400))).hex()})
    bad = L.build_batch(msgs)
    o_st = oracle.encode_batch(bad)[2]
    assert (o_st[::7] != 0).all() and (o_st[1::7][(np.arange(1, 20_000, 7) % 11) != 0] == 0).all()
    _check(R, codec, oracle, bad)


@pytest.mark.parametrize("shift", [0, 4, 7, 12])
def test_two_span_edges(codec, R, oracle, shift):
    """configs[0]-shaped records (benches/bench.rs:86-101 + 64 B payload):
    every 64-record tile streams as two spans on the word path, whose
    partial edge chunks are loaded before the stream's first steps
    (encode.hip EdgeChunks) — at writer positions that put the span edges
    at every dword offset inside a chunk, and with the capacity ending
    inside a tile's second span and inside a chunk."""
    hb = S.cpu_roundtrip(20_000, seed=41)
    _check(R, codec, oracle, hb, shift=shift)
    total = len(oracle.encode_batch(hb)[0])
    # record 64 * 157 + 50 lies in tile 157's second span; cut 3 bytes into its payload
    rec = 64 * 157 + 50
    cap = int(oracle.encode_batch(hb)[1][rec]) + 128 + 3
    assert cap < total
    _check(R, codec, oracle, hb, shift=shift, cap=cap)


def test_maximal_auth_unix(codec, R, oracle):
    """Credential and verifier both AUTH_UNIX at the 200-byte limit (460-byte
    headers) with odd payloads: several spans per tile on the byte path."""
    rng = np.random.default_rng(38)
    msgs = []
    for i in range(3000):
        def unix(name_len, ngids):
            return {"kind": "unix", "stamp": int(rng.integers(0, 2**32)), "machine_name": rng.bytes(name_len).hex(),
                    "uid": 1, "gid": 2, "gids": [int(x) for x in rng.integers(0, 2**32, ngids)]}
        shapes = [(124, 16), (188, 0)]
        c = shapes[int(rng.integers(0, 2))]
        v = shapes[int(rng.integers(0, 2))]
        plen = int(rng.choice([0, 1, 3, 15, 17, 255, 1021]))
        msgs.append({"xid": i, "type": "call", "program": 1, "program_version": 2, "procedure": 3,
                     "cred": unix(*c), "verf": unix(*v), "payload": rng.bytes(plen).hex()})
    hb = L.build_batch(msgs)
    _check(R, codec, oracle, hb)
    _check(R, codec, oracle, hb, shift=13)
