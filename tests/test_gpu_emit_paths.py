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
# on every shape; tile: the wave-per-tile kernel; tile_replan: the same
# re-planning each record instead of reading the plan's lengths (0x20000)
PATHS = {"ws": 0x200, "ws_pipeline": 0x10200, "tile": 0x400, "tile_replan": 0x20400}


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


@pytest.mark.parametrize("ntiles,last", [(1025, 5), (1024 + 300, 64), (1024 + 511, 33), (1024 + 600, 64),
                                         (2048 + 3, 1)])
def test_last_round_split(codec, R, oracle, ntiles, last):
    """Tile counts around multiples of the wave-specialised kernel's 1024
    persistent workgroups (a last round of 1, 300, 511 and 600 tiles, and
    of 3 after two full rounds), a last tile of 5 records and one of a
    single record: configs[1]-shaped records at writer positions 0 and 7
    (the word and the byte path), a mixed batch with invalid records, and a
    capacity ending inside the last round. (Round 4 measured cutting the
    last round's tiles into parts, one per workgroup, and did not keep it:
    the shapes stay as its tests.)"""
    n = 64 * (ntiles - 1) + last
    hb = S.call_none(n, 256, seed=ntiles)
    _check(R, codec, oracle, hb)
    _check(R, codec, oracle, hb, shift=7)
    mx = S.mixed(n, seed=ntiles + 1, pmin=100, pmax=700, exotic=0.1)
    _check(R, codec, oracle, mx, shift=3)
    o_off = oracle.encode_batch(mx)[1]
    cap = int(o_off[64 * (ntiles - 2) + 20]) + 5
    _check(R, codec, oracle, mx, shift=3, cap=cap)


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


# ---------------------------------------------------------------------------
# Declared AUTH_UNIX lengths (ABI 6, include/onc_rpc.h onc_auth): the length
# pass plans a declared auth from the descriptor alone and the emit runs the
# parameter-block checks it deferred.
# ---------------------------------------------------------------------------
def _enc_oracle_sized(R, codec, hb, oracle, shift=0, cap=None, fill=0x5A):
    import torch
    o_wire, o_off, o_st, o_len = oracle.encode_batch(hb) if cap is None else oracle.encode_batch(hb, out_cap=cap)
    total = int(o_off[hb.n])
    cap = total if cap is None else cap
    db = R.DeviceBatch.from_host(hb)
    buf = torch.full((shift + max(cap, total) + 64,), fill, dtype=torch.uint8, device="cuda")
    rec_off = torch.empty(hb.n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(max(hb.n, 1), dtype=torch.int32, device="cuda")
    rl = torch.empty(max(hb.n, 1), dtype=torch.int32, device="cuda")
    codec.encode(db, buf[shift:], rec_off, st, rl, out_cap=cap)
    codec.sync()
    b = buf.cpu().numpy()
    assert np.array_equal(st.cpu().numpy()[:hb.n], o_st), \
        f"status {np.nonzero(st.cpu().numpy()[:hb.n] != o_st)[0][:8]}"
    assert np.array_equal(rec_off.cpu().numpy().view(np.uint64), o_off)
    assert np.array_equal(rl.cpu().numpy().view(np.uint32)[:hb.n], o_len)
    assert b[shift:shift + len(o_wire)].tobytes() == o_wire
    assert (b[:shift] == fill).all() and (b[shift + cap:] == fill).all()
    return o_st, o_len


def _adversarial(seed, n=3000):
    """random_messages with declared lengths, then a quarter of the AUTH_UNIX
    auths (credentials and verifiers, Calls and accepted replies) broken:
    declared != serialised (+4 / -4), a 300-byte machine name or 17 gids in
    the block (panics) under a plausible declared length, an implausible
    declared length (3, 18, 400: planned in full), or a block failure next to
    a failing descriptor-only check (a 201-byte opaque verifier: the full
    plan's reference-order status)."""
    rng = np.random.default_rng(seed)
    hb = L.build_batch(S.random_messages(n, seed=seed, max_payload=300))
    m, u = hb.msgs, hb.unix
    for f in ("cred", "verf"):
        isu = ((m[f + "_kind_len"] >> 24) == L.KIND_UNIX) & (m[f + "_kind_len"] & 0xFFFFFF != 0)
        for i in np.nonzero(isu)[0]:
            c = int(rng.integers(0, 8))
            ref = int(m[f + "_ref"][i])
            ln = int(m[f + "_kind_len"][i] & 0xFFFFFF)
            if c == 0:
                m[f + "_kind_len"][i] = int(L.pack_kind_len(L.KIND_UNIX, ln + 4))
            elif c == 1 and ln >= 24:
                m[f + "_kind_len"][i] = int(L.pack_kind_len(L.KIND_UNIX, ln - 4))
            elif c == 2:
                u["name_len"][ref] = 300
            elif c == 3:
                u["ngids"][ref] = 17
            elif c == 4:
                m[f + "_kind_len"][i] = int(L.pack_kind_len(L.KIND_UNIX, int(rng.choice([3, 18, 400]))))
            elif c == 5 and m["msg_type"][i] == L.MSG_CALL and f == "cred":
                u["ngids"][ref] = 17
                m["verf_kind_len"][i] = int(L.pack_kind_len(L.KIND_SHORT, 201))
                m["verf_ref"][i] = 0
    return hb


@pytest.mark.parametrize("seed", [71, 72])
def test_declared_lengths_broken_blocks(codec, R, oracle, seed):
    """Records whose only failure is a deferred block check keep the extent
    their descriptor declares (a placeholder header: the record mark of the
    extent, then zeros — ABI 7; payload in place) with the
    check's status; the others get the full plan's reference-order status
    and no bytes — the oracle's restatement of the rule, bit-exact, at two
    writer positions and with a capacity inside the batch. onc_encode_lengths
    checks every block up front and reports the same extents (what a caller
    sizes its send buffer with)."""
    import torch
    hb = _adversarial(seed)
    o_st, o_len = _enc_oracle_sized(R, codec, hb, oracle)
    assert (o_st != 0).sum() > 200 and ((o_st != 0) & (o_len != 0)).sum() > 100   # both kinds of failure
    _enc_oracle_sized(R, codec, hb, oracle, shift=7)
    total = int(o_len.astype(np.int64).sum())
    _enc_oracle_sized(R, codec, hb, oracle, shift=3, cap=total // 2 + 5)
    db = R.DeviceBatch.from_host(hb)
    rl = torch.empty(hb.n, dtype=torch.int32, device="cuda")
    st = torch.empty(hb.n, dtype=torch.int32, device="cuda")
    codec.encode_lengths(db, rl, st)
    codec.sync()
    assert np.array_equal(st.cpu().numpy(), o_st)
    assert np.array_equal(rl.cpu().numpy().view(np.uint32), o_len)


def test_declared_equals_undeclared(codec, R, oracle):
    """The same messages with every AUTH_UNIX length declared and with none:
    identical wire, offsets and statuses (and the oracle's)."""
    msgs = S.random_messages(4000, seed=73, max_payload=500)
    a = _enc_oracle_sized(R, codec, L.build_batch(msgs, declare=True), oracle, shift=1)
    b = _enc_oracle_sized(R, codec, L.build_batch(msgs, declare=False), oracle, shift=1)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    ow_a = oracle.encode_batch(L.build_batch(msgs, declare=True))[0]
    ow_b = oracle.encode_batch(L.build_batch(msgs, declare=False))[0]
    assert ow_a == ow_b


def test_declared_name_outside_arena(codec, R, oracle):
    """A declared credential whose machine name lies outside the auth arena
    (the GPU's bounds check, which the oracle does not model): BAD_DESCRIPTOR
    with the declared extent — the same bytes and offsets as the oracle's for
    the same record failing another deferred check (17 gids)."""
    hb = S.call_unix16(2000, 40, seed=74)
    hb.unix["name_len"][100:110] = 8        # declared lengths follow the names
    hb.msgs["cred_kind_len"][100:110] = int(L.pack_kind_len(L.KIND_UNIX, L.unix_body_len(8, 16)))
    hb.auth_arena = np.zeros(64, np.uint8)
    hb.unix["name_off"][100:110] = 16
    ref = L.HostBatch(hb.msgs.copy(), hb.unix.copy(), hb.auth_arena, hb.payload_arena)
    ref.unix["ngids"][[103, 107]] = 17
    hb.unix["name_off"][[103, 107]] = 1 << 40
    import torch
    o_wire, o_off, o_st, o_len = oracle.encode_batch(ref)
    db = R.DeviceBatch.from_host(hb)
    total = int(o_off[hb.n])
    buf = torch.zeros(total + 64, dtype=torch.uint8, device="cuda")
    off = torch.empty(hb.n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(hb.n, dtype=torch.int32, device="cuda")
    codec.encode(db, buf, off, st, out_cap=total)
    codec.sync()
    g_st = st.cpu().numpy()
    want = o_st.copy()
    want[[103, 107]] = 104                  # ONC_ENC_BAD_DESCRIPTOR
    assert np.array_equal(g_st, want)
    assert np.array_equal(off.cpu().numpy().view(np.uint64), o_off)
    assert buf.cpu().numpy()[:total].tobytes() == o_wire
