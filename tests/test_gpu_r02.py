"""GPU parity, round 2: the writer position, descriptor bounds, maximal
AUTH_UNIX headers, configs[4]'s per-GPU shard size, and the multi-rank path
running the HIP codec on every rank. Bit-exact against the CPU oracle."""
import os
import socket
import sys

import numpy as np
import pytest

import _onc_pkg  # the hyphenated package directory as onc_rpc_amd (also in spawned ranks)

_onc_pkg.load()
import onc_rpc_amd.layout as L  # noqa: E402
import onc_rpc_amd.synth as S  # noqa: E402

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODES = [L.DECODE_SLICE, L.DECODE_BYTES]


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


def _enc_at(R, codec, hb, shift, cap=None, fill=0xA5, tail=64):
    """Encode into out[shift:] of a buffer pre-filled with `fill`; returns
    (host buffer, rec_off, status)."""
    import torch
    db = R.DeviceBatch.from_host(hb)
    total = int(R.codec_lengths(codec, db).sum())
    cap = total if cap is None else cap
    buf = torch.full((shift + max(cap, total) + tail,), fill, dtype=torch.uint8, device="cuda")
    rec_off = torch.empty(hb.n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(max(hb.n, 1), dtype=torch.int32, device="cuda")
    codec.encode(db, buf[shift:], rec_off, st, out_cap=cap)
    codec.sync()
    return (buf.cpu().numpy(), rec_off.cpu().numpy().view(np.uint64), st.cpu().numpy()[:hb.n], total)


@pytest.mark.parametrize("gen", ["call_none", "mixed"])
def test_encode_at_any_writer_position(codec, R, oracle, gen):
    """serialise_into writes at the writer's current position
    (rpc_message.rs:136; buffer reuse README.md:11): the batch lands at any
    byte address, bit-exact, and no byte before it or past its end (or past
    out_cap) is touched."""
    hb = S.call_none(3000, 256) if gen == "call_none" else S.mixed(2500, seed=12, pmin=0, pmax=700, exotic=0.1)
    o_wire, o_off, o_st, _ = oracle.encode_batch(hb)
    total = len(o_wire)
    for shift in (0, 1, 2, 3, 4, 5, 7, 8, 12, 13, 15, 16, 17, 4093):
        buf, off, st, t = _enc_at(R, codec, hb, shift)
        assert t == total
        assert np.array_equal(st, o_st) and np.array_equal(off, o_off), shift
        assert (buf[:shift] == 0xA5).all(), f"shift {shift}: bytes before the writer position written"
        assert buf[shift:shift + total].tobytes() == o_wire, f"shift {shift}"
        assert (buf[shift + total:] == 0xA5).all(), f"shift {shift}: bytes past the batch written"
    # capacity-limited at an odd position: WRITE_ZERO parity, nothing past out_cap
    for shift, cap in ((3, total // 2 + 5), (9, 37), (14, total - 1)):
        buf, off, st, _ = _enc_at(R, codec, hb, shift, cap=cap)
        w2, off2, st2, _ = oracle.encode_batch(hb, out_cap=cap)
        assert np.array_equal(st, st2) and np.array_equal(off, off2)
        assert (buf[:shift] == 0xA5).all()
        assert buf[shift:shift + len(w2)].tobytes() == w2
        assert (buf[shift + cap:] == 0xA5).all()


def test_descriptor_bounds(codec, R, oracle):
    """A descriptor referencing outside the arenas' declared sizes (onc_batch
    unix_count / auth_len / payload_len) is ONC_ENC_BAD_DESCRIPTOR and
    occupies 0 bytes; everything else is bit-exact vs the oracle, whose
    batch has those records replaced by an unrepresentable descriptor (the
    same status). The out-of-range references still point inside the
    physical tensors, so a missed check could not fault."""
    import torch
    hb = S.mixed(1200, seed=33, pmin=0, pmax=300, exotic=0.3)
    m = hb.msgs.copy()
    unix = hb.unix
    n_unix = len(unix)
    auth_len = len(hb.auth_arena)
    pay_len = len(hb.payload_arena)
    rng = np.random.default_rng(4)
    bad = np.zeros(hb.n, bool)
    is_call = m["msg_type"] == L.MSG_CALL
    has_pay = (is_call | ((m["reply_stat"] == L.REPLY_ACCEPTED) & (m["stat"] == 0))) & (m["payload_len"] > 0)
    # payload past the declared arena end
    idx = rng.choice(np.nonzero(has_pay)[0], 40, replace=False)
    m["payload_off"][idx] = np.uint64(pay_len) - m["payload_len"][idx].astype(np.uint64) + np.uint64(1)
    bad[idx] = True
    # AUTH_UNIX credential index past the table
    cu = np.nonzero(is_call & ((m["cred_kind_len"] >> 24) == L.KIND_UNIX) & ~bad)[0]
    idx = rng.choice(cu, 30, replace=False)
    m["cred_ref"][idx] = np.uint64(n_unix)
    # (undeclared: index n_unix is the private row below, whose name lies
    # outside the arena — a declared credential keeps its extent then)
    m["cred_kind_len"][idx] = int(L.pack_kind_len(L.KIND_UNIX, 0))
    bad[idx] = True
    # opaque auth body past the arena
    op = np.nonzero(is_call & ((m["verf_kind_len"] >> 24) != L.KIND_UNIX) & ((m["verf_kind_len"] & 0xFFFFFF) > 0)
                    & ~bad)[0]
    idx = op[:20]
    m["verf_ref"][idx] = np.uint64(auth_len)
    bad[idx] = True
    # machine name past the arena (a private unix row)
    unix2 = np.concatenate([unix, unix[:1]])
    unix2["name_len"][-1] = 5
    unix2["name_off"][-1] = auth_len - 2
    cu = np.nonzero(is_call & ((m["cred_kind_len"] >> 24) == L.KIND_UNIX) & ~bad)[0][:10]
    m["cred_ref"][cu] = len(unix2) - 1
    # (undeclared: a declared credential's name is checked by the emit and the
    # record keeps its extent — test_gpu_emit_paths.py::test_declared_name_outside_arena)
    m["cred_kind_len"][cu] = int(L.pack_kind_len(L.KIND_UNIX, 0))
    bad[cu] = True
    # device batch: physical tensors padded well past the declared sizes
    pad = 4096
    dev = "cuda"
    db = R.DeviceBatch(hb.n, R.to_device(m, dev),
                       R.to_device(np.concatenate([unix2, np.zeros(4, L.UNIX_DTYPE)]), dev),
                       R.to_device(np.concatenate([hb.auth_arena, np.zeros(pad, np.uint8)]), dev),
                       R.to_device(np.concatenate([hb.payload_arena, np.zeros(pad, np.uint8)]), dev),
                       unix_count=len(unix2), auth_len=auth_len, payload_len=pay_len)
    lens = R.codec_lengths(codec, db)
    total = int(lens.sum())
    out = torch.zeros(total + 16, dtype=torch.uint8, device=dev)
    rec_off = torch.empty(hb.n + 1, dtype=torch.int64, device=dev)
    st = torch.empty(hb.n, dtype=torch.int32, device=dev)
    codec.encode(db, out, rec_off, st)
    codec.sync()
    g_st = st.cpu().numpy()
    ref = m.copy()
    ref["msg_type"][bad] = 7
    o_wire, o_off, o_st, _ = oracle.encode_batch(L.HostBatch(ref, unix2, hb.auth_arena, hb.payload_arena))
    assert (o_st[bad] == 104).all()
    assert np.array_equal(g_st, o_st), np.nonzero(g_st != o_st)[0][:10]
    assert np.array_equal(rec_off.cpu().numpy().view(np.uint64), o_off)
    assert out[:total].cpu().numpy().tobytes() == o_wire


def _max_unix(name_len, ngids, seed):
    rng = np.random.default_rng(seed)
    return {"kind": "unix", "stamp": int(rng.integers(0, 2**32)), "machine_name": rng.bytes(name_len).hex(),
            "uid": int(rng.integers(0, 2**32)), "gid": int(rng.integers(0, 2**32)),
            "gids": [int(x) for x in rng.integers(0, 2**32, ngids)]}


@pytest.mark.parametrize("shift", [0, 3])
def test_maximal_auth_unix_spans(codec, R, oracle, shift):
    """Calls whose credential AND verifier are both AUTH_UNIX at the
    associated-data limit (124-byte name + 16 gids, 188-byte name + 0 gids:
    54-word auths, 460-byte headers — flavor.rs:110, unix_params.rs:234-245),
    with odd and small payloads, so enc_emit's byte path cuts every tile into
    several LDS spans of maximal records. Encode bit-exact (also at an odd
    writer position); decode parity in both modes (these encode but do not
    decode: the wire body is 208 > 200 bytes for 124 + 16, flavor.rs:83)."""
    msgs = []
    rng = np.random.default_rng(77)
    for i in range(700):
        shapes = [(124, 16), (188, 0)]
        c = shapes[int(rng.integers(0, 2))]
        v = shapes[int(rng.integers(0, 2))]
        plen = int(rng.choice([0, 1, 3, 5, 15, 17, 31, 33, 255, 1021]))
        msgs.append({"xid": i, "type": "call", "program": 1, "program_version": 2, "procedure": 3,
                     "cred": _max_unix(*c, seed=2 * i), "verf": _max_unix(*v, seed=2 * i + 1),
                     "payload": rng.bytes(plen).hex()})
    hb = L.build_batch(msgs)
    o_wire, o_off, o_st, _ = oracle.encode_batch(hb)
    assert (o_st == 0).all()
    hw = np.diff(o_off.astype(np.int64)) - hb.msgs["payload_len"].astype(np.int64)
    assert hw.max() == 460
    buf, off, st, total = _enc_at(R, codec, hb, shift)
    assert np.array_equal(st, o_st) and np.array_equal(off, o_off)
    assert buf[shift:shift + total].tobytes() == o_wire
    w = np.frombuffer(o_wire + b"\0" * 16, np.uint8).copy()
    for mode in MODES:
        g = R.decode_host_wire(codec, w, o_off, mode)
        o = oracle.decode_batch(w, o_off, mode)
        assert np.array_equal(g[2], o[2]) and np.array_equal(g[3], o[3]) and np.array_equal(g[4], o[4])
        assert np.array_equal(g[0].view(np.uint8), o[0].view(np.uint8))


def test_configs4_shard_8m(codec, R, oracle):
    """configs[4]'s per-GPU shard at 8 GPUs: records [56M, 64M) of the 64M
    batch (8M x 300 B, generated on the device like bench.py's c4 leg),
    encode -> decode in both modes with size-independent checks (all OK,
    offsets = 300 i, xids = record index, payload bytes = the arena), the
    whole buffer re-encoded from the decoded descriptors (parse -> serialise
    identity), and a 20k-record window bit-exact vs the oracle."""
    import torch
    lo, hi = 56_000_000, 64_000_000
    n = hi - lo
    db, _ = S.call_none_device(lo, hi, 256, seed=4)
    out = torch.empty(n * 300 + 16, dtype=torch.uint8, device="cuda")
    rec_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    codec.reserve(n)
    codec.encode(db, out, rec_off, st)
    codec.sync()
    assert int((st != 0).sum()) == 0
    assert torch.equal(rec_off, torch.arange(n + 1, device="cuda", dtype=torch.int64) * 300)
    assert torch.equal(out[: n * 300].view(n, 300)[:, 44:].reshape(-1), db.payload_arena[: n * 256])
    want_xid = torch.arange(lo, hi, device="cuda", dtype=torch.int64).to(torch.int32)
    bufs = R.DecodeBuffers(n)
    for mode in MODES:
        codec.decode(out, rec_off, n, mode, bufs.msgs, bufs.unix, bufs.status, bufs.aux0, bufs.aux1)
        codec.sync()
        assert int((bufs.status != 0).sum()) == 0, mode
        xid = bufs.msgs.view(-1, 64)[:, 0:4].contiguous().view(torch.int32).view(-1)
        assert torch.equal(xid, want_xid), mode
    again = R.DeviceBatch(n, bufs.msgs, bufs.unix, out, out)
    out2 = torch.empty_like(out)
    codec.encode(again, out2, rec_off, st)
    codec.sync()
    assert int((st != 0).sum()) == 0
    assert torch.equal(out2[: n * 300], out[: n * 300])
    del out2, again, bufs
    w0, w1 = 4_000_000, 4_020_000
    sub = S.host_window(db, w0, w1)
    o_wire = oracle.encode_batch(sub)[0]
    assert out[w0 * 300:w1 * 300].cpu().numpy().tobytes() == o_wire
    torch.cuda.empty_cache()


# ---------------------------------------------------------------------------
# multi-rank: every rank runs the HIP codec on its shard (both on cuda:0,
# gloo for the one control-plane all_gather of byte totals)
# ---------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_worker(rank, world, port, n, outdir):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import _onc_pkg
    _onc_pkg.load()
    import onc_rpc_amd.runtime as R
    import onc_rpc_amd.shard as SH
    import onc_rpc_amd.synth as S

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    codec = R.Codec(0)
    hb = S.mixed(n, seed=21, pmin=0, pmax=300, exotic=0.2)
    lo, hi = SH.shard_bounds(n, world, rank)
    wire, off, st, _ = R.encode_host_batch(codec, SH.shard_batch(hb, lo, hi))
    bases, grand = SH.exclusive_bases(SH.allgather_totals(len(wire)))
    base = int(bases[rank])
    w = np.frombuffer(wire + b"\0" * 16, np.uint8).copy()
    res = {"wire": np.frombuffer(wire, np.uint8), "off": off + np.uint64(base), "st": st,
           "grand": np.array([grand], np.uint64)}
    for mode in (0, 1):
        msgs, unix, dst, a0, a1 = R.decode_host_wire(codec, w, off, mode)
        gm, gu = SH.rebase_decoded(msgs, unix, lo, base)
        res.update({f"msgs{mode}": gm.view(np.uint8), f"unix{mode}": gu.view(np.uint8), f"dst{mode}": dst,
                    f"a0{mode}": a0, f"a1{mode}": a1})
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **res)
    codec.close()
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_hip_codec_concatenate(codec, R, oracle, tmp_path):
    """World size 2, both ranks on cuda:0 running the HIP encode + decode on
    their contiguous shard; the concatenated shard wires, rebased offsets and
    rebased decoded descriptors equal the single-process GPU result and the
    oracle, in both decode modes (records are independent,
    rpc_message.rs:235-271 / :136-164)."""
    import torch.multiprocessing as mp
    n, world = 3001, 2
    mp.start_processes(_rank_worker, args=(world, _free_port(), n, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    parts = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    hb = S.mixed(n, seed=21, pmin=0, pmax=300, exotic=0.2)
    g_wire, g_off, g_st, _ = R.encode_host_batch(codec, hb)
    o_wire, o_off, o_st, _ = oracle.encode_batch(hb)
    assert g_wire == o_wire
    cat = b"".join(p["wire"].tobytes() for p in parts)
    assert cat == g_wire
    assert int(parts[0]["grand"][0]) == len(g_wire) == int(parts[1]["grand"][0])
    got_off = np.concatenate([p["off"][:-1] for p in parts] + [parts[-1]["off"][-1:]])
    assert np.array_equal(got_off, g_off) and np.array_equal(got_off, o_off)
    assert np.array_equal(np.concatenate([p["st"] for p in parts]), o_st)
    w = np.frombuffer(g_wire + b"\0" * 16, np.uint8).copy()
    for mode in MODES:
        gm, gu, gs, ga0, ga1 = R.decode_host_wire(codec, w, g_off, mode)
        om, ou, os_, _, _ = oracle.decode_batch(w, g_off, mode)
        dst = np.concatenate([p[f"dst{mode}"] for p in parts])
        assert np.array_equal(dst, gs) and np.array_equal(dst, os_)
        cm = np.concatenate([p[f"msgs{mode}"] for p in parts]).view(L.MSG_DTYPE)
        cu = np.concatenate([p[f"unix{mode}"] for p in parts]).view(L.UNIX_DTYPE)
        # AUTH_UNIX slots are packed per 64-record group of each decode call,
        # so the shards' refs differ from the whole batch's: compare resolved
        assert np.array_equal(gm.view(np.uint8), om.view(np.uint8))
        cm_r, cp = L.resolve_unix(cm, cu, dst)
        gm_r, gp = L.resolve_unix(gm, gu, gs)
        om_r, op = L.resolve_unix(om, ou, os_)
        assert np.array_equal(cm_r.view(np.uint8), gm_r.view(np.uint8))
        assert np.array_equal(cm_r.view(np.uint8), om_r.view(np.uint8))
        assert np.array_equal(cp, gp) and np.array_equal(cp, op)


@pytest.mark.parametrize("force", [False, True])
def test_scan_lengths_sizes_and_alignment(R, force):
    """onc_scan_lengths: the two-launch path (lenblk -> lenoff, up to 8M
    records) and the three-launch path (ONC_OPT_FORCE_SCAN, or beyond 8M)
    at block boundaries, with misaligned length / offset pointers (slices):
    rec_off = base + exclusive prefix sum, rec_off[n] = base + total."""
    import torch
    c = R.Codec(0, force_scan=force)
    rng = np.random.default_rng(11)
    sizes = [1, 15, 16, 17, 4095, 4096, 4097, 8191, 65536 + 3, 2048 * 4096, 2048 * 4096 + 1]
    for n in sizes:
        lens = rng.integers(0, 1 << 31, n, dtype=np.uint64).astype(np.uint32) if n < 100 else \
            rng.integers(0, 5000, n).astype(np.uint32)
        for lshift, oshift in ((0, 0), (1, 1), (3, 2)):
            if n > 100000 and (lshift, oshift) != (0, 0):
                continue
            d = torch.zeros(n + lshift, dtype=torch.int32, device="cuda")
            d[lshift:] = torch.from_numpy(lens.view(np.int32).copy()).cuda()
            off = torch.zeros(n + 1 + oshift, dtype=torch.int64, device="cuda")
            c.scan_lengths(d[lshift:], n, 987654321, off[oshift:])
            c.sync()
            want = np.concatenate([[0], np.cumsum(lens.astype(np.uint64))]) + np.uint64(987654321)
            got = off[oshift:].cpu().numpy().view(np.uint64)
            assert np.array_equal(got, want), (n, lshift, oshift, np.nonzero(got != want)[0][:5])
    c.close()


def test_encode_plan_emit(codec, R, oracle):
    """onc_encode in two phases (onc_encode_plan = enc_len, onc_encode_emit =
    enc_emit): the same bytes, offsets and statuses as onc_encode and the
    oracle, at any writer position, the plan reusable for several emits;
    an emit of a batch that is not the handle's last plan is refused."""
    import torch
    hb = S.mixed(1500, seed=19, pmin=0, pmax=500, exotic=0.2)
    o_wire, o_off, o_st, o_len = oracle.encode_batch(hb)
    db = R.DeviceBatch.from_host(hb)
    total = len(o_wire)
    st = torch.empty(hb.n, dtype=torch.int32, device="cuda")
    rl = torch.empty(hb.n, dtype=torch.int32, device="cuda")
    codec.encode_plan(db, st, rl)
    codec.sync()
    assert np.array_equal(rl.cpu().numpy().view(np.uint32), o_len)
    for shift in (0, 5):
        buf = torch.full((total + shift + 32,), 0x5A, dtype=torch.uint8, device="cuda")
        off = torch.empty(hb.n + 1, dtype=torch.int64, device="cuda")
        codec.encode_emit(db, buf[shift:], off, st, out_cap=total)
        codec.sync()
        b = buf.cpu().numpy()
        assert b[shift:shift + total].tobytes() == o_wire and (b[:shift] == 0x5A).all()
        assert np.array_equal(off.cpu().numpy().view(np.uint64), o_off)
        assert np.array_equal(st.cpu().numpy(), o_st)
    other = R.DeviceBatch.from_host(S.call_none(10, 16))
    with pytest.raises(R.CodecError):
        codec.encode_emit(other, buf, off, st)


def test_kernel_timing(R, oracle):
    """onc_codec_enable_timing / onc_codec_kernel_stats (the bench's
    measurement path: timed launches go through hipExtLaunchKernelGGL with
    start/stop events): every launch of a timed kernel is counted with a
    positive duration, a mask times only its kernels, stats reset, and the
    outputs are the same as untimed and bit-exact."""
    hb = S.mixed(6000, seed=21, pmin=0, pmax=600, exotic=0.1)
    o_wire, o_off, o_st, _ = oracle.encode_batch(hb)
    c = R.Codec(0)
    try:
        plain = R.encode_host_batch(c, hb)
        dec_plain = R.decode_host_wire(c, np.frombuffer(plain[0] + b"\0" * 16, np.uint8), plain[1], L.DECODE_SLICE)
        c.enable_timing(True)
        timed = R.encode_host_batch(c, hb)
        dec_timed = R.decode_host_wire(c, np.frombuffer(timed[0] + b"\0" * 16, np.uint8), timed[1], L.DECODE_SLICE)
        st = c.kernel_stats()
        # encode_host_batch: lengths pass (enc_len) + encode (enc_len, enc_emit)
        assert st["enc_len_kernel"][1] == 2 and st["enc_len_kernel"][0] > 0, st
        assert st["enc_emit_kernel"][1] == 1 and st["enc_emit_kernel"][0] > 0, st
        assert st["decode_kernel"][1] == 1 and st["decode_kernel"][0] > 0, st
        assert timed[0] == plain[0] == o_wire
        assert np.array_equal(timed[1], o_off) and np.array_equal(timed[2], o_st)
        for x, y in zip(dec_timed, dec_plain):
            assert np.array_equal(x, y)
        c.reset_stats()
        c.enable_timing(True, kernels=[R.K_ENC_EMIT])
        R.encode_host_batch(c, hb)
        R.decode_host_wire(c, np.frombuffer(plain[0] + b"\0" * 16, np.uint8), plain[1], L.DECODE_SLICE)
        st = c.kernel_stats()
        assert st["enc_emit_kernel"][1] == 1
        assert all(v[1] == 0 for k, v in st.items() if k != "enc_emit_kernel"), st
        c.enable_timing(False)
        c.reset_stats()
        R.encode_host_batch(c, hb)
        assert all(v[1] == 0 for v in c.kernel_stats().values())
    finally:
        c.close()
