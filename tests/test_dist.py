"""Multi-rank sharding of the batch with world_size 2 over
gloo on the CPU.

Each rank takes its contiguous record range, encodes and decodes it alone
(the oracle stands in for the per-GPU codec here: these tests cover the
partitioning, the one control-plane all_gather of byte totals and the
rebasing — the kernels themselves are covered by the -m gpu tests), and the
concatenation in rank order must equal the single-process result bit for
bit. No data-path collective is used: only the byte totals cross ranks.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, mode, outdir):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist

    import _onc_pkg
    _onc_pkg.load()
    import oracle_ffi
    import onc_rpc_amd.shard as SH
    import onc_rpc_amd.synth as S

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    hb = S.mixed(n, seed=21, pmin=0, pmax=300, exotic=0.2)
    lo, hi = SH.shard_bounds(n, world, rank)
    shard = SH.shard_batch(hb, lo, hi)
    wire, off, st, _ = oracle_ffi.encode_batch(shard)
    totals = SH.allgather_totals(len(wire))
    bases, grand = SH.exclusive_bases(totals)
    base = int(bases[rank])
    # decode this shard's byte range alone, then rebase to global coordinates
    w = np.frombuffer(wire + b"\0" * 16, np.uint8).copy()
    msgs, unix, dst, a0, a1 = oracle_ffi.decode_batch(w, off, mode)
    gm, gu = SH.rebase_decoded(msgs, unix, lo, base)
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), wire=np.frombuffer(wire, np.uint8), off=off + np.uint64(base),
             st=st, msgs=gm.view(np.uint8), unix=gu.view(np.uint8), dst=dst, a0=a0, a1=a1,
             grand=np.array([grand], np.uint64), lo=np.array([lo]), hi=np.array([hi]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", [0, 1])
def test_two_rank_shards_concatenate_to_single_process(tmp_path, mode):
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ffi
    import onc_rpc_amd.layout as L
    import onc_rpc_amd.synth as S

    n, world = 3001, 2
    mp.start_processes(_worker, args=(world, _free_port(), n, mode, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    parts = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]

    hb = S.mixed(n, seed=21, pmin=0, pmax=300, exotic=0.2)
    wire, off, st, _ = oracle_ffi.encode_batch(hb)
    # encode: concatenated shard bytes == single-process send buffer
    assert b"".join(p["wire"].tobytes() for p in parts) == wire
    assert int(parts[0]["grand"][0]) == len(wire)
    got_off = np.concatenate([p["off"][:-1] for p in parts] + [parts[-1]["off"][-1:]])
    assert np.array_equal(got_off, off)
    assert np.array_equal(np.concatenate([p["st"] for p in parts]), st)

    # decode: rebased shard descriptors == single-process decode
    w = np.frombuffer(wire + b"\0" * 16, np.uint8).copy()
    msgs, unix, dst, a0, a1 = oracle_ffi.decode_batch(w, off, mode)
    assert np.array_equal(np.concatenate([p["dst"] for p in parts]), dst)
    gm = np.concatenate([p["msgs"] for p in parts]).view(L.MSG_DTYPE)
    gu = np.concatenate([p["unix"] for p in parts]).view(L.UNIX_DTYPE)
    # AUTH_UNIX slots are packed per 64-record group of each decode call
    # (include/onc_rpc.h onc_decoded): the shards' refs differ from the whole
    # batch's, the resolved parameters do not
    gm_r, gp = L.resolve_unix(gm, gu, dst)
    om_r, op = L.resolve_unix(msgs, unix, dst)
    assert np.array_equal(gm_r.view(np.uint8), om_r.view(np.uint8))
    assert np.array_equal(gp, op)
    assert gp.any()                       # the batch has AUTH_UNIX auths
