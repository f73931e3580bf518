"""Multi-GPU partitioning of a record batch.

Records are independent (the reference API is one message per call with no
shared state, src/rpc_message.rs:235-271 / :136-164), so a batch shards by
contiguous record ranges with NO data-path collective. The only cross-rank
fact is each shard's encoded byte total; an exclusive scan of those G
numbers gives every shard's base offset in the global send buffer (a
control-plane all_gather of one int64 per rank).

Decode shards the same way: rank k takes records [lo_k, hi_k) and the wire
byte range [rec_off[lo_k], rec_off[hi_k]); offsets inside a shard are
local and are rebased by the shard's byte base.
"""
from __future__ import annotations

import numpy as np

from . import layout as L


def shard_bounds(n: int, world: int, rank: int):
    """Contiguous record range [lo, hi) of `rank` (balanced to within 1)."""
    return n * rank // world, n * (rank + 1) // world


def exclusive_bases(totals):
    """Per-shard byte totals (rank order) -> per-shard base offsets and grand total."""
    t = np.asarray(totals, dtype=np.uint64)
    base = np.zeros(len(t), np.uint64)
    if len(t) > 1:
        np.cumsum(t[:-1], out=base[1:])
    return base, int(t.sum())


def allgather_totals(local_total: int, group=None):
    """all_gather one int64 per rank (control plane; CPU tensor works with
    gloo, a CUDA tensor with nccl/RCCL)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    backend = dist.get_backend(group)
    dev = "cuda" if backend == "nccl" else "cpu"
    t = torch.tensor([int(local_total)], dtype=torch.int64, device=dev)
    outs = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    return [int(o.item()) for o in outs]


def shard_batch(hb: L.HostBatch, lo: int, hi: int) -> L.HostBatch:
    """The descriptors of records [lo, hi) (arenas shared, offsets unchanged)."""
    return L.HostBatch(hb.msgs[lo:hi].copy(), hb.unix, hb.auth_arena, hb.payload_arena)


def rebase_decoded(msgs, unix, rec_lo: int, byte_base: int):
    """Shard-local decode output -> global coordinates: wire offsets + byte_base,
    AUTH_UNIX slot indices + 2*rec_lo (unix slot contents are moved by the
    caller by concatenation in rank order)."""
    m = msgs.copy()
    u = unix.copy()
    # descriptors of failed records are all zero in both coordinate systems
    live = ~(msgs.view(np.uint8).reshape(len(msgs), 64) == 0).all(axis=1) if len(msgs) else np.zeros(0, bool)
    call = live & (m["msg_type"] == L.MSG_CALL)
    accepted = live & (m["msg_type"] == L.MSG_REPLY) & (m["reply_stat"] == L.REPLY_ACCEPTED)
    has_payload = call | (accepted & (m["stat"] == 0))
    m["payload_off"][has_payload] += np.uint64(byte_base)
    for f, used in (("cred", call), ("verf", call | accepted)):
        is_unix = used & ((m[f + "_kind_len"] >> 24) == L.KIND_UNIX)
        opaque = used & ~is_unix
        m[f + "_ref"][is_unix] += np.uint64(2 * rec_lo)
        m[f + "_ref"][opaque] += np.uint64(byte_base)
    u["name_off"] += np.uint64(byte_base)
    return m, u
