"""Lab: what the configs[2] decode pays for mixing record kinds in a wave.

The decode runs one lane per record, so a 64-record wave of configs[2]
executes the parse of every kind its records have (AUTH_NONE and AUTH_UNIX
calls, accepted and denied replies). This lab builds the same 1M records in
other orders — kinds sorted within groups of G consecutive records (what a
workgroup of G lanes could do by exchanging records among its waves), and
the whole batch sorted — encodes each into its own wire and times the
decode (onc_decode_lengths, the codec's HIP events) cold, rotating over 5
copies as bench.py --cache cold does, under each decode policy (auto: the
line/standard choice from the previous launch's sampled workgroups; forced
standard; forced line). Same records, same lengths; only which records share
a wave changes.

Usage (GPU box): python tools/sort_lab.py [records] [reps]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _onc_pkg  # noqa: E402

_onc_pkg.load()
import onc_rpc_amd.layout as L  # noqa: E402
import onc_rpc_amd.runtime as R  # noqa: E402
import onc_rpc_amd.synth as S  # noqa: E402


def kind_key(m):
    """A record's parse path: call by credential kind, reply by status."""
    call = m["msg_type"] == 0
    cred = (m["cred_kind_len"] >> 24).astype(np.int64)
    reply = 100 + 10 * m["reply_stat"].astype(np.int64) + m["stat"].astype(np.int64)
    return np.where(call, cred, reply)


def order(key, g):
    n = len(key)
    if g >= n:
        return np.argsort(key, kind="stable")
    idx = np.arange(n)
    grp = idx // g
    return np.lexsort((idx, key, grp))      # by group, then kind, then position


def main():
    import torch
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    hb = S.mixed(n, seed=2)
    key = kind_key(hb.msgs)
    kinds, counts = np.unique(key, return_counts=True)
    print("kinds (key: records):", dict(zip(kinds.tolist(), counts.tolist())), flush=True)
    c = R.Codec(0)
    c.reserve(n)
    # the AUTH_UNIX credentials replaced by AUTH_NONE, the record kept as long
    # (the payload grows by the credential body; the arena is long enough)
    nu = hb.msgs.copy()
    isu = (nu["msg_type"] == 0) & ((nu["cred_kind_len"] >> 24) == L.KIND_UNIX)
    grow = (nu["cred_kind_len"][isu] & 0xFFFFFF).astype(np.uint32)
    room = len(hb.payload_arena) - (nu["payload_off"][isu] + nu["payload_len"][isu])
    nu["payload_len"][isu] += np.minimum(grow, room).astype(np.uint32)
    nu["cred_kind_len"][isu] = L.pack_kind_len(L.KIND_NONE, 0)
    nu["cred_id"][isu] = 0
    nu["cred_ref"][isu] = 0
    for name, g in (("as generated", 1), ("sorted in groups of 128", 128), ("sorted in groups of 256", 256),
                    ("sorted in groups of 1024", 1024), ("whole batch sorted", n),
                    ("no AUTH_UNIX (AUTH_NONE, same lengths)", 0)):
        perm = np.arange(n) if g <= 1 else order(key, g)
        hbp = L.HostBatch((nu if g == 0 else hb.msgs)[perm].copy(), hb.unix, hb.auth_arena, hb.payload_arena)
        db = R.DeviceBatch.from_host(hbp)
        rl = torch.empty(n, dtype=torch.int32, device="cuda")
        st = torch.empty(n, dtype=torch.int32, device="cuda")
        c.encode_lengths(db, rl, st)
        total = int(rl.cpu().numpy().view(np.uint32).astype(np.int64).sum())
        wire = torch.zeros(total + 16, dtype=torch.uint8, device="cuda")
        off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        c.encode(db, wire, off, st, rl)
        c.sync()
        assert (st == 0).all()
        dec = R.DecodeBuffers(n)
        copies = [wire] + [wire.clone() for _ in range(4)]
        res = []
        for pol, pname in ((R.DECODE_POLICY_AUTO, "auto"), (R.DECODE_POLICY_STANDARD, "standard"),
                           (R.DECODE_POLICY_LINE, "line")):
            c.set_decode_policy(pol)
            c.reset_stats()
            c.enable_timing(True, kernels=[R.K_DEC_PARSE])
            for i in range(reps + 2):
                c.decode_lengths(copies[i % 5], rl, n, 0, L.DECODE_SLICE, dec.msgs, dec.unix, dec.status, dec.aux0,
                                 dec.aux1)
            ms, cnt = c.kernel_stats()["decode_kernel"]
            c.enable_timing(False)
            c.sync()
            assert (dec.status[:n] == 0).all()
            # the decoded descriptors match the (permuted) input's fields
            got = dec.to_host()[0]
            assert (got["xid"] == hbp.msgs["xid"]).all() and (got["payload_len"] == hbp.msgs["payload_len"]).all()
            res.append(f"{pname} {ms / cnt * 1e3:6.1f}")
        c.set_decode_policy(R.DECODE_POLICY_AUTO)
        print(f"{name:40s} decode us (cold, 5 copies): " + ", ".join(res), flush=True)
        del copies, wire, dec, db
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
