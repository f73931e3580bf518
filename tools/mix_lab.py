"""Lab: the enc_emit kernel choice on batches whose head and tail differ
(round-4 verdict item 7). 1M records: a header-heavy half (configs[0]'s
message: AUTH_UNIX with 16 gids + 64 B payload) and a payload-heavy half
(configs[1]'s: AUTH_NONE + 256 B), in both orders. Each batch is encoded
with the codec's own choice and with each kernel forced (ONC_VARIANT_*:
0x400 the wave-per-tile kernel, 0x10200 the wave-specialised pipeline on
every shape, 0x200 the wave-specialised kernel with its header-heavy
fallback), enc_emit timed with the codec's HIP events; every output is
checked equal to the automatic choice's.

Usage (GPU box): python tools/mix_lab.py [records] [reps]
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


def concat(a, b):
    """HostBatch a followed by b (b's references rebased onto the joined arenas)."""
    m2 = b.msgs.copy()
    m2["payload_off"] += np.uint64(a.payload_arena.nbytes)
    for f in ("cred", "verf"):
        unix = (m2[f + "_kind_len"] >> 24) == L.KIND_UNIX
        m2[f + "_ref"][unix] += np.uint64(len(a.unix))
        m2[f + "_ref"][~unix] += np.uint64(a.auth_arena.nbytes)
    u2 = b.unix.copy()
    u2["name_off"] += np.uint64(a.auth_arena.nbytes)
    return L.HostBatch(np.concatenate([a.msgs, m2]), np.concatenate([a.unix, u2]),
                       np.concatenate([a.auth_arena, b.auth_arena]), np.concatenate([a.payload_arena, b.payload_arena]))


def emit_us(db, n, var, reps):
    import torch
    c = R.Codec(0, variant=var)
    c.reserve(n)
    lens = R.codec_lengths(c, db)
    total = int(lens.sum())
    out = torch.zeros(total + 64, dtype=torch.uint8, device="cuda")
    off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    for _ in range(3):
        c.encode(db, out, off, st)
    c.sync()
    c.reset_stats()
    c.enable_timing(True, kernels=[R.K_ENC_EMIT])
    for _ in range(reps):
        c.encode(db, out, off, st)
    ms, cnt = c.kernel_stats()["enc_emit_kernel"]
    c.close()
    return ms / cnt * 1e3, total


def sweep(n, reps):
    """tile (0x400) against the wave-specialised pipeline (0x10200) over
    payload / header ratios: AUTH_NONE calls (44-byte headers) and AUTH_UNIX
    16-gid calls (128-byte headers) at several payload sizes, and c0/c1
    mixes; prints payload bytes per header byte and both times."""
    shapes = []
    for p in (64, 128, 192, 256, 384):
        shapes.append((f"none_p{p}", S.call_none(n, p, seed=p)))
    for p in (64, 256, 512, 1024):
        shapes.append((f"unix16_p{p}", S.call_unix16(n, p, seed=p)))
    for q in (4, 2):
        k = n // q
        shapes.append((f"c0x1/{q}+c1", concat(S.cpu_roundtrip(k, seed=5), S.call_none(n - k, 256, seed=6))))
    shapes.append(("c0x3/4+c1", concat(S.cpu_roundtrip(3 * n // 4, seed=7), S.call_none(n - 3 * n // 4, 256, seed=8))))
    for name, hb in shapes:
        db = R.DeviceBatch.from_host(hb)
        pay = int(hb.msgs["payload_len"].astype(np.int64).sum())
        t_tile, total = emit_us(db, hb.n, 0x400, reps)
        t_ws, _ = emit_us(db, hb.n, 0x10200, reps)
        t_auto, _ = emit_us(db, hb.n, 0, reps)
        hdr = total - pay
        print(f"{name:14s} payload/header {pay / hdr:5.2f}  header/rec {hdr / hb.n:6.1f}  tile {t_tile:7.1f}  "
              f"ws_pipeline {t_ws:7.1f}  auto {t_auto:7.1f}  best {'ws' if t_ws < t_tile else 'tile'}", flush=True)


def main():
    import torch
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    if len(sys.argv) > 3 and sys.argv[3] == "sweep":
        sweep(n, reps)
        return
    heavy = S.cpu_roundtrip(n // 2, seed=1)
    light = S.call_none(n - n // 2, 256, seed=2)
    cases = {"auto": 0, "tile": 0x400, "ws_pipeline": 0x10200, "ws_fallback": 0x200}
    for order, hb in (("heavy_then_light", concat(heavy, light)), ("light_then_heavy", concat(light, heavy))):
        db = R.DeviceBatch.from_host(hb)
        ref = None
        res = {}
        for name, var in cases.items():
            c = R.Codec(0, variant=var)
            c.reserve(hb.n)
            total = int(R.codec_lengths(c, db).sum())
            out = torch.zeros(total + 64, dtype=torch.uint8, device="cuda")
            off = torch.empty(hb.n + 1, dtype=torch.int64, device="cuda")
            st = torch.empty(hb.n, dtype=torch.int32, device="cuda")
            for _ in range(3):
                c.encode(db, out, off, st)
            c.sync()
            c.reset_stats()
            c.enable_timing(True, kernels=[R.K_ENC_EMIT])
            for _ in range(reps):
                c.encode(db, out, off, st)
            ms, cnt = c.kernel_stats()["enc_emit_kernel"]
            c.enable_timing(False)
            res[name] = ms / cnt * 1e3
            b = out[:total].cpu().numpy().tobytes()
            assert (st.cpu().numpy() == 0).all()
            if ref is None:
                ref = b
            assert b == ref, f"{order} {name}: output differs"
            c.close()
        best = min(v for k, v in res.items() if k != "auto")
        print(order, {k: round(v, 1) for k, v in res.items()}, "auto / best forced", round(res["auto"] / best, 3),
              flush=True)


if __name__ == "__main__":
    main()
