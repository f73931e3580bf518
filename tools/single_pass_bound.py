"""Upper bound of a single-pass encode (lab; SURVEY §8(d) configs[1] step).

A single-pass encode would place tiles inside enc_emit (decoupled look-back
over dynamically claimed tiles) and drop the enc_len launch. Its best case is
the step with enc_len's time removed and nothing added: that is measured here
by planning the batch once (onc_encode_plan) and timing steps of
onc_encode_emit + onc_decode of the same batch (the plan stays valid: the
descriptors never change), interleaved with the product step (onc_encode +
onc_decode), on one box. Prints both per-step times and the ratio.

Usage: python tools/single_pass_bound.py [workload c1|c0|c3] [records] [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import _onc_pkg
    _onc_pkg.load()
    import onc_rpc_amd.layout as L
    import onc_rpc_amd.runtime as R
    import onc_rpc_amd.synth as S

    wl = sys.argv[1] if len(sys.argv) > 1 else "c1"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    hb = {"c1": lambda: S.call_none(n, 256, seed=1), "c0": lambda: S.cpu_roundtrip(n, seed=0),
          "c3": lambda: S.call_unix16(n, 1024, seed=3)}[wl]()
    db = R.DeviceBatch.from_host(hb)
    c = R.Codec(0)
    c.reserve(n)
    total = int(R.codec_lengths(c, db).sum())
    out = torch.zeros(total + 16, dtype=torch.uint8, device="cuda")
    off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    d = R.DecodeBuffers(n)

    def full():
        c.encode(db, out, off, st)
        c.decode(out, off, n, L.DECODE_SLICE, d.msgs, d.unix, d.status, d.aux0, d.aux1)

    def emit_only():
        c.encode_emit(db, out, off, st)
        c.decode(out, off, n, L.DECODE_SLICE, d.msgs, d.unix, d.status, d.aux0, d.aux1)

    def timed(fn, steps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / steps * 1e3

    res = {"full": [], "emit_only": []}
    for _ in range(reps):
        res["full"].append(timed(full))
        c.encode_plan(db, st)            # plan once; every emit_only step re-emits from it
        torch.cuda.synchronize()
        res["emit_only"].append(timed(emit_only))
        ok = int((st != 0).sum()) == 0 and int((d.status[:n] != 0).sum()) == 0 and int(off[n]) == total
        assert ok
    f, e = float(np.median(res["full"])), float(np.median(res["emit_only"]))
    print(f"{wl} n={n}: step us full (enc_len + enc_emit + decode) median {f:.1f} {sorted(round(x, 1) for x in res['full'])}")
    print(f"{wl} n={n}: step us emit from a standing plan (enc_emit + decode) median {e:.1f} "
          f"{sorted(round(x, 1) for x in res['emit_only'])}")
    print(f"{wl}: upper bound of a single-pass encode: {100 * (f / e - 1):.1f} % more Mmsgs/s "
          f"({n / f:.0f} -> {n / e:.0f} Mmsgs/s)")
    c.close()


if __name__ == "__main__":
    main()
