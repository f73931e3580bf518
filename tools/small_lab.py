"""Lab: the latency of a small encode (one message up to 512 records) —
the one-launch path (codec.hip small_batch) against the two-pass path
(enc_len + enc_emit, forced with the wave-per-tile variant bit), host wall
clock of onc_encode + onc_codec_sync, median of many calls, configs[0]'s
message. Inputs and outputs in HBM.

Usage (GPU box): python tools/small_lab.py [calls]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _onc_pkg  # noqa: E402

_onc_pkg.load()
import onc_rpc_amd.runtime as R  # noqa: E402
import onc_rpc_amd.synth as S  # noqa: E402


def main():
    import torch
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    for n in (1, 64, 512):
        hb = S.cpu_roundtrip(n)
        db = R.DeviceBatch.from_host(hb)
        out = torch.empty(192 * n + 64, dtype=torch.uint8, device="cuda")
        off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        st = torch.empty(n, dtype=torch.int32, device="cuda")
        res = []
        wires = []
        for name, variant in (("one launch", 0), ("two-pass", R.VARIANT_EMIT_TILE)):
            c = R.Codec(0, variant=variant)
            c.reserve(n)
            t = []
            for i in range(calls + 50):
                t0 = time.perf_counter()
                c.encode(db, out, off, st)
                c.sync()
                t.append(time.perf_counter() - t0)
            wires.append(out.cpu().numpy().tobytes())
            c.close()
            res.append(f"{name} {np.median(t[50:]) * 1e6:5.1f} us")
        assert wires[0] == wires[1]
        print(f"n={n:4d}: onc_encode + sync, median of {calls}: " + ", ".join(res), flush=True)


if __name__ == "__main__":
    main()
