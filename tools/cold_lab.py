"""Lab: how cold is "cold"? configs[2]'s decode (onc_decode_lengths of 1M
mixed records) timed with the codec's HIP events while rotating over K
identical wire copies (K = 1 is the warm case; bench.py --cache cold uses
K = 5), and with an untimed 1 GiB scrub of another buffer before every
decode of one copy: a write scrub (torch fill: leaves L2 + Infinity Cache
full of dirty lines, written back while the decode reads) and a read scrub
(torch sum: evicts without dirtying). If the K >= 3 times and the read-scrub
time agree, the rotation reaches the clean cold steady state.

Usage (GPU box): python tools/cold_lab.py [records] [reps]
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


def main():
    import torch
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    hb = S.mixed(n, seed=2)
    db = R.DeviceBatch.from_host(hb)
    c = R.Codec(0)
    c.reserve(n)
    rl = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    c.encode_lengths(db, rl, st)
    total = int(rl.cpu().numpy().view(np.uint32).astype(np.int64).sum())
    wire = torch.zeros(total + 16, dtype=torch.uint8, device="cuda")
    off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    c.encode(db, wire, off, st, rl)
    c.sync()
    dec = R.DecodeBuffers(n)
    copies = [wire] + [wire.clone() for _ in range(8)]
    scrub = torch.ones(1 << 30, dtype=torch.uint8, device="cuda")
    scrub_words = scrub.view(torch.int32)
    sink = torch.zeros(2, dtype=torch.int64, device="cuda")

    def run(k, do_scrub=None):
        c.sync()
        c.reset_stats()
        c.enable_timing(True, kernels=[R.K_DEC_PARSE])
        for i in range(reps + 2):
            if do_scrub == "write":
                scrub.fill_(i & 0xFF)
            elif do_scrub == "read":
                sink[i % 2] = scrub_words.sum()
            c.decode_lengths(copies[i % k], rl, n, 0, L.DECODE_SLICE, dec.msgs, dec.unix, dec.status, dec.aux0,
                             dec.aux1)
        ms, cnt = c.kernel_stats()["decode_kernel"]
        c.enable_timing(False)
        assert (dec.status[:n] == 0).all()
        return ms / cnt * 1e3

    for k in (1, 2, 3, 5, 9):
        print(f"copies {k}: decode {run(k):.1f} us", flush=True)
    for kind in ("write", "read"):
        print(f"1 GiB {kind} scrub before each decode of one copy: decode {run(1, kind):.1f} us", flush=True)
        print(f"1 GiB {kind} scrub + 5 copies: decode {run(5, kind):.1f} us", flush=True)


if __name__ == "__main__":
    main()
