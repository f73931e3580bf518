"""Lab: configs[1] encode -> decode steps with two batches in flight.

bench.py's step runs the encode and the decode of one batch on one stream,
one step after the other. A server encodes batch k+1 while it decodes batch
k; this lab measures what that buys on one MI355X: the same step on two
codecs with their own streams (and their own wire / decode buffers),
alternating, so that one codec's enc_emit can run next to the other's
decode. Host wall clock over K steps between device synchronisations,
median of R rounds; every codec's last wire and decode are checked against
the one-stream run's.

Usage (GPU box): python tools/overlap_lab.py [records] [steps] [rounds]
"""
import os
import sys
import time

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
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 7
    hb = S.call_none(n, 256, seed=1)
    db = R.DeviceBatch.from_host(hb)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    codecs = [R.Codec(0, stream=s.cuda_stream) for s in streams]
    for c in codecs:
        c.reserve(n)
    rl = torch.empty(n, dtype=torch.int32, device="cuda")
    st0 = torch.empty(n, dtype=torch.int32, device="cuda")
    codecs[0].encode_lengths(db, rl, st0)
    codecs[0].sync()
    total = int(rl.cpu().numpy().view(np.uint32).astype(np.int64).sum())
    bufs = []
    for _ in codecs:
        bufs.append(dict(out=torch.zeros(total + 16, dtype=torch.uint8, device="cuda"),
                         off=torch.empty(n + 1, dtype=torch.int64, device="cuda"),
                         st=torch.empty(n, dtype=torch.int32, device="cuda"),
                         dec=R.DecodeBuffers(n)))

    def step(k):
        c, b = codecs[k], bufs[k]
        c.encode(db, b["out"], b["off"], b["st"])
        c.decode(b["out"], b["off"], n, L.DECODE_SLICE, b["dec"].msgs, b["dec"].unix, b["dec"].status,
                 b["dec"].aux0, b["dec"].aux1)

    def timed(pattern):
        ts = []
        for _ in range(rounds):
            for i in range(4):
                step(pattern(i))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(steps):
                step(pattern(i))
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / steps * 1e6)
        return float(np.median(ts)), float(min(ts))

    one, one_min = timed(lambda i: 0)
    two, two_min = timed(lambda i: i & 1)
    ref = (bufs[0]["out"].cpu().numpy().tobytes(), bufs[0]["dec"].msgs.cpu().numpy().tobytes())
    for b in bufs:
        assert (b["st"] == 0).all() and (b["dec"].status == 0).all()
        assert b["out"].cpu().numpy().tobytes() == ref[0] and b["dec"].msgs.cpu().numpy().tobytes() == ref[1]
    print(f"n={n} steps={steps} rounds={rounds}: one stream {one:.1f} us/step (min {one_min:.1f}), "
          f"{n / one:.0f} Mmsgs/s; two codecs on two streams, alternating {two:.1f} us/step (min {two_min:.1f}), "
          f"{n / two:.0f} Mmsgs/s; outputs checked equal", flush=True)


if __name__ == "__main__":
    main()
