"""Lab: encode a batch, decode it, re-encode the decoded descriptors straight
from the wire (auth_arena = payload_arena = wire: serialise(try_from(buf)))
and compare the kernels' times (HIP events, onc_codec_kernel_stats).

Usage: python tools/reencode_lab.py [c0|c1|c3] [records] [reps]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import _onc_pkg  # noqa: E402

_onc_pkg.load()
import torch  # noqa: E402

import onc_rpc_amd.layout as L  # noqa: E402
import onc_rpc_amd.runtime as R  # noqa: E402
import onc_rpc_amd.synth as S  # noqa: E402


def timed(codec, fn, reps):
    fn()
    torch.cuda.synchronize()
    codec.reset_stats()
    codec.enable_timing(True)
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    codec.enable_timing(False)
    st = codec.kernel_stats()
    return {k: 1e3 * ms / cnt for k, (ms, cnt) in st.items() if cnt}


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c0"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    hb = {"c0": lambda: S.cpu_roundtrip(n, seed=0), "c1": lambda: S.call_none(n, 256, seed=1),
          "c3": lambda: S.call_unix16(n, 1024, seed=3)}[wl]()
    codec = R.Codec(0)
    codec.reserve(n)
    db = R.DeviceBatch.from_host(hb)
    lens = R.codec_lengths(codec, db)
    total = int(lens.sum())
    out = torch.zeros(total + 16, dtype=torch.uint8, device="cuda")
    off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    t_enc = timed(codec, lambda: codec.encode(db, out, off, st), reps)
    dec = R.DecodeBuffers(n)
    codec.decode(out, off, n, L.DECODE_SLICE, dec.msgs, dec.unix, dec.status, dec.aux0, dec.aux1)
    torch.cuda.synchronize()
    assert int((dec.status[:n] != 0).sum()) == 0
    db2 = R.DeviceBatch(n, dec.msgs, dec.unix, out, out, unix_count=2 * n, auth_len=total, payload_len=total)
    out2 = torch.zeros_like(out)
    off2 = torch.empty_like(off)
    st2 = torch.empty_like(st)
    t_re = timed(codec, lambda: codec.encode(db2, out2, off2, st2), reps)
    same = torch.equal(out, out2) and torch.equal(off, off2)
    print(f"{wl} n={n} re-encode bit-exact: {same}")
    for k in sorted(set(t_enc) | set(t_re)):
        print(f"  {k:20s} first {t_enc.get(k, 0):8.1f} us   re-encode {t_re.get(k, 0):8.1f} us")
    codec.close()


if __name__ == "__main__":
    main()
