"""Lab: the configs[2] decode against its own memory access pattern.

Times, on the real c2 wire (bench.py's synthetic mixed Call/Reply batch):
  decode  — the product decode step (onc_decode_lengths, kernel timing)
  loads   — tools/line_lab.hip: the same header-window loads, no parse
  loads+o — the loads plus the decode's 76 B/record of output stores
so the decode's time can be set against what its loads and stores alone cost.

Usage: python tools/line_lab.py [records] [reps]   (needs tools/libline_lab.so)
"""
import ctypes
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


def ev_time(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return float(np.median(ts))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libline_lab.so"))
    lib.line_lab_run.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64] + [ctypes.c_void_p] * 2 + \
        [ctypes.c_int, ctypes.c_void_p]
    hb = S.mixed(n, seed=2)
    codec = R.Codec(0)
    codec.reserve(n)
    db = R.DeviceBatch.from_host(hb)
    rec_len = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    codec.encode_lengths(db, rec_len, st)
    lens = rec_len.cpu().numpy().view(np.uint32).astype(np.int64)
    total = int(lens.sum())
    wire = torch.zeros(total + 16, dtype=torch.uint8, device="cuda")
    off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    codec.encode(db, wire, off, st, rec_len)
    dec = R.DecodeBuffers(n)
    dec_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    unix_cred = (hb.msgs["cred_kind_len"] >> 24) == L.KIND_UNIX
    hdr_np = (lens - hb.msgs["payload_len"].astype(np.int64)).astype(np.uint32)
    hdr = torch.from_numpy((hdr_np | np.where(unix_cred, 0x80000000, 0).astype(np.uint32)).view(np.int32)).cuda()
    sink = torch.empty(n, dtype=torch.int32, device="cuda")
    out = torch.empty(n * (76 + 192) + 64, dtype=torch.uint8, device="cuda")

    def decode():
        codec.decode_lengths(wire, rec_len, n, 0, L.DECODE_SLICE, dec.msgs, dec.unix, dec.status, dec.aux0,
                             dec.aux1, rec_off=dec_off)

    def lab(with_out):
        s = torch.cuda.current_stream().cuda_stream
        rc = lib.line_lab_run(wire.data_ptr(), off.data_ptr(), hdr.data_ptr(), n, sink.data_ptr(), out.data_ptr(),
                              with_out, s)
        assert rc == 0

    t_dec = ev_time(decode, reps)
    assert int((dec.status != 0).sum()) == 0
    t_a = ev_time(lambda: lab(0), reps)
    t_b = ev_time(lambda: lab(1), reps)
    t_c = ev_time(lambda: lab(2), reps)
    t_d = ev_time(lambda: lab(3), reps)
    t_e = ev_time(lambda: lab(4), reps)
    t_f = ev_time(lambda: lab(5), reps)
    t_g = ev_time(lambda: lab(6), reps)
    w0 = off.cpu().numpy()
    base = w0[:-1] & 15
    hl = hdr_np.astype(np.int64)
    want = np.minimum((base + np.minimum(hl, np.minimum(lens, 160 - base)) + 15) >> 4, 10)
    lines = ((w0[:-1] + want * 16 - 1) >> 7) - (w0[:-1] >> 7) + 1
    print(f"c2 n={n} wire {total / 1e9:.3f} GB, header extent mean {hl.mean():.1f} B, "
          f"128-B lines touched {lines.sum() / n:.3f}/record")
    print(f"  decode (product)       {t_dec:8.1f} us")
    print(f"  loads only             {t_a:8.1f} us")
    print(f"  loads + 76 B/rec out   {t_b:8.1f} us")
    print(f"  loads, 10 KiB LDS/wg   {t_c:8.1f} us   (the decode's occupancy: 4 waves/SIMD)")
    print(f"  loads + out, 10 KiB    {t_d:8.1f} us")
    print(f"  + AUTH_UNIX slots      {t_e:8.1f} us   ({unix_cred.mean():.3f} of records, 128 B each at 192 B * i)")
    print(f"  + slots, nontemporal   {t_f:8.1f} us")
    print(f"  + slots, compacted     {t_g:8.1f} us   (96 B each, consecutive per wave)")
    codec.close()


if __name__ == "__main__":
    main()
