#!/usr/bin/env python3
"""Headline benchmark: device-resident ONC-RPC encode+decode on MI355X.

BASELINE.json metric: "device-resident ONC-RPC encode+decode: Mmsgs/s and
GiB/s vs HBM roofline". One step = one pass of the hot path over one batch:
RpcMessage::serialise_into of every record into one send buffer
(src/rpc_message.rs:136-164) followed by RpcMessage::try_from of every
record of that buffer (src/rpc_message.rs:235-271), inputs resident in HBM.

Workloads (--workload; the default is the headline line):
  c1  configs[1] — 1M Call(prog 100003, vers 4, proc 1, AuthNone(None) x2)
      + 256 B random payload (W = 300 B) per GPU, encode -> decode loopback
      (weak scaling: every rank its own 1M records).
  c2  configs[2] — 1M mixed Call/Reply, payloads 64..4096 B: decode step =
      scan of rec_len into offsets + decode (input wire encoded once, untimed).
  c3  configs[3] — 4M Call(AuthUnix 16 gids) + 1 KiB payload (W = 1152),
      encode -> decode loopback.
  c0  configs[0]'s message (benches/bench.rs:86-101) as a 1M batch.
  c4  configs[4] — 64M configs[1] records IN TOTAL, sharded contiguously
      over the ranks (64M / 32M / 16M / 8M per GPU at 1 / 2 / 4 / 8 GPUs:
      strong scaling), generated on the device; per-GPU and aggregate
      Mmsgs/s, every shard's base in the global send buffer from one
      all_gather of the byte totals (no data-path collective).
Unless --c4-leg off, a run of c0..c3 also runs the configs[4] leg after the
headline and reports it as `configs4` in the same JSON line (so the
driver's 1/2/4/8-GPU runs record configs[4] at every N).

Launch: `python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the
environment starts N ranks itself (python -m torch.distributed.run, one
process per GPU, as a child process before any GPU call) and exits with
their status; under torch.distributed.run (WORLD_SIZE set) every rank
checks that the world size equals --gpus.

Besides the device-resident `value`, every run also times the PCIe-inclusive
rate (pinned host inputs -> H2D -> kernels -> D2H of the outputs), reported
as `pcie_inclusive` (never as `value`).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident ONC-RPC encode+decode: Mmsgs/s and GiB/s vs HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)
DEFAULT_RECORDS = {"c0": 1_000_000, "c1": 1_000_000, "c2": 1_000_000, "c3": 4_000_000, "c4": 64_000_000}
C4_W, C4_H = 300, 44          # configs[4] record: wire bytes / parsed header bytes


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs, one rank each (default: WORLD_SIZE or 1); N > 1 without WORLD_SIZE spawns N ranks")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=["c0", "c1", "c2", "c3", "c4"], default="c1")
    ap.add_argument("--records", type=int, default=None, help="records per GPU (c0-c3) / in total (c4)")
    ap.add_argument("--c4-leg", choices=["on", "off"], default="on",
                    help="also run the configs[4] strong-scaling leg after a c0..c3 headline")
    ap.add_argument("--c4-records", type=int, default=DEFAULT_RECORDS["c4"], help="configs[4] leg: records in total")
    ap.add_argument("--mode", choices=["slice", "bytes"], default="slice")
    ap.add_argument("--frame", action="store_true",
                    help="c2: frame the raw stream on the device (onc_frame_stream) instead of scanning rec_len")
    ap.add_argument("--iov", action="store_true",
                    help="c0/c1/c3: the step is the vectored encode (onc_encode_iov: packed headers + one iovec "
                         "per record, payloads referenced in place) instead of encode + decode")
    ap.add_argument("--iov-leg", choices=["on", "off"], default="on",
                    help="with the c1 workload: also run the vectored encode of the same configs[1] batch and report "
                         "it as `vectored_encode`")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend of the ranks (control plane only)")
    ap.add_argument("--check-launch", action="store_true",
                    help="start the ranks, check the world size and print it; no GPU work (launcher test)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU-baseline threads (0 = every core available)")
    ap.add_argument("--pcie-reps", type=int, default=3)
    ap.add_argument("--pcie-chunks", type=int, default=8,
                    help="record chunks of the pipelined PCIe-inclusive leg (two streams)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-check-records", type=int, default=0,
                    help="--check-launch only: rehearse the closing CPU-baseline step on this many records")
    ap.add_argument("--no-pcie", action="store_true")
    ap.add_argument("--traffic-json", default=None,
                    help="per-kernel PMC traffic (default: the newest profiles/traffic_rNN[_<workload>].json)")
    ap.add_argument("--cache", choices=["cold", "warm"], default="cold",
                    help="c2: cold = every step decodes another of K identical wire copies, so the header lines a "
                         "step reads were last touched >= 2x the 256 MiB Infinity Cache of other traffic ago; "
                         "warm = the same wire every step")
    ap.add_argument("--cache-leg", choices=["on", "off"], default="on",
                    help="also measure the other cache state (c2: warm; c1: decode-only legs, warm and cold) and "
                         "report it next to the primary line")
    ap.add_argument("--decode-policy", choices=["auto", "standard", "line"], default="auto",
                    help="pin the decode's first-round policy for every codec of the run (A/B measurements)")
    ap.add_argument("--variant", type=lambda s: int(s, 0), default=0,
                    help="kernel variant bits (onc_codec_options.variant; A/B measurements only)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# launcher
# ---------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(gpus, argv):
    """One process per GPU under torch.distributed.run, started as a child
    (this process never touches the GPU); returns their exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd, env=dict(os.environ))


def check_launch(args, world, rank):
    """--check-launch: the ranks rendezvous, all_gather (rank, pid) and rank 0
    prints the world as the process group sees it. No GPU call. With
    --cpu-seconds > 0 the line also goes through the same closing step as a
    GPU run (finish(): rank 0 times the CPU baseline after every rank's legs,
    the others at the barrier) on a small configs[1] sample whose "GPU wire"
    is the oracle's own encoding (CPU-only rehearsal of the N > 1 path)."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group(args.backend)
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
        t = torch.tensor([rank, os.getpid()], dtype=torch.int64)
        outs = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(outs, t)
        ranks = [[int(x) for x in o] for o in outs]
    else:
        ranks = [[0, os.getpid()]]
        dist = None
    result = {"check_launch": True, "n_gpus": world, "gpus_arg": args.gpus, "ranks": ranks,
              "backend": args.backend if world > 1 else None}
    pending = None
    if rank == 0 and args.cpu_check_records:
        import numpy as np
        import _onc_pkg
        _onc_pkg.load()
        import onc_rpc_amd.synth as S
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_ffi
        hb = S.call_none(args.cpu_check_records, 256, seed=1)
        wire, off, _, _ = oracle_ffi.encode_batch(hb)
        pending = ("c1", hb, wire, np.frombuffer(wire + b"\0" * 16, np.uint8), off, 0)
    finish(args, result, pending, dist, rank, world)
    if dist is not None:
        dist.destroy_process_group()


# ---------------------------------------------------------------------------
# CPU baseline
# ---------------------------------------------------------------------------
def cpu_info():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model, os.cpu_count()


def cpu_available():
    """CPUs this process may use: its affinity mask, capped by the cgroup
    CPU quota (cpu.max) when one is set."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    return (min(n, quota) if quota else n), n, quota


def native_oracle():
    """The oracle compiled -O3 -march=native for THIS host (BASELINE.md's
    CPU-baseline build), cached per CPU model/flags and oracle source under
    oracle/_native.
    Returns (path, flags) or (None, reason) when gcc is unavailable."""
    import hashlib
    try:
        with open("/proc/cpuinfo") as f:
            first = f.read().split("\n\n")[0]
    except OSError:
        first = ""
    h = hashlib.sha1(first.encode())
    for src in ("onc_oracle.c", "onc_oracle.h"):      # a source change rebuilds it
        with open(os.path.join(ROOT, "oracle", src), "rb") as f:
            h.update(f.read())
    key = h.hexdigest()[:12]
    d = os.path.join(ROOT, "oracle", "_native", key)
    so = os.path.join(d, "liboncoracle.so")
    flags = ["-O3", "-march=native", "-std=c11", "-fPIC", "-shared"]
    if not os.path.exists(so):
        os.makedirs(d, exist_ok=True)
        tmp = so + f".{os.getpid()}"
        try:
            subprocess.check_call(["gcc", *flags, "-o", tmp, os.path.join(ROOT, "oracle", "onc_oracle.c"), "-lpthread"])
            os.replace(tmp, so)
        except (OSError, subprocess.CalledProcessError) as e:
            return None, f"native build failed ({e}); prebuilt -O2 oracle used"
    return so, " ".join(flags)


def parsed_bytes(hb, rec_len):
    """H per record (SURVEY §8 notation): wire bytes minus the payload and
    minus opaque bodies + padding, which a zero-copy decode returns as slices."""
    import numpy as np
    import onc_rpc_amd.layout as L
    m = hb.msgs
    h = rec_len.astype(np.int64) - m["payload_len"].astype(np.int64)
    for f in ("cred", "verf"):
        kl = m[f + "_kind_len"]
        kind = kl >> 24
        ln = (kl & 0xFFFFFF).astype(np.int64)
        h -= np.where(kind != L.KIND_UNIX, (ln + 3) // 4 * 4, 0)
        isu = kind == L.KIND_UNIX
        if isu.any():
            nl = hb.unix["name_len"][m[f + "_ref"][isu].astype(np.int64)].astype(np.int64)
            h[isu] -= (nl + 3) // 4 * 4
    return h


def cpu_baseline(args, wl, hb, gpu_wire_prefix, wire_np, rec_off_np, mode):
    """Oracle (C restatement of the reference, compiled -O3 -march=native on
    this host) on the GPU box's host cores, on a bounded sample of the same
    workload: every available core over whole batches (contiguous record
    partition), and 1 thread on 20k-record slices. Also checks a slice of
    the CPU output against the GPU's bytes."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np

    import oracle_ffi
    import onc_rpc_amd.layout as L

    so, build = native_oracle()
    if so:
        oracle_ffi.use_library(so)
    model, ncpu = cpu_info()
    avail, affinity, quota = cpu_available()
    threads = args.cpu_threads if args.cpu_threads > 0 else avail
    decode_only = wl == "c2"
    chunk = min(20_000, hb.n)
    sub = L.HostBatch(hb.msgs[:chunk].copy(), hb.unix, hb.auth_arena, hb.payload_arena)
    wire, off, st, _ = oracle_ffi.encode_batch(sub)
    parity = wire == gpu_wire_prefix[: len(wire)]

    def run(seconds, fn, per):
        done = 0
        t0 = time.perf_counter()
        while True:
            fn()
            done += per
            el = time.perf_counter() - t0
            if el >= seconds:
                return done, el

    # single thread, 20k-record slices
    w1 = np.frombuffer(wire + b"\0" * 16, np.uint8)

    def one():
        if not decode_only:
            oracle_ffi.encode_batch(sub)
        oracle_ffi.decode_batch(w1, off, mode)
    d1, e1 = run(args.cpu_seconds / 2, one, chunk)

    # all threads, whole batch
    if decode_only:
        def many():
            oracle_ffi.decode_batch(wire_np, rec_off_np, mode, threads=threads)
    else:
        buf = np.zeros(int(rec_off_np[-1]) + 16, np.uint8)

        def many():
            out, ro, _, _ = oracle_ffi.encode_batch_mt(hb, threads, out=buf)
            oracle_ffi.decode_batch(out, ro, mode, threads=threads)
    dn, en = run(args.cpu_seconds / 2, many, hb.n)
    what = "decode" if decode_only else "encode+decode round trip"
    return {
        "value": dn / en / 1e6,
        "unit": "Mmsgs/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{dn} records ({hb.n}-record batches of the same {wl} workload, {what}) in "
                  f"{en:.1f} s on {threads} threads (contiguous record partition) of a {ncpu}-CPU host ({model}); "
                  f"oracle built {build}",
        "host_cpus": ncpu, "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
        "single_thread": {"value": d1 / e1 / 1e6, "unit": "Mmsgs/s", "cores": 1,
                          "sample": f"{d1} records ({chunk}-record slices) in {e1:.1f} s"},
        "sample_bit_exact_vs_gpu": bool(parity),
    }


# ---------------------------------------------------------------------------
# PCIe-inclusive legs
# ---------------------------------------------------------------------------
def pcie_pipelined(args, torch, R, wl, hb, db, out, total_bytes, lens_np, rec_len, dec_off, dec, mode, h_in,
                   local_rank, dist, n_total):
    """PCIe-inclusive rate with the copies overlapped: the batch is cut into
    --pcie-chunks record ranges that flow through three streams — H2D on a
    copy-in stream, kernels on the codec's stream, D2H on a copy-out stream,
    chained per chunk by events — so chunk k+1's H2D and chunk k-1's D2H run
    in both directions of the link (one DMA engine each) under chunk k's
    kernels (measured on the box: one-direction copies 57 GB/s; H2D and D2H
    interleaved on two streams 86 GB/s; both directions from one stream do
    not overlap). Every output of a chunk (wire, offsets, statuses, decoded
    descriptors, aux words, and the AUTH_UNIX slots when the chunk has
    AUTH_UNIX auths) is written by the kernels into one device slab and comes
    back as ONE copy (7 copies per chunk before: the per-copy cost showed as a
    drop from 8 to 16 chunks); the chunks' copy lists, sub-batches and slab
    views are built before the timed region, so the timed loop only issues.
    Every byte of the serialized leg is still copied."""
    import numpy as np
    n = hb.n
    K = max(1, min(args.pcie_chunks, n))
    bounds = [(k * n // K, (k + 1) * n // K) for k in range(K)]
    s_in, s_k, s_out = (torch.cuda.Stream(device=local_rank) for _ in range(3))
    codec = R.Codec(local_rank, stream=s_k.cuda_stream)
    streams = [s_in, s_k, s_out]
    pref = np.concatenate([[0], np.cumsum(lens_np)])
    dev = out.device

    def slab(parts):
        """One device slab and its pinned host twin, carved into 256-B aligned
        typed views: parts = [(name, bytes, dtype)]."""
        offs, o = {}, 0
        for name, nb, _ in parts:
            offs[name] = o
            o += (int(nb) + 255) // 256 * 256
        d = torch.empty(max(o, 256), dtype=torch.uint8, device=dev)
        h = torch.empty(max(o, 256), dtype=torch.uint8, pin_memory=True)
        dv, hv = {}, {}
        for name, nb, dt in parts:
            a, b = offs[name], offs[name] + int(nb)
            dv[name] = d[a:b].view(dt)
            hv[name] = h[a:b].view(dt)
        return d[:o], h[:o], dv, hv

    plans = []
    if wl == "c2":
        h_wire, h_len = h_in
    else:
        h_msgs, h_unix, h_auth, h_pay = h_in
        msgs = hb.msgs
        pst = msgs["payload_off"].astype(np.int64)
        pen = pst + msgs["payload_len"].astype(np.int64)
        import onc_rpc_amd.layout as L
        kinds = [(msgs["cred_kind_len"] >> 24) == L.KIND_UNIX, (msgs["verf_kind_len"] >> 24) == L.KIND_UNIX]
        refs = [msgs["cred_ref"].astype(np.int64), msgs["verf_ref"].astype(np.int64)]
    for k, (lo, hi) in enumerate(bounds):
        nk = hi - lo
        wb = int(pref[hi] - pref[lo])
        if wl == "c2":
            w_lo, w_hi = int(pref[lo]), int(pref[hi])
            cp_in = [(out[w_lo:w_hi], h_wire[w_lo:w_hi]), (rec_len[lo:hi], h_len[lo:hi])]
            d, h, dv, hv = slab([("off", 8 * (nk + 1), torch.int64), ("msgs", 64 * nk, torch.uint8),
                                 ("unix", 192 * nk, torch.uint8), ("status", 4 * nk, torch.int32),
                                 ("aux0", 4 * nk, torch.int32), ("aux1", 4 * nk, torch.int32)])

            def kern(c, lo=lo, hi=hi, nk=nk, w_lo=w_lo, dv=dv):
                c.scan_lengths(rec_len[lo:hi], nk, 0, dv["off"])
                c.decode(out[w_lo:], dv["off"], nk, mode, dv["msgs"], dv["unix"], dv["status"], dv["aux0"],
                         dv["aux1"])
        else:
            p_lo, p_hi = int(pst[lo:hi].min()), int(pen[lo:hi].max())
            u = [r[lo:hi][kk[lo:hi]] for r, kk in zip(refs, kinds)]
            u = np.concatenate(u) if len(u[0]) + len(u[1]) else np.zeros(0, np.int64)
            u_lo, u_hi = (int(u.min()), int(u.max()) + 1) if len(u) else (0, 0)
            cp_in = [(db.msgs[64 * lo:64 * hi], h_msgs[64 * lo:64 * hi]),
                     (db.payload_arena[p_lo:p_hi], h_pay[p_lo:p_hi]),
                     (db.unix[96 * u_lo:96 * u_hi], h_unix[96 * u_lo:96 * u_hi])]
            if k == 0:
                cp_in.append((db.auth_arena, h_auth))
            cp_in = [(dd, hh) for dd, hh in cp_in if dd.numel()]
            # decoded AUTH_UNIX slots come back only for chunks with AUTH_UNIX auths
            parts = [("wire", wb, torch.uint8), ("off", 8 * (nk + 1), torch.int64), ("st", 4 * nk, torch.int32),
                     ("msgs", 64 * nk, torch.uint8), ("status", 4 * nk, torch.int32), ("aux0", 4 * nk, torch.int32),
                     ("aux1", 4 * nk, torch.int32)]
            if u_hi > u_lo:
                parts.append(("unix", 192 * nk, torch.uint8))
            d, h, dv, hv = slab(parts)
            unix_out = dv["unix"] if u_hi > u_lo else dec.unix[192 * lo:]
            sub = R.DeviceBatch(nk, db.msgs[64 * lo:], db.unix, db.auth_arena, db.payload_arena)

            def kern(c, sub=sub, nk=nk, wb=wb, dv=dv, unix_out=unix_out):
                c.encode(sub, dv["wire"], dv["off"], dv["st"], out_cap=wb)
                c.decode(dv["wire"], dv["off"], nk, mode, dv["msgs"], unix_out, dv["status"], dv["aux0"],
                         dv["aux1"])
        plans.append((cp_in, kern, (h, d), hv, (lo, hi)))
    bytes_h2d = sum(hh.numel() * hh.element_size() for cp_in, _, _, _, _ in plans for _, hh in cp_in)
    bytes_d2h = sum(p[2][0].numel() for p in plans)

    def run():
        c = codec
        # a new batch starts after the previous one has fully drained
        s_in.wait_stream(s_out)
        s_k.wait_stream(s_out)
        for cp_in, kern, (h, d), _, _ in plans:
            with torch.cuda.stream(s_in):          # H2D; this chunk's kernels wait for it
                for dd, hh in cp_in:
                    dd.copy_(hh, non_blocking=True)
            s_k.wait_stream(s_in)
            with torch.cuda.stream(s_k):
                kern(c)
            s_out.wait_stream(s_k)                 # D2H after this chunk's kernels: one copy
            with torch.cuda.stream(s_out):
                h.copy_(d, non_blocking=True)

    cur = torch.cuda.current_stream(local_rank)
    for s in streams:
        s.wait_stream(cur)
    run()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    reps = args.pcie_reps
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    pms = (time.perf_counter() - t0) * 1e3 / reps
    ok = True
    if wl != "c2":
        ref = out[: total_bytes].cpu()     # the device-resident encode's output
    for _, _, _, hv, (lo, hi) in plans:
        ok = ok and bool((hv["status"] == 0).all())
        if wl != "c2":
            ok = ok and bool((hv["st"] == 0).all())
            # the host wire equals the device-resident encode's output, chunk by chunk
            ok = ok and torch.equal(hv["wire"], ref[int(pref[lo]):int(pref[hi])])
    pt = torch.tensor([pms, 0.0 if ok else 1.0], dtype=torch.float64, device=cdev(out.device))
    if dist is not None:
        dist.all_reduce(pt, op=dist.ReduceOp.MAX)
    pms = float(pt[0])
    codec.close()
    return {"value": n_total / (pms / 1e3) / 1e6, "unit": "Mmsgs/s", "ms_per_step": pms,
            "h2d_bytes_per_gpu": bytes_h2d, "d2h_bytes_per_gpu": bytes_d2h,
            "pcie_GBs_per_gpu": (bytes_h2d + bytes_d2h) / (pms / 1e3) / 1e9, "chunks": K,
            "validated": ok and float(pt[1]) == 0.0,
            "note": "host wall clock; %d record chunks through copy-in / kernel / copy-out streams: H2D, "
                    "kernels and D2H of neighbouring chunks overlap; each chunk's outputs come back as one slab "
                    "copy; decoded AUTH_UNIX slots copied back for chunks with AUTH_UNIX auths" % K}


def _event_ms(torch, fn, reps, sync_streams=()):
    """Average ms of `fn` over `reps` calls after one untimed call, by events
    on the current stream (every stream in sync_streams joined back into it
    before the stop event). Local to the rank: the legs that use it reduce
    their results over ranks afterwards (reduce_leg), outside any try block,
    so a rank that fails a leg cannot leave the others waiting in a
    collective."""
    fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    cur = torch.cuda.current_stream()
    e0.record()
    for s in sync_streams:
        s.wait_stream(cur)
    for _ in range(reps):
        fn()
    for s in sync_streams:
        cur.wait_stream(s)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def _path(d, key):
    for k in key.split(".") if key else []:
        d = d.get(k) if isinstance(d, dict) else None
    return d


def reduce_leg(torch, dist, dev, res, keys, n_total):
    """MAX over ranks of each sub-leg's ms_per_step (keys: dotted paths into
    `res`, "" = res itself), AND of their `validated`; values recomputed
    from the reduced times. Every rank calls it with the same keys, whatever
    its legs did (a missing or failed sub-leg counts as +inf ms, not
    validated)."""
    import math
    vals = []
    for k in keys:
        d = _path(res, k)
        ms = d.get("ms_per_step") if isinstance(d, dict) else None
        ok = bool(d.get("validated")) if isinstance(d, dict) else False
        vals += [ms if (ms is not None and math.isfinite(ms)) else math.inf, 0.0 if ok else 1.0]
    if dist is not None:
        t = torch.tensor(vals, dtype=torch.float64, device=cdev(dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        vals = [float(x) for x in t.cpu()]
    for i, k in enumerate(keys):
        d = _path(res, k)
        if not isinstance(d, dict):
            continue
        ms, bad = vals[2 * i], vals[2 * i + 1]
        d["ms_per_step"] = ms if math.isfinite(ms) else None
        d["value"] = n_total / (ms / 1e3) / 1e6 if math.isfinite(ms) else None
        d["validated"] = bad == 0.0 and math.isfinite(ms)
    return res


def _pick_best(res, names):
    """res.value / ms_per_step / best from the fastest validated sub-leg."""
    cands = [k for k in names if isinstance(res.get(k), dict) and res[k].get("validated")]
    if cands:
        best = max(cands, key=lambda k: res[k]["value"])
        res.update({"value": res[best]["value"], "ms_per_step": res[best]["ms_per_step"], "best": best})
    else:
        res.update({"value": None, "ms_per_step": None, "best": None})
    res["validated"] = all(isinstance(res.get(k), dict) and res[k].get("validated") for k in names)
    return res


class MappedDecodeOut:
    """Decode outputs in mapped host memory: the decode kernel writes them
    there directly (onc_host_register), no copy-back."""

    def __init__(self, R, codec, n):
        m = max(n, 1)
        self.msgs = R.HostMapped(codec, 64 * m)
        self.unix = R.HostMapped(codec, 192 * m)
        self.status = R.HostMapped(codec, 4 * m)
        self.aux0 = R.HostMapped(codec, 4 * m)
        self.aux1 = R.HostMapped(codec, 4 * m)
        self.off = R.HostMapped(codec, 8 * (m + 1))

    def all(self):
        return (self.msgs, self.unix, self.status, self.aux0, self.aux1, self.off)

    def nbytes(self, n, with_unix, with_off=True):
        return n * (64 + 12) + (192 * n if with_unix else 0) + (8 * (n + 1) if with_off else 0)

    def close(self):
        for b in self.all():
            b.close()


def pcie_zero_copy(args, torch, R, wl, hb, codec, out, total_bytes, lens_np, rec_off, dec_off, dec, mode,
                   n_total, has_unix):
    """PCIe-inclusive rate with nothing staged (ABI 7 onc_host_register): the
    bytes stay in mapped host memory and the kernels read and write them in
    place over the link, so only what a kernel touches crosses it.
    c2 (decode): the wire and its lengths sit in the host "socket buffer";
    onc_decode_lengths parses it in place — only the 16-byte granules of the
    headers cross PCIe (call_body.rs:53-59: payloads are sliced, never read)
    — and writes descriptors, statuses, aux words, AUTH_UNIX slots and
    offsets straight into host memory. Loopbacks (c1, c0, c3): descriptors,
    AUTH_UNIX table and arenas read in place by the encode; variant
    `in_place`: the wire written straight into a mapped host send buffer and
    decoded from there; variant `wire_on_device`: the wire in HBM, decoded
    there while a copy stream brings it back (the decode's outputs mapped).
    Validated against the device-resident step's outputs."""
    import numpy as np
    n = hb.n
    reps = max(1, args.pcie_reps)
    dev = out.device
    res = {"unit": "Mmsgs/s", "note": "host-mapped buffers (onc_host_register): kernels read/write host memory "
                                      "in place over PCIe; nothing staged; events on the codec's stream"}
    keep = []
    try:
        o = MappedDecodeOut(R, codec, n)
        keep.append(o)
        ref_msgs = dec.msgs[:64 * n].cpu().numpy()
        ref_off = dec_off[:n + 1].cpu().numpy()

        def check_dec(with_off=True):
            ok = bool((o.status.view(np.int32)[:n] == 0).all())
            ok = ok and np.array_equal(o.msgs.host[:64 * n], ref_msgs)
            if with_off:
                ok = ok and np.array_equal(o.off.view(np.int64)[:n + 1], ref_off)
            return ok
        if wl == "c2":
            w = R.HostMapped(codec, total_bytes + 16)
            keep.append(w)
            w.host[:] = out[:total_bytes + 16].cpu().numpy()           # the socket buffer (untimed)
            rl = R.HostMapped.from_array(codec, lens_np.astype(np.uint32))
            keep.append(rl)

            if args.frame:
                # the raw socket buffer: framed on the device where it lies
                # (onc_frame_stream, rpc_message.rs:343-367), then decoded in place
                fres = torch.zeros(5, dtype=torch.int64, device=dev)

                def step():
                    codec.frame_stream(w, total_bytes, o.off, n, fres)
                    codec.decode(w, o.off, n, mode, o.msgs, o.unix, o.status, o.aux0, o.aux1)
            else:
                def step():
                    codec.decode_lengths(w, rl, n, 0, mode, o.msgs, o.unix, o.status, o.aux0, o.aux1,
                                         rec_off=o.off)
            ms = _event_ms(torch, step, reps)
            ok = check_dec()
            if args.frame:
                ok = ok and [int(x) for x in fres.cpu()[:3]] == [n, total_bytes, 0]
            if not args.frame:
                res["variants"] = c2_zero_copy_variants(args, torch, R, codec, w, rl, o, n, n_total, total_bytes,
                                                        mode, check_dec)
            wire_np = w.host[:total_bytes]
            g_std = decode_granules(wire_np, lens_np)
            g_line = decode_granules(wire_np, lens_np, line=True)
            gr = int(g_std.sum())
            link_ms = (LINK_NS_PER_REC * n + LINK_NS_PER_GRANULE * gr) / 1e6
            link_ms_line = (LINK_NS_PER_REC * n + LINK_NS_PER_GRANULE * int(g_line.sum())) / 1e6
            res.update({"value": n_total / (ms / 1e3) / 1e6, "ms_per_step": ms, "validated": ok,
                        "h2d_bytes_touched_per_gpu": 16 * gr + (0 if args.frame else 4 * n),
                        "h2d_granules": {"standard": gr, "line": int(g_line.sum()),
                                         "mean_per_record_standard": gr / max(n, 1)},
                        "link_model_ms": {"standard": link_ms, "line": link_ms_line},
                        "d2h_bytes_per_gpu": o.nbytes(n, has_unix),
                        "h2d_note": "16 B x the wire granules the decode's window rounds request under the "
                                    "standard policy (bench.decode_granules, counted on this wire)" +
                                    (" + the framer's sweep and chase reads" if args.frame else
                                     " + 4 B of length per record") + f"; the wire is {total_bytes} bytes. "
                                    "link_model_ms: the link_lab fit (2.82 ns per record + 0.41 ns per "
                                    "granule, profiles/r06_link_lab.log) for those requests",
                        "step": ("onc_frame_stream + onc_decode of the mapped socket buffer" if args.frame else
                                 "onc_decode_lengths of the mapped socket buffer from its mapped lengths")})
            return res
        # loopbacks
        mb = R.MappedHostBatch(codec, hb)
        keep.append(mb)
        in_bytes = hb.msgs.nbytes + (hb.unix.nbytes if has_unix else 0) + hb.payload_arena.nbytes
        # (a) in place: wire into a mapped send buffer, decoded from there
        wh = R.HostMapped(codec, total_bytes + 16)
        keep.append(wh)
        roh = R.HostMapped(codec, 8 * (n + 1))
        sth = R.HostMapped(codec, 4 * max(n, 1))
        keep += [roh, sth]

        def step_a():
            codec.encode(mb, wh, roh, sth, out_cap=total_bytes)
            codec.decode(wh, roh, n, mode, o.msgs, o.unix, o.status, o.aux0, o.aux1)
        ms_a = _event_ms(torch, step_a, reps)
        ok_a = check_dec(with_off=False) and bool((sth.view(np.int32)[:n] == 0).all())
        ok_a = ok_a and np.array_equal(roh.view(np.int64)[:n + 1], ref_off)
        ref_wire = out[:total_bytes].cpu().numpy()
        ok_a = ok_a and np.array_equal(wh.host[:total_bytes], ref_wire)
        # (b) wire in HBM, decoded there while a copy stream brings it home
        cs = torch.cuda.Stream(device=dev)
        h_wire = torch.empty(total_bytes, dtype=torch.uint8, pin_memory=True)
        h_off = torch.empty(n + 1, dtype=torch.int64, pin_memory=True)
        st = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        h_st = torch.empty(max(n, 1), dtype=torch.int32, pin_memory=True)
        cur = torch.cuda.current_stream(dev)

        def step_b():
            cur.wait_stream(cs)                     # the previous step's copy has read `out`
            codec.encode(mb, out, rec_off, st)
            cs.wait_stream(cur)
            with torch.cuda.stream(cs):
                h_wire.copy_(out[:total_bytes], non_blocking=True)
                h_off.copy_(rec_off[:n + 1], non_blocking=True)
                h_st.copy_(st, non_blocking=True)
            codec.decode(out, rec_off, n, mode, o.msgs, o.unix, o.status, o.aux0, o.aux1)
        ms_b = _event_ms(torch, step_b, reps, sync_streams=(cs,))
        torch.cuda.synchronize()
        ok_b = check_dec(with_off=False) and bool((h_st[:n] == 0).all())
        ok_b = ok_b and np.array_equal(h_off.numpy(), ref_off) and np.array_equal(h_wire.numpy(), ref_wire)
        d2h = total_bytes + 8 * (n + 1) + 4 * n + o.nbytes(n, has_unix, with_off=False)
        var = {"in_place": {"value": n_total / (ms_a / 1e3) / 1e6, "ms_per_step": ms_a, "validated": ok_a,
                            "h2d_bytes_per_gpu": in_bytes, "d2h_bytes_per_gpu": d2h,
                            "note": "encode reads descriptors + arenas in place and writes the wire into the "
                                    "mapped send buffer; the decode parses that host wire in place (its header "
                                    "lines cross the link again)"},
               "wire_on_device": {"value": n_total / (ms_b / 1e3) / 1e6, "ms_per_step": ms_b, "validated": ok_b,
                                  "h2d_bytes_per_gpu": in_bytes, "d2h_bytes_per_gpu": d2h,
                                  "note": "encode reads descriptors + arenas in place into an HBM wire; the wire, "
                                          "offsets and statuses come back on a copy stream while the decode "
                                          "writes its outputs into mapped host memory"}}
        res["variants"] = var                         # best picked after the reduction over ranks
        return res
    except Exception as e:                            # report, do not lose the line
        res.update({"value": None, "validated": False, "error": repr(e)})
        return res
    finally:
        torch.cuda.synchronize()
        for k in keep:
            k.close()


def c2_zero_copy_variants(args, torch, R, codec, w, rl, o, n, n_total, total_bytes, mode, check_dec):
    """What else a server pays or picks on the c2 zero-copy decode
    (VERDICT r05 item 3):
    register_per_batch — the socket buffer NOT registered beforehand: every
      step pins it (onc_host_register of the 1.9 GB wire and of its lengths),
      decodes it in place, synchronises and unpins it; host wall clock (the
      registration is synchronous host work). The data is written into the
      buffer before the timed calls (the pages are resident, as after a recv).
      A fresh buffer pair per batch (register_per_batch) and the same pair
      every batch (register_per_batch_recycled) are timed apart: the runtime
      re-pins a range it has pinned before far faster.
    policy_standard / policy_line / policy_auto — the same registered-once
      decode under each first-round policy pinned (onc_codec_set_decode_policy):
      STANDARD fetches each record's first 44 bytes (a 64-byte span), LINE the
      rest of its first 128-byte line; over PCIe every fetched granule crosses
      the link."""
    import ctypes as C
    import mmap
    import time
    import numpy as np
    out = {}
    reps = max(1, args.pcie_reps)
    for name, pol in (("policy_standard", R.DECODE_POLICY_STANDARD), ("policy_line", R.DECODE_POLICY_LINE),
                      ("policy_auto", R.DECODE_POLICY_AUTO)):
        codec.set_decode_policy(pol)

        def step():
            codec.decode_lengths(w, rl, n, 0, mode, o.msgs, o.unix, o.status, o.aux0, o.aux1, rec_off=o.off)
        ms = _event_ms(torch, step, reps)
        out[name] = {"value": n_total / (ms / 1e3) / 1e6, "ms_per_step": ms, "validated": check_dec()}
    codec.set_decode_policy(R.DECODE_POLICY_AUTO)
    # register per batch: plain (unpinned) buffers holding the same bytes,
    # a fresh pair every step (never registered before: a server receiving
    # into new memory), filled outside the timed calls; each call timed on
    # the host clock
    lib = codec.lib

    class _Dev:
        def __init__(self, p):
            self.p = p

        def data_ptr(self):
            return self.p

    def make_pair():
        # {"mm": mmaps, "a": numpy views, "p": their addresses}; close()
        # drops the views before unmapping (an exported buffer cannot close)
        mm = (mmap.mmap(-1, total_bytes + 16 + 4096), mmap.mmap(-1, 4 * n + 4096))
        hb_w = np.frombuffer(mm[0], np.uint8, count=total_bytes + 16)
        hb_w[:] = w.host[:total_bytes + 16]
        hb_l = np.frombuffer(mm[1], np.uint8, count=4 * n)
        hb_l[:] = rl.host[:4 * n]
        return {"mm": mm, "a": [hb_w, hb_l], "p": (hb_w.ctypes.data, hb_l.ctypes.data)}

    def one(pair):
        aw, al = pair["p"]
        dw, dl = C.c_void_p(), C.c_void_p()
        t0 = time.perf_counter()
        codec._check(lib.onc_host_register(codec.h, C.c_void_p(aw), total_bytes + 16, C.byref(dw)), "register")
        codec._check(lib.onc_host_register(codec.h, C.c_void_p(al), 4 * n, C.byref(dl)), "register")
        t1 = time.perf_counter()
        codec.decode_lengths(_Dev(dw.value), _Dev(dl.value), n, 0, mode, o.msgs, o.unix, o.status, o.aux0,
                             o.aux1, rec_off=o.off)
        codec.sync()
        t2 = time.perf_counter()
        codec._check(lib.onc_host_unregister(codec.h, C.c_void_p(aw)), "unregister")
        codec._check(lib.onc_host_unregister(codec.h, C.c_void_p(al)), "unregister")
        t3 = time.perf_counter()
        return (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3

    def close(pair):
        pair["a"].clear()
        for m in pair["mm"]:
            m.close()

    def leg(parts, r, note):
        reg, dec, unreg = (float(x) for x in np.array(parts).mean(axis=0))
        ms = reg + dec + unreg
        return {"value": n_total / (ms / 1e3) / 1e6, "ms_per_step": ms, "validated": check_dec(),
                "register_ms": reg, "decode_sync_ms": dec, "unregister_ms": unreg, "batches": r, "note": note}
    r = max(2, min(reps, 4))
    # fresh: a new buffer pair per batch (never registered before)
    parts = []
    for k in range(r + 1):
        pair = make_pair()
        try:
            t = one(pair)
        finally:
            close(pair)
        if k:
            parts.append(t)
    out["register_per_batch"] = leg(parts, r,
        f"a fresh unpinned buffer pair per batch (pages already written, as after a recv): onc_host_register of "
        f"the {total_bytes}-byte wire + its lengths, the in-place decode and a synchronisation, "
        "onc_host_unregister (host wall clock of each call, mean over batches)")
    # recycled: the same buffer pair registered and unregistered every batch
    # (a server recycling its receive buffers without keeping them pinned)
    pair = make_pair()
    try:
        one(pair)
        parts = [one(pair) for _ in range(r)]
    finally:
        close(pair)
    out["register_per_batch_recycled"] = leg(parts, r,
        "the same unpinned buffer pair registered, decoded in place and unregistered every batch "
        "(host wall clock of each call, mean over batches)")
    return out


def iov_gather_ok(hdr, e, payload, ref_wire, wire_base=0, step=1 << 16):
    """The bytes a writev of every record's two iovecs sends — its header
    slice of `hdr`, then its payload slice of the host payload arena —
    equal `ref_wire` (numpy, host), and the iovecs tile [wire_base,
    wire_base + len(ref_wire)) contiguously. e: IOV_DTYPE records."""
    import numpy as np
    n = len(e)
    hl = e["hdr_len"].astype(np.int64)
    pl = e["payload_len"].astype(np.int64)
    ho = e["hdr_off"].astype(np.int64)
    po = e["payload_off"].astype(np.int64)
    wo = e["wire_off"].astype(np.int64) - wire_base
    if n == 0:
        return len(ref_wire) == 0
    if not np.array_equal(wo[1:], wo[:-1] + hl[:-1] + pl[:-1]) or wo[0] != 0 or wo[-1] + hl[-1] + pl[-1] != len(ref_wire):
        return False
    for a in range(0, n, step):
        b = min(n, a + step)
        w0, w1 = int(wo[a]), int(wo[b - 1] + hl[b - 1] + pl[b - 1])
        buf = np.empty(w1 - w0, np.uint8)
        for ln, src_off, dst_off, src in ((hl[a:b], ho[a:b], wo[a:b] - w0, hdr),
                                          (pl[a:b], po[a:b], wo[a:b] - w0 + hl[a:b], payload)):
            tot = int(ln.sum())
            if tot == 0:
                continue
            within = np.arange(tot, dtype=np.int64) - np.repeat(np.cumsum(ln) - ln, ln)
            buf[np.repeat(dst_off, ln) + within] = src[np.repeat(src_off, ln) + within]
        if not np.array_equal(buf, ref_wire[w0:w1]):
            return False
    return True


def pcie_iov(args, torch, R, L, hb, db, codec, n_total, hdr_total, total_bytes, out):
    """PCIe-inclusive legs of the vectored encode (onc_encode_iov): the
    payloads never cross the link (README.md:71-75, rpc_message.rs:19 — the
    sender's writev gathers them from where they lie); the payload arena
    stays in host memory (mapped: the kernels only bound-check descriptors
    against its size). In: descriptors (+ the AUTH_UNIX table and auth arena
    when used); out: packed headers, 32-byte iovecs, statuses.
    serialised: H2D, kernels, D2H on one stream; pipelined: --pcie-chunks
    record chunks through copy-in / kernel / copy-out streams; zero_copy:
    descriptors read and outputs written in place in mapped host memory.
    Each validated on the host: the wire a writev of the iovecs would send
    (header slices + host payload slices) equals the device-resident
    contiguous encode's bytes."""
    import numpy as np
    n = hb.n
    dev = out.device
    reps = max(1, args.pcie_reps)
    kinds = np.concatenate([hb.msgs["cred_kind_len"] >> 24, hb.msgs["verf_kind_len"] >> 24])
    has_unix = bool((kinds == L.KIND_UNIX).any())
    ref_wire = out[:total_bytes].cpu().numpy()
    pay = np.ascontiguousarray(hb.payload_arena)
    keep = []
    res = {"unit": "Mmsgs/s", "note": "payloads never cross PCIe: they stay in host memory and the iovecs point "
                                      "at them; validated by gathering the wire on the host from the iovecs"}
    try:
        pay_h = R.HostMapped.from_array(codec, pay if pay.size else np.zeros(16, np.uint8))
        keep.append(pay_h)
        in_parts = [(db.msgs, torch.from_numpy(hb.msgs.view(np.uint8).reshape(-1).copy()).pin_memory())]
        if has_unix:
            in_parts.append((db.unix, torch.from_numpy(hb.unix.view(np.uint8).reshape(-1).copy()).pin_memory()))
        if hb.auth_arena.size:
            in_parts.append((db.auth_arena[:hb.auth_arena.size],
                             torch.from_numpy(hb.auth_arena.copy()).pin_memory()))
        h2d = sum(h.numel() for _, h in in_parts)
        sb = R.DeviceBatch(n, db.msgs, db.unix, db.auth_arena, pay_h, payload_len=pay.size)
        hdr_d = torch.zeros(hdr_total + 16, dtype=torch.uint8, device=dev)
        iov_d = torch.zeros(32 * max(n, 1), dtype=torch.uint8, device=dev)
        st_d = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)
        hdr_h = torch.empty(hdr_total, dtype=torch.uint8, pin_memory=True)
        iov_h = torch.empty(32 * n, dtype=torch.uint8, pin_memory=True)
        st_h = torch.empty(n, dtype=torch.int32, pin_memory=True)
        d2h = hdr_total + 36 * n

        def ser():
            for d, h in in_parts:
                d.copy_(h, non_blocking=True)
            codec.encode_iov(sb, hdr_d, iov_d, st_d, None, hdr_total)
            hdr_h.copy_(hdr_d[:hdr_total], non_blocking=True)
            iov_h.copy_(iov_d[:32 * n], non_blocking=True)
            st_h.copy_(st_d[:n], non_blocking=True)
        ms = _event_ms(torch, ser, reps)
        ok = bool((st_h == 0).all()) and iov_gather_ok(hdr_h.numpy(), iov_h.numpy().view(L.IOV_DTYPE), pay, ref_wire)
        res["serialised"] = {"value": n_total / (ms / 1e3) / 1e6, "ms_per_step": ms, "validated": ok,
                             "h2d_bytes_per_gpu": h2d, "d2h_bytes_per_gpu": d2h,
                             "pcie_GBs_per_gpu": (h2d + d2h) / (ms / 1e3) / 1e9}
        # pipelined: record chunks, each its own sub-batch, slab and codec call
        K = max(1, min(args.pcie_chunks, n))
        bounds = [(k * n // K, (k + 1) * n // K) for k in range(K)]
        s_in, s_k, s_out = (torch.cuda.Stream(device=dev) for _ in range(3))
        pc = R.Codec(dev.index if dev.index is not None else 0, stream=s_k.cuda_stream)
        keep.append(pc)
        pc.reserve(n)
        hdr_len = np.zeros(n, np.int64)
        # per-record header bytes from the main run's iovecs (the plan a chunk's slab is sized by)
        plans = []
        msgs_h = in_parts[0][1]
        e_ref = iov_h.numpy().view(L.IOV_DTYPE)
        hdr_len[:] = e_ref["hdr_len"]
        hpre = np.concatenate([[0], np.cumsum(hdr_len)])
        for k, (lo, hi) in enumerate(bounds):
            nk = hi - lo
            hb_k = int(hpre[hi] - hpre[lo])
            cp = [(db.msgs[64 * lo:64 * hi], msgs_h[64 * lo:64 * hi])]
            if k == 0:
                cp += in_parts[1:]
            o_hdr = (hb_k + 255) // 256 * 256
            o_iov = o_hdr + (32 * nk + 255) // 256 * 256
            slab = torch.empty(o_iov + 4 * nk + 16, dtype=torch.uint8, device=dev)
            slab_h = torch.empty(slab.numel(), dtype=torch.uint8, pin_memory=True)
            sub = R.DeviceBatch(nk, db.msgs[64 * lo:], db.unix, db.auth_arena, pay_h, payload_len=pay.size)
            plans.append((cp, sub, slab, slab_h, hb_k, o_hdr, o_iov, nk, lo))

        def pipe():
            s_in.wait_stream(s_out)
            s_k.wait_stream(s_out)
            for cp, sub, slab, slab_h, hb_k, o_hdr, o_iov, nk, lo in plans:
                with torch.cuda.stream(s_in):
                    for d, h in cp:
                        d.copy_(h, non_blocking=True)
                s_k.wait_stream(s_in)
                pc.encode_iov(sub, slab[:max(hb_k, 16)], slab[o_hdr:], slab[o_iov:].view(torch.int32), None, hb_k)
                s_out.wait_stream(s_k)
                with torch.cuda.stream(s_out):
                    slab_h.copy_(slab, non_blocking=True)
        ms_p = _event_ms(torch, pipe, reps, sync_streams=(s_in, s_k, s_out))
        okp = True
        for cp, sub, slab, slab_h, hb_k, o_hdr, o_iov, nk, lo in plans:
            sh = slab_h.numpy()
            e = sh[o_hdr:o_hdr + 32 * nk].view(L.IOV_DTYPE)
            w0 = int(np.int64(e_ref["wire_off"][lo])) if nk else 0
            okp = okp and bool((sh[o_iov:o_iov + 4 * nk].view(np.int32) == 0).all())
            w1 = w0 + int((e["hdr_len"].astype(np.int64) + e["payload_len"]).sum())
            okp = okp and iov_gather_ok(sh[:hb_k], e, pay, ref_wire[w0:w1])
        okp = okp and w1 == total_bytes
        res["pipelined"] = {"value": n_total / (ms_p / 1e3) / 1e6, "ms_per_step": ms_p, "validated": okp,
                            "chunks": K, "h2d_bytes_per_gpu": h2d, "d2h_bytes_per_gpu": d2h,
                            "note": "events on the copy-in / kernel / copy-out streams joined into one"}
        # zero copy: descriptors read and outputs written in mapped host memory
        mb = R.MappedHostBatch(codec, hb)
        keep.append(mb)
        hdr_m = R.HostMapped(codec, hdr_total + 16)
        iov_m = R.HostMapped(codec, 32 * max(n, 1))
        st_m = R.HostMapped(codec, 4 * max(n, 1))
        keep += [hdr_m, iov_m, st_m]

        def zc():
            codec.encode_iov(mb, hdr_m, iov_m, st_m, None, hdr_total)
        ms_z = _event_ms(torch, zc, reps)
        okz = bool((st_m.view(np.int32)[:n] == 0).all()) and iov_gather_ok(
            hdr_m.host[:hdr_total], iov_m.view(L.IOV_DTYPE)[:n], pay, ref_wire)
        res["zero_copy"] = {"value": n_total / (ms_z / 1e3) / 1e6, "ms_per_step": ms_z, "validated": okz,
                            "h2d_bytes_per_gpu": h2d, "d2h_bytes_per_gpu": d2h,
                            "note": "onc_host_register: iov_len / iov_emit read the descriptors and write the "
                                    "headers, iovecs and statuses in host memory in place"}
        return res                                    # best picked after the reduction over ranks
    except Exception as e:
        res.update({"value": None, "validated": False, "error": repr(e)})
        return res
    finally:
        torch.cuda.synchronize()
        for k in keep:
            k.close()


# link_lab (tools/link_lab.hip, profiles/r06_link_lab.log): one lane's
# scattered read of g consecutive 16-byte granules of mapped host memory,
# 1M lanes, records 1936 bytes apart: 3.23 / 3.60 / 4.01 / 4.40 / 6.01 /
# 9.32 ms for g = 1 / 2 / 3 / 4 / 8 / 16 -> a least-squares line of
# ~2.82 ns per record plus ~0.41 ns per granule (the link moves requests,
# not lines: 64 B cost 1.36x of 16 B, 128 B 1.86x)
LINK_NS_PER_REC = 2.82
LINK_NS_PER_GRANULE = 0.406


def decode_granules(wire, lens_np, line=False):
    """16-byte granules of the wire that the decode's window rounds request,
    per record (decode.hip stage_window, the standard policy or, `line`,
    the line policy): round 1 min(r44, avail) (line: up to the record's
    first 128-byte line and 128 bytes, at most 8), then round 2 up to the
    header extent read from round 1 (call: 36 + cred body + verifier;
    reply: 24 + verifier + 12). `wire` is the packed wire from offset 0 (a
    16-byte aligned buffer); returns an int64 array of granules per record."""
    import numpy as np
    L = lens_np.astype(np.int64)
    n = L.size
    start = np.zeros(n, np.int64)
    if n > 1:
        start[1:] = np.cumsum(L)[:-1]
    q0 = start & 15
    W = 10                                                   # ONC_DEC_WIN
    avail = np.minimum(W, (q0 + L + 15) >> 4)
    r44 = np.minimum(4, (q0 + np.minimum(L, 44) + 15) >> 4)
    if line:
        win = start - q0
        rln = (((win | 127) + 1) - win) >> 4
        r128 = (q0 + np.minimum(L, 128) + 15) >> 4
        nch = np.minimum(np.minimum(8, np.maximum(np.maximum(r44, rln), r128)), avail)
    else:
        nch = np.minimum(r44, avail)
    buf = np.frombuffer(bytes(wire), np.uint8) if not isinstance(wire, np.ndarray) else wire.view(np.uint8)
    top = buf.size - 4

    def be32(off):
        o = np.clip(off, 0, top)
        b = buf[o[:, None] + np.arange(4)].astype(np.int64)
        return (b[:, 0] << 24) | (b[:, 1] << 16) | (b[:, 2] << 8) | b[:, 3]

    def pad4(x):
        return (4 - (x & 3)) & 3
    need = np.minimum(L, 16 * W)
    head = (L >= 36) & (16 * nch >= q0 + 36)
    mt = be32(start + 8)
    call = head & (mt == 0)
    reply = head & (mt == 1)
    cl = be32(start + 32)
    vpos = 36 + cl + pad4(cl) + 4
    vin = (q0 + vpos + 4 <= 16 * nch) & (vpos + 4 <= L)
    vl = be32(start + np.where(vin, vpos, 0))
    need_call = np.where(cl > 200, 36,
                         np.where(vin, vpos + 4 + np.where(vl <= 200, vl + pad4(vl), 0), vpos + 4 + 16))
    rv = be32(start + 20)
    need_reply = np.where(rv <= 200, 24 + rv + pad4(rv) + 12, 24)
    need = np.where(call, need_call, np.where(reply, need_reply, need))
    want = np.minimum(avail, (q0 + need + 15) >> 4)
    g = np.maximum(nch, want)
    return np.where(L > 0, g, 0)


# ---------------------------------------------------------------------------
# timing + roofline (shared by every workload)
# ---------------------------------------------------------------------------
BACKEND = ["nccl"]


def cdev(dev):
    """Device of the control-plane collective tensors: the GPU under RCCL
    (`nccl`), the host under gloo."""
    return dev if BACKEND[0] == "nccl" else "cpu"


ALG_CTX = {"unix_refs": 0}     # AUTH_UNIX auths of the batch (iov_emit's parameter-block reads)

ALG_PER_LAUNCH = {
    # algorithmic bytes per launch: encode reads ~W and writes
    # W; zero-copy decode reads H + 4 (the length) and writes ~H.
    "enc_len_kernel": lambda n, W, H: n * (64 + 4),          # descriptor read + status write
    "scan_tiles_kernel": lambda n, W, H: 0,
    "enc_emit_kernel": lambda n, W, H: 2 * W,
    "decode_kernel": lambda n, W, H: 2 * H + 4 * n,
    "len_tiles_kernel": lambda n, W, H: 4 * n,
    "len_apply_kernel": lambda n, W, H: 12 * n,
    # vectored encode (H here = the packed header bytes): descriptors read by
    # both kernels, status written by iov_len; iov_emit reads the wire-carried
    # data once (descriptor + the 96-byte parameter block of every AUTH_UNIX
    # auth) and writes the headers + 32-byte iovecs
    "iov_len_kernel": lambda n, W, H: n * (64 + 4),
    "iov_emit_kernel": lambda n, W, H: n * (64 + 32) + H + 96 * ALG_CTX["unix_refs"],
    "frame_chunks_kernel": lambda n, W, H: 0,
    "frame_write_kernel": lambda n, W, H: 8 * n,
    "frame_walk_kernel": lambda n, W, H: 0,
    "frame_counts_kernel": lambda n, W, H: 0,
    "frame_guess_kernel": lambda n, W, H: 0,
}


class Timing:
    """W warmup steps; a breakdown pass with every launch timed by HIP events
    (to find the dominant kernel); the timed region: exactly K steps
    bracketed by barrier + synchronize on both sides, the dominant kernel's
    launches of every K//5-th step timed by HIP events on the codec's stream
    (hipExtLaunchKernelGGL start/stop events: the dispatch's own timestamps);
    and an event-free pass of the same K steps."""

    def __init__(self, torch, R, codec, step, steps, warmup, barrier, codecs=None, drain=None):
        codecs = codecs or [codec]
        drain = drain or (lambda: None)

        def stats():
            tot = {}
            for c in codecs:
                for k, (ms, cnt) in c.kernel_stats().items():
                    a, b = tot.get(k, (0.0, 0))
                    tot[k] = (a + ms, b + cnt)
            return tot

        def timing(on, kernels=None):
            for c in codecs:
                c.enable_timing(on, kernels=kernels)

        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        for c in codecs:
            c.reset_stats()
        timing(True)
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        timing(False)
        self.breakdown = stats()
        # launches of each kernel per step (a chunked encode launches
        # enc_len / enc_emit once per 1M-record chunk); the dominant kernel
        # is the one with the most time per step
        self.per_step = {k: cnt / steps for k, (_, cnt) in self.breakdown.items()}
        self.dom_id = max(range(R.K_COUNT), key=lambda k: self.breakdown[R.K_NAMES[k]][0])
        for c in codecs:
            c.reset_stats()
        timing(True, kernels=[self.dom_id])
        barrier()
        torch.cuda.synchronize()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        # The dominant kernel is timed on every `stride`-th step (>= 5 launches):
        # a timed launch still costs the step ~6 us of dispatch serialisation
        # (the profiling completion signal), which is not the kernel's work.
        self.stride = max(1, steps // 5)
        if os.environ.get("ONC_BENCH_TIMED_STRIDE"):      # lab: how the timed-launch stride perturbs the step
            self.stride = max(1, int(os.environ["ONC_BENCH_TIMED_STRIDE"]))
        t_wall0 = time.perf_counter()
        ev0.record()
        for i in range(steps):
            if self.stride > 1:
                timing(i % self.stride == 0, kernels=[self.dom_id])
            step()
        drain()
        ev1.record()
        torch.cuda.synchronize()
        barrier()
        self.wall_s = time.perf_counter() - t_wall0
        timing(False)
        self.ms = ev0.elapsed_time(ev1)
        self.kstats = stats()
        torch.cuda.synchronize()
        ev2 = torch.cuda.Event(enable_timing=True)
        ev3 = torch.cuda.Event(enable_timing=True)
        ev2.record()
        for _ in range(steps):
            step()
        drain()
        ev3.record()
        torch.cuda.synchronize()
        self.ms_clean = ev2.elapsed_time(ev3)
        self.dom = R.K_NAMES[self.dom_id]
        self.steps_n = steps


MALL_BYTES = 256 * 2**20       # MI355X Infinity Cache (MI355X_MICROARCH.md chip table)


def cold_copies(buf, touched_per_step):
    """`buf` and identical clones of it, enough that a step rotating through
    them reads lines last touched >= 2x the Infinity Cache of other steps'
    reads ago (touched_per_step: bytes of lines one step reads; at least 3
    copies)."""
    k = 1 + max(2, -(-2 * MALL_BYTES // max(1, touched_per_step)))
    return [buf] + [buf.clone() for _ in range(k - 1)]


def rotating(copies):
    """A callable returning the next of `copies` on every call."""
    it = [0]

    def nxt():
        b = copies[it[0] % len(copies)]
        it[0] += 1
        return b
    return nxt


def dom_summary(tm, n, sum_W, sum_H, ms_per_step):
    dom_ms, dom_cnt = tm.kstats[tm.dom]
    us = dom_ms / dom_cnt * 1e3
    alg = ALG_PER_LAUNCH[tm.dom](n, sum_W, sum_H) / max(1, round(tm.per_step.get(tm.dom, 1)))
    return {"Mmsgs_per_s": n / (ms_per_step / 1e3) / 1e6, "ms_per_step": ms_per_step,
            "ms_per_step_without_kernel_events": tm.ms_clean / tm.steps_n,
            "kernel": tm.dom, "avg_launch_us": us, "achieved_GBs": alg / (us * 1e-6) / 1e9,
            "frac": alg / (us * 1e-6) / 1e9 / HBM_PEAK_GBS}


def load_traffic(path, wl, n, dom):
    """HBM bytes per launch of `dom` from the newest PMC traffic file for this
    workload and batch size (profiles/traffic_rNN[_wl].json), else None."""
    import glob
    if path:
        cands = [path]
    else:
        suffix = "" if wl == "c1" else f"_{wl}"
        cands = sorted(glob.glob(os.path.join(ROOT, "profiles", f"traffic_r[0-9][0-9]{suffix}.json")), reverse=True)
    for p in cands:
        try:
            with open(p) as f:
                tj = json.load(f)
        except (OSError, ValueError):
            continue
        if tj.get("records") == n and tj.get("workload_id", "c1") == wl and dom in tj.get("kernels", {}):
            return tj["kernels"][dom]["hbm_bytes_per_launch"], os.path.relpath(p, ROOT)
    return None, None


def roofline(tm, n, sum_W, sum_H, step_alg, ms_per_step, traffic, traffic_src):
    dom_ms, dom_cnt = tm.kstats[tm.dom]
    dom_us = dom_ms / dom_cnt * 1e3
    per_step = max(1, round(tm.per_step.get(tm.dom, 1)))
    alg = ALG_PER_LAUNCH[tm.dom](n, sum_W, sum_H) / per_step
    achieved = alg / (dom_us * 1e-6) / 1e9
    step_gbs = step_alg / (ms_per_step / 1e3) / 1e9
    return {"bound": "hbm", "kernel": tm.dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
            "alg_bytes_per_launch": alg, "avg_launch_us": dom_us, "launches_timed": dom_cnt,
            "launches_per_step": per_step,
            "timed_every_nth_step": tm.stride,
            **({"kernel_note": "ONC_K_ENC_EMIT launch: the wave-specialised enc_emit_ws_kernel for batches "
                               "(or 1M-record chunks of larger batches) with >= 128 B mean payload, else "
                               "enc_emit_kernel_t (codec.hip enc_args)"} if tm.dom == "enc_emit_kernel" else {}),
            # the whole step (every kernel of the metric), per GPU
            "step_alg_bytes": step_alg, "step_achieved": step_gbs, "step_frac": step_gbs / HBM_PEAK_GBS}


def breakdown_dict(tm, n, sum_W, sum_H):
    kern = {}
    for name, (tot_ms, cnt) in tm.breakdown.items():
        if cnt:
            per_step = max(1, round(tm.per_step.get(name, 1)))
            kern[name] = {"avg_us": tot_ms / cnt * 1e3, "launches": cnt, "launches_per_step": per_step,
                          "alg_bytes_per_launch": ALG_PER_LAUNCH[name](n, sum_W, sum_H) / per_step}
    return kern


def gather_per_gpu(torch, dist, dev, rank, n, ms_per_step, ms_clean_per_step):
    """[records, ms/step, event-free ms/step] of every rank (control plane)."""
    t = torch.tensor([float(n), ms_per_step, ms_clean_per_step], dtype=torch.float64, device=cdev(dev))
    if dist is None:
        rows = [t]
    else:
        rows = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(rows, t)
    out = []
    for r, row in enumerate(rows):
        nr, ms, msc = (float(x) for x in row.cpu())
        out.append({"rank": r, "records": int(nr), "ms_per_step": ms, "Mmsgs_per_s": nr / (ms / 1e3) / 1e6,
                    "ms_per_step_without_kernel_events": msc})
    return out


def agree(torch, dist, dev, ok):
    """Every rank's flag, AND-ed (one collective all ranks always reach)."""
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=cdev(dev))
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


# ---------------------------------------------------------------------------
# configs[4]: 64M records in total, sharded over the ranks (strong scaling)
# ---------------------------------------------------------------------------
def run_c4(args, torch, R, S, SH, L, dist, rank, world, local_rank, total, mode, steps, warmup):
    dev = torch.device("cuda", local_rank)
    lo, hi = SH.shard_bounds(total, world, rank)
    n = hi - lo
    err = None
    try:
        db, gseed = S.call_none_device(lo, hi, 256, seed=4, device=dev)
        codec = R.Codec(local_rank)
        codec.reserve(n)
        local_bytes = n * C4_W
        out = torch.empty(local_bytes + 16, dtype=torch.uint8, device=dev)
        rec_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        enc_status = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        dec = R.DecodeBuffers(n, dev)
        torch.cuda.synchronize()
    except Exception as e:          # e.g. out of memory: every rank learns it below
        err = repr(e)
    if not agree(torch, dist, dev, err is None):
        return {"error": err or "another rank failed to allocate"}

    def step():
        codec.encode(db, out, rec_off, enc_status)
        codec.decode(out, rec_off, n, mode, dec.msgs, dec.unix, dec.status, dec.aux0, dec.aux1)

    def barrier():
        if dist is not None:
            dist.barrier()

    tm = Timing(torch, R, codec, step, steps, warmup, barrier)
    t = torch.tensor([tm.ms, tm.ms_clean], dtype=torch.float64, device=cdev(dev))
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms_max, ms_clean_max = float(t[0]), float(t[1])

    # validation of the last step (device side) + global placement of the shard
    ok = int((enc_status[:n] != 0).sum()) == 0 and int((dec.status[:n] != 0).sum()) == 0
    enc_total = int(rec_off[n]) if n else 0
    ok = ok and enc_total == local_bytes
    ok = ok and c4_wire_bytes_ok(torch, out, db, lo, n)
    xid = dec.msgs.view(-1, 64)[:n, 0:4].contiguous().view(torch.int32).view(-1)
    want = (torch.arange(lo, hi, dtype=torch.int64, device=dev) & 0xFFFFFFFF).to(torch.int32)
    ok = ok and torch.equal(xid, want)
    totals = SH.allgather_totals(enc_total) if dist is not None else [enc_total]
    bases, grand = SH.exclusive_bases(totals)
    ok = ok and grand == total * C4_W
    ok = agree(torch, dist, dev, ok)

    per_gpu = gather_per_gpu(torch, dist, dev, rank, n, tm.ms / steps, tm.ms_clean / steps)
    for r, row in enumerate(per_gpu):
        row["global_base"] = int(bases[r])
        row["shard"] = list(SH.shard_bounds(total, world, r))
    ms_per_step = ms_max / steps
    sum_W, sum_H = local_bytes, n * C4_H
    step_alg = 2 * sum_W + 2 * sum_H + 4 * n
    traffic, tsrc = load_traffic(None, "c4", n, tm.dom)
    res = {
        "metric": METRIC, "value": total / (ms_per_step / 1e3) / 1e6, "unit": "Mmsgs/s", "n_gpus": world,
        "steps": steps, "warmup": warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
        "scaling": "strong", "dtype": "u8",
        "data": f"synthetic (device RNG, seed {gseed} on rank {rank}): configs[4] records = configs[1]'s "
                "Call(AuthNone(None) x2) + 256 B",
        "config": {"workload": f"configs[4]: {total} x 300 B records in total, {n} on rank {rank} "
                               f"(contiguous shards, {args.mode} mode), encode -> decode, HBM-resident",
                   "records_total": total, "records_per_gpu": n, "wire_bytes_total": grand,
                   "parallelism": f"record-sharded x{world} (no collective on the data path)"},
        "per_gpu": per_gpu,
        "ms_per_step_without_kernel_events": ms_clean_max / steps,
        "roofline": roofline(tm, n, sum_W, sum_H, step_alg, ms_per_step, traffic, tsrc),
        "kernels_breakdown_pass": breakdown_dict(tm, n, sum_W, sum_H),
        "global_send_buffer": {"shard_bytes": totals, "bases": [int(b) for b in bases], "total": grand,
                               "note": "exclusive scan of one all_gather'ed int64 per rank "
                                       "(shard.allgather_totals + exclusive_bases)"},
        "validated": ok,
        "wall_s_timed_region": tm.wall_s,
    }
    codec.close()
    del db, out, rec_off, enc_status, dec
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return res


def c4_wire_bytes_ok(torch, out, db, lo, n, chunk=1 << 22):
    """Every byte of a configs[4] shard's wire, on the device: record i is the
    44-byte header of Call(xid lo + i, prog 100003, vers 4, proc 1,
    AuthNone(None) x2) with record mark (300 - 4) | 1 << 31
    (rpc_message.rs:136-164 with call_body.rs:98-108, flavor.rs:119-122), then
    its 256 payload bytes from the arena (call_body.rs:107). Chunked, so the
    comparison temporaries stay at a few GB."""
    import numpy as np
    words = [0x80000000 | (C4_W - 4), 0, 0, 2, 100003, 4, 1, 0, 0, 0, 0]
    tmpl = torch.from_numpy(np.array(words, ">u4").view(np.uint8).copy()).to(out.device)
    wire = out[: n * C4_W].view(n, C4_W)
    pay = db.payload_arena[: n * 256].view(n, 256)
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        w = wire[a:b]
        if not torch.equal(w[:, 44:], pay[a:b]):
            return False
        if not torch.equal(w[:, :4], tmpl[:4].expand(b - a, 4)) or not torch.equal(w[:, 8:44], tmpl[8:44].expand(b - a, 36)):
            return False
        x = torch.arange(lo + a, lo + b, dtype=torch.int64, device=out.device) & 0xFFFFFFFF
        xb = torch.stack([(x >> s_) & 0xFF for s_ in (24, 16, 8, 0)], 1).to(torch.uint8)
        if not torch.equal(w[:, 4:8], xb):
            return False
    return True


def validate_iov(torch, n, iov, hdr_out, iov_tot, iov_status, wire, rec_off, hdr_len_ref, plen, hb, total_bytes,
                 hdr_total, dev):
    """The vectored encode against the contiguous encode of the same batch:
    every iovec {hdr_off, payload_off, wire_off, hdr_len, payload_len} and
    every byte of the packed headers (gathered from the wire on the device)."""
    import numpy as np
    if int((iov_status[:n] != 0).sum()) or int(iov_tot[0]) != hdr_total or int(iov_tot[1]) != total_bytes:
        return False
    e = iov[: 32 * n].view(torch.int64).view(n, 4)
    hoff, poff, woff = e[:, 0].contiguous(), e[:, 1], e[:, 2].contiguous()
    hl = e[:, 3] & 0xFFFFFFFF
    pl = (e[:, 3] >> 32) & 0xFFFFFFFF
    if not torch.equal(woff, rec_off[:n]) or not torch.equal(hl, hdr_len_ref) or not torch.equal(pl, plen):
        return False
    want_poff = torch.from_numpy(hb.msgs["payload_off"].astype(np.int64)).to(dev)
    if not torch.equal(poff, want_poff):
        return False
    if not torch.equal(hoff, torch.cumsum(hl, 0) - hl):
        return False
    ok = True
    step = 1 << 26                              # header bytes per gather slice
    for p0 in range(0, hdr_total, step):
        p = torch.arange(p0, min(hdr_total, p0 + step), dtype=torch.int64, device=dev)
        r = torch.searchsorted(hoff, p, right=True) - 1
        src = woff[r] + (p - hoff[r])
        if not torch.equal(hdr_out[p], wire[src]):
            ok = False
            break
    return ok


# ---------------------------------------------------------------------------
# c0..c3
# ---------------------------------------------------------------------------
def run_main(args, torch, R, S, SH, L, dist, rank, world, local_rank, mode):
    import numpy as np
    dev = torch.device("cuda", local_rank)
    wl = args.workload
    per_gpu_n = args.records or DEFAULT_RECORDS[wl]
    n_total = per_gpu_n * world
    lo, hi = SH.shard_bounds(n_total, world, rank)
    n = hi - lo
    if wl == "c1":
        hb = S.call_none(n, 256, seed=1 + rank, first_xid=lo)

        desc = "configs[1]: Call(prog 100003, vers 4, proc 1, AuthNone(None) x2) + 256 B payload, encode -> decode"
    elif wl == "c2":
        hb = S.mixed(n, seed=2 + rank)
        desc = ("configs[2]: mixed Call/Reply (payloads 64..4096 B), " +
                ("device stream framing" if args.frame else "rec_len scan") + " + decode")
    elif wl == "c0":
        hb = S.cpu_roundtrip(n, seed=rank)
        desc = ("configs[0] message (benches/bench.rs:86-101: Call(AuthUnix 16 gids) + AuthNone + 64 B payload) "
                "as a batch, encode -> decode")
    else:
        hb = S.call_unix16(n, 1024, seed=3 + rank)
        desc = "configs[3]: Call(AuthUnix 16 gids) + AuthNone + 1 KiB payload, encode -> decode"
    db = R.DeviceBatch.from_host(hb, dev)
    codec = R.Codec(local_rank)
    codec.reserve(n)

    # record lengths (device), output sized to the exact total
    rec_len = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    enc_status = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    codec.encode_lengths(db, rec_len, enc_status)
    lens_np = rec_len[:n].cpu().numpy().view(np.uint32).astype(np.int64)
    total_bytes = int(lens_np.sum())
    out = torch.zeros(total_bytes + 16, dtype=torch.uint8, device=dev)
    rec_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    dec_off = rec_off
    dec = R.DecodeBuffers(n, dev)
    H = parsed_bytes(hb, lens_np)
    sum_W, sum_H = total_bytes, int(H.sum())

    cache_note = ("loopback: the decode reads the wire this step's encode has just written (nontemporal stores); "
                  "descriptors and payloads are re-read every step")
    if wl == "c2":
        codec.encode(db, out, rec_off, enc_status, rec_len)     # input wire (untimed)
        torch.cuda.synchronize()
        dec_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        frame_res = torch.zeros(5, dtype=torch.int64, device=dev)
        # cold: a server decodes fresh socket bytes, so every step decodes
        # another identical copy of the wire (the header lines it reads were
        # last touched >= 2 x 256 MiB of other steps' reads ago); warm: the
        # same wire every step (its header lines stay in the Infinity Cache)
        copies = cold_copies(out, min(total_bytes, 128 * n)) if args.cache == "cold" else [out]
        cache_note = (f"cold: the step decodes one of {len(copies)} identical wire copies in rotation (>= 2x the "
                      f"256 MiB Infinity Cache of other reads between two reads of a line)" if len(copies) > 1 else
                      "warm: the same wire every step (its header lines stay in the 256 MiB Infinity Cache)")

        def make_step(nxt):
            def step():
                w = nxt()
                if args.frame:
                    codec.frame_stream(w, total_bytes, dec_off, n, frame_res)
                    codec.decode(w, dec_off, n, mode, dec.msgs, dec.unix, dec.status, dec.aux0, dec.aux1)
                else:
                    # offsets from the lengths inside the decode (onc_decode_lengths);
                    # they are also written out (dec_off: the validation below)
                    codec.decode_lengths(w, rec_len, n, 0, mode, dec.msgs, dec.unix, dec.status, dec.aux0,
                                         dec.aux1, rec_off=dec_off)
            return step
        step = make_step(rotating(copies))
    elif args.iov:
        # vectored encode; the contiguous encode of the same batch (untimed) is
        # the reference its headers and iovecs are checked against below
        codec.encode(db, out, rec_off, enc_status)
        plen = torch.from_numpy(hb.msgs["payload_len"].astype(np.int64)).to(dev)
        hdr_len_ref = rec_len[:n].to(torch.int64) & 0xFFFFFFFF
        hdr_len_ref = hdr_len_ref - torch.where(hdr_len_ref > 0, plen, torch.zeros_like(plen))
        iov_hdr_total = int(hdr_len_ref.sum())
        hdr_out = torch.zeros(iov_hdr_total + 16, dtype=torch.uint8, device=dev)
        iov = torch.zeros(max(n, 1) * 32, dtype=torch.uint8, device=dev)
        iov_tot = torch.zeros(2, dtype=torch.int64, device=dev)
        iov_status = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        sum_H = iov_hdr_total
        ALG_CTX["unix_refs"] = int(((hb.msgs["cred_kind_len"] >> 24) == L.KIND_UNIX).sum() +
                                   ((hb.msgs["verf_kind_len"] >> 24) == L.KIND_UNIX).sum())
        desc = desc.replace("encode -> decode", "vectored encode (packed headers + iovecs, payloads in place)")

        def step():
            codec.encode_iov(db, hdr_out, iov, iov_status, iov_tot, iov_hdr_total)
    else:
        def step():
            codec.encode(db, out, rec_off, enc_status)
            codec.decode(out, rec_off, n, mode, dec.msgs, dec.unix, dec.status, dec.aux0, dec.aux1)

    def barrier():
        if dist is not None:
            dist.barrier()

    tm = Timing(torch, R, codec, step, args.steps, args.warmup, barrier)
    t = torch.tensor([tm.ms, tm.ms_clean], dtype=torch.float64, device=cdev(dev))
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms_max, ms_clean_max = float(t[0]), float(t[1])

    # The other cache state, next to the primary line (SURVEY §7 "Cache
    # effects"): c2 warm (or cold); for the loopbacks, the decode alone on the
    # wire the last step encoded — the same buffer every step (warm) and
    # rotating identical copies (cold, as a server decoding fresh bytes).
    cache_legs = None
    if args.cache_leg == "on" and not args.iov:
        cache_legs = {}

        def leg(stepfn):
            tl = Timing(torch, R, codec, stepfn, args.steps, args.warmup, barrier)
            return dom_summary(tl, n, sum_W, sum_H, tl.ms / args.steps)
        if wl == "c2":
            other = [out] if args.cache == "cold" else cold_copies(out, min(total_bytes, 128 * n))
            key = "warm" if args.cache == "cold" else "cold"
            cache_legs[key] = {**leg(make_step(rotating(other))), "copies": len(other)}
            del other
        else:
            torch.cuda.synchronize()
            cc = cold_copies(out, min(total_bytes, 128 * n))

            def dec_step(nxt):
                def s():
                    codec.decode(nxt(), rec_off, n, mode, dec.msgs, dec.unix, dec.status, dec.aux0, dec.aux1)
                return s
            cache_legs["decode_only_warm"] = {**leg(dec_step(rotating([out]))), "copies": 1}
            cache_legs["decode_only_cold"] = {**leg(dec_step(rotating(cc))), "copies": len(cc)}
            del cc
        torch.cuda.empty_cache()

    # Validation of the last step (device-side, size-independent checks).
    ok = True
    if wl != "c2" and int((enc_status[:n] != 0).sum()):
        ok = False
    if args.iov:
        # every iovec and every packed header byte against the contiguous wire
        ok = ok and validate_iov(torch, n, iov, hdr_out, iov_tot, iov_status, out, rec_off, hdr_len_ref, plen,
                                 hb, total_bytes, iov_hdr_total, dev)
    else:
        if int((dec.status[:n] != 0).sum()):
            ok = False
        if int(dec_off[n]) != total_bytes:
            ok = False
        xid = dec.msgs.view(-1, 64)[:n, 0:4].contiguous().view(torch.int32).view(-1)
        want_xid = torch.from_numpy(hb.msgs["xid"].view(np.int32).copy()).to(dev)
        if not torch.equal(xid, want_xid):
            ok = False
    # global placement of this rank's shard in the job's send buffer
    shard_bytes = total_bytes if args.iov else int(dec_off[n])
    totals = SH.allgather_totals(shard_bytes) if dist is not None else [shard_bytes]
    bases, grand = SH.exclusive_bases(totals)
    ok = agree(torch, dist, dev, ok)

    # PCIe-inclusive rate: pinned host inputs -> H2D -> step -> D2H outputs.
    pcie = None
    if not args.no_pcie and not args.iov:
        if wl == "c2":
            d_in = [out, rec_len]
            d_out = [dec_off, dec.msgs, dec.unix, dec.status, dec.aux0, dec.aux1]
        else:
            d_in = [db.msgs, db.unix, db.auth_arena, db.payload_arena]
            # decoded AUTH_UNIX slots come back only if the batch has AUTH_UNIX
            # auths: no other record references a slot (onc_decoded.unix_params)
            kinds = np.concatenate([hb.msgs["cred_kind_len"] >> 24, hb.msgs["verf_kind_len"] >> 24])
            has_unix = bool((kinds == L.KIND_UNIX).any())
            d_out = [out, rec_off, enc_status, dec.msgs] + ([dec.unix] if has_unix else []) + \
                    [dec.status, dec.aux0, dec.aux1]
        h_in = [x.cpu().pin_memory() for x in d_in]
        h_out = [torch.empty(x.shape, dtype=x.dtype, pin_memory=True) for x in d_out]
        bytes_h2d = sum(x.numel() * x.element_size() for x in h_in)
        bytes_d2h = sum(x.numel() * x.element_size() for x in h_out)

        def pcie_step():
            for d, h in zip(d_in, h_in):
                d.copy_(h, non_blocking=True)
            step()
            for h, d in zip(h_out, d_out):
                h.copy_(d, non_blocking=True)
        pcie_step()
        torch.cuda.synchronize()
        barrier()
        e4 = torch.cuda.Event(enable_timing=True)
        e5 = torch.cuda.Event(enable_timing=True)
        e4.record()
        for _ in range(args.pcie_reps):
            pcie_step()
        e5.record()
        torch.cuda.synchronize()
        pms = e4.elapsed_time(e5) / args.pcie_reps
        pt = torch.tensor([pms], dtype=torch.float64, device=cdev(dev))
        if dist is not None:
            dist.all_reduce(pt, op=dist.ReduceOp.MAX)
        pms = float(pt[0])
        # the outputs that came back are the device-resident step's (checked
        # against the oracle / the encode above), byte for byte
        copied_ok = all(torch.equal(h.to(d.device, non_blocking=False), d) for h, d in zip(h_out, d_out))
        pcie = {"value": n_total / (pms / 1e3) / 1e6, "unit": "Mmsgs/s", "ms_per_step": pms, "validated": copied_ok,
                "h2d_bytes_per_gpu": bytes_h2d, "d2h_bytes_per_gpu": bytes_d2h,
                "pcie_GBs_per_gpu": (bytes_h2d + bytes_d2h) / (pms / 1e3) / 1e9,
                "note": "pinned host buffers; H2D, kernels and D2H serialized on one stream; decoded AUTH_UNIX "
                        "slots copied back when the batch has AUTH_UNIX auths"}
        pcie["pipelined"] = pcie_pipelined(args, torch, R, wl, hb, db, out, total_bytes, lens_np, rec_len,
                                           dec_off, dec, mode, h_in, local_rank, dist, n_total)
        kinds = np.concatenate([hb.msgs["cred_kind_len"] >> 24, hb.msgs["verf_kind_len"] >> 24])
        barrier()
        zc = pcie_zero_copy(args, torch, R, wl, hb, codec, out, total_bytes, lens_np, rec_off, dec_off, dec, mode,
                            n_total, bool((kinds == L.KIND_UNIX).any()))
        if wl == "c2":
            zc = reduce_leg(torch, dist, dev, zc, [""] + ([] if args.frame else [
                "variants.register_per_batch", "variants.register_per_batch_recycled", "variants.policy_standard",
                "variants.policy_line",
                "variants.policy_auto"]), n_total)
        else:
            zc.setdefault("variants", {})
            zc = reduce_leg(torch, dist, dev, zc, ["variants.in_place", "variants.wire_on_device"], n_total)
            _pick_best(zc["variants"], ["in_place", "wire_on_device"])
            v = zc["variants"]
            zc.update({"value": v.pop("value"), "ms_per_step": v.pop("ms_per_step"), "best": v.pop("best"),
                       "validated": v.pop("validated")})
        pcie["zero_copy"] = zc
        pcie = reduce_leg(torch, dist, dev, pcie, [""], n_total)
    elif args.iov and not args.no_pcie:
        barrier()
        pcie = pcie_iov(args, torch, R, L, hb, db, codec, n_total, iov_hdr_total, total_bytes, out)
        pcie = reduce_leg(torch, dist, dev, pcie, ["serialised", "pipelined", "zero_copy"], n_total)
        _pick_best(pcie, ["serialised", "pipelined", "zero_copy"])

    steps = args.steps
    ms_per_step = ms_max / steps
    value = n_total / (ms_per_step / 1e3) / 1e6       # whole-job Mmsgs/s
    wire_gibs = sum_W * world / (ms_per_step / 1e3) / 2**30
    if args.iov:
        step_alg = ALG_PER_LAUNCH["iov_len_kernel"](n, sum_W, sum_H) + ALG_PER_LAUNCH["iov_emit_kernel"](n, sum_W, sum_H)
    else:
        step_alg = (2 * sum_H + 4 * n) + (0 if wl == "c2" else 2 * sum_W)
    traffic, tsrc = load_traffic(args.traffic_json, wl, n, tm.dom)
    per_gpu = gather_per_gpu(torch, dist, dev, rank, n, tm.ms / steps, tm.ms_clean / steps)
    for r, row in enumerate(per_gpu):
        row["global_base"] = int(bases[r])
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "Mmsgs/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": f"synthetic (seeded): {desc}",
        "config": {"workload": f"{desc}; {n} records per GPU ({args.mode} mode), HBM-resident",
                   "records_per_gpu": n, "wire_bytes_per_gpu": sum_W, "parsed_bytes_per_gpu": sum_H,
                   "decode_mode": args.mode,
                   "cache": (args.cache if wl == "c2" else "loopback"), "cache_note": cache_note,
                   "parallelism": f"record-sharded x{world} (no collective)"},
        "cache_legs": cache_legs,
        "wire_GiB_per_s": wire_gibs,
        "ms_per_step_without_kernel_events": ms_clean_max / steps,
        "step_alg_GBs": step_alg * world / (ms_per_step / 1e3) / 1e9,
        "roofline": roofline(tm, n, sum_W, sum_H, step_alg, ms_per_step, traffic, tsrc),
        "per_gpu": per_gpu,
        "global_send_buffer": {"shard_bytes": totals, "bases": [int(b) for b in bases], "total": grand},
        "kernels_breakdown_pass": breakdown_dict(tm, n, sum_W, sum_H),
        "pcie_inclusive": pcie,
        "validated": ok,
        "wall_s_timed_region": tm.wall_s,
    }
    if args.iov:
        result["config"]["header_bytes_per_gpu"] = sum_H
        result["config"].pop("parsed_bytes_per_gpu", None)
        result["config"].pop("decode_mode", None)
    if rank == 0 and not args.no_cpu_baseline and not args.iov:
        prefix = out[: min(total_bytes, 20_000 * 4300)].cpu().numpy().tobytes()
        wire_np = out.cpu().numpy()
        off_np = dec_off.cpu().numpy().view(np.uint64)
        if world == 1:
            result["cpu_baseline"] = cpu_baseline(args, wl, hb, prefix, wire_np, off_np, mode)
        else:
            # N > 1: rank 0 times it after every GPU leg of every rank (main()),
            # so no rank's timed region shares the host with it
            result["_cpu_pending"] = (wl, hb, prefix, wire_np, off_np, mode)
    elif rank == 0:
        result["cpu_baseline"] = None
    codec.close()
    del db, out, rec_off, dec_off, dec, enc_status, rec_len
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return result


def host_pinned_peak(dist, world):
    """Peak pinned host memory of this run: torch's pinned allocator (the
    staging legs' pin_memory buffers) + the host ranges registered through
    runtime.HostMapped (the zero-copy legs), per rank and summed over the
    ranks that share this host (the sum of per-rank peaks bounds the
    simultaneous total from above)."""
    import torch
    R = sys.modules.get("onc_rpc_amd.runtime")
    if R is None or not torch.cuda.is_available():          # (--check-launch: no GPU legs ran)
        return None
    st = torch.cuda.host_memory_stats() if hasattr(torch.cuda, "host_memory_stats") else {}
    tp = 0
    for k in ("allocated_bytes.peak", "reserved_bytes.peak", "allocated_bytes.all.peak"):
        if k in st:
            tp = max(tp, int(st[k]))
    mine = float(tp + R.HostMapped.peak_bytes)
    out = {"per_rank_peak_bytes": mine, "torch_pinned_peak_bytes": tp, "host_mapped_peak_bytes": R.HostMapped.peak_bytes}
    if dist is not None and world > 1:
        t = torch.tensor([mine, mine], dtype=torch.float64, device=cdev(torch.cuda.current_device()))
        s = t.clone()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        out.update({"per_rank_peak_bytes_max": float(t[0]), "sum_over_ranks_bytes": float(s[0])})
    else:
        out["sum_over_ranks_bytes"] = mine
    return out


def finish(args, result, pending, dist, rank, world):
    """Closing step of every run: with N > 1 ranks, rank 0 times the CPU
    baseline (`pending`: the arguments cpu_baseline needs) only after every
    rank's GPU legs are done — no timed region shares the host with it —
    then rank 0 prints the one JSON line."""
    if dist is not None:
        dist.barrier()                  # every rank's GPU legs are done
    result["host_pinned"] = host_pinned_peak(dist, world)
    if pending is not None:
        cb = cpu_baseline(args, *pending)
        if world > 1:
            cb["note"] = (f"timed on rank 0 after all {world} ranks finished their GPU legs (the other ranks "
                          f"wait at the closing barrier); rank 0's shard of the same workload")
        result["cpu_baseline"] = cb
    if dist is not None:
        dist.barrier()
    if rank == 0:
        print(json.dumps(result), flush=True)


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and (args.gpus or 1) > 1:
        # one process per GPU, started before this process touches the GPU
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(world_env or "1")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("ONC_BENCH_SAME_DEVICE") == "1":
        # lab: every rank on GPU 0 (exercises the multi-rank path on a 1-GPU box; use --backend gloo)
        local_rank = 0
    if args.gpus is None:
        args.gpus = world
    if args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.check_launch:
        check_launch(args, world, rank)
        return

    import torch

    import _onc_pkg

    _onc_pkg.load()
    import onc_rpc_amd.layout as L
    import onc_rpc_amd.runtime as R
    import onc_rpc_amd.shard as SH
    import onc_rpc_amd.synth as S

    if args.variant:
        R.DEFAULT_OPTIONS["variant"] = args.variant     # A/B measurements: every codec of the run
    if args.decode_policy != "auto":
        R.DEFAULT_OPTIONS["decode_policy"] = {"standard": R.DECODE_POLICY_STANDARD,
                                              "line": R.DECODE_POLICY_LINE}[args.decode_policy]
    dist = None
    torch.cuda.set_device(local_rank)
    if world > 1:
        import torch.distributed as dist
        BACKEND[0] = args.backend
        dist.init_process_group(args.backend)
        if dist.get_world_size() != args.gpus:
            sys.exit(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
    mode = L.DECODE_BYTES if args.mode == "bytes" else L.DECODE_SLICE

    if args.workload == "c4":
        result = run_c4(args, torch, R, S, SH, L, dist, rank, world, local_rank,
                        args.records or DEFAULT_RECORDS["c4"], mode, args.steps, args.warmup)
        result["vs_baseline"] = None
        ok = result.get("validated", False)
    else:
        result = run_main(args, torch, R, S, SH, L, dist, rank, world, local_rank, mode)
        ok = result["validated"]
        if args.workload == "c1" and not args.iov and args.iov_leg == "on":
            import copy
            la = copy.copy(args)
            la.iov, la.no_cpu_baseline = True, True
            leg = run_main(la, torch, R, S, SH, L, dist, rank, world, local_rank, mode)
            ok = ok and leg["validated"]
            result["vectored_encode"] = {k: leg[k] for k in ("value", "unit", "ms_per_step", "validated", "data",
                                                             "roofline", "kernels_breakdown_pass",
                                                             "pcie_inclusive")}
            result["vectored_encode"]["note"] = ("onc_encode_iov (SURVEY §8(f) rank 2) of the same configs[1] "
                                                 "batch: packed headers + 32-byte iovecs, payloads in place; "
                                                 "checked byte for byte against the contiguous encode")
        if args.c4_leg == "on":
            result["configs4"] = run_c4(args, torch, R, S, SH, L, dist, rank, world, local_rank,
                                        args.c4_records, mode, args.steps, args.warmup)
    finish(args, result, result.pop("_cpu_pending", None) if rank == 0 else None, dist, rank, world)
    if dist is not None:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
