"""Markdown rows of DESIGN.md §5's round-6 table from the committed bench
lines (profiles/bench_r06_*.log): value, µs/step (event-free), dominant
kernel, achieved GB/s, fraction of 8 TB/s, whole-step fraction, counted HBM
traffic per launch."""
import json
import sys

ROWS = [("default", "**c1** (headline: 1M × Call/AuthNone + 256 B, encode → decode)"),
        ("c2", "c2 (1M mixed Call/Reply 64–4096 B: `onc_decode_lengths`, cold)"),
        ("c3", "c3 (4M × Call/AuthUnix16 + 1 KiB)"),
        ("c0", "c0 (configs[0]'s message as a 1M batch)"),
        ("c4", "c4 (configs[4]: 64M × 300 B on one GPU)"),
        ("c2f", "c2 + device framing (`--frame`)"),
        ("iov_c1", "c1 vectored encode (`--iov`)"),
        ("iov_c3", "c3 vectored encode"),
        ("iov_c0", "c0 vectored encode")]


def line(path):
    return json.loads([x for x in open(path) if x.startswith("{")][-1])


def main(root="profiles"):
    print("| Workload | value (Mmsgs/s) | µs/step (no events) | dominant kernel (per launch) | achieved | frac of 8 TB/s "
          "| step frac | HBM traffic / launch |")
    print("|---|---|---|---|---|---|---|---|")
    for tag, name in ROWS:
        try:
            d = line(f"{root}/bench_r06_{tag}.log")
        except (OSError, IndexError):
            continue
        r = d["roofline"]
        t = r.get("traffic")
        alg = r.get("alg_bytes_per_launch")
        traffic = f"{t / 1e6:.0f} MB (alg {alg / 1e6:.0f} MB)" if t else (f"— (alg {alg / 1e6:.0f} MB)" if alg else "—")
        ok = "" if d.get("validated") else " (NOT validated)"
        def g(x):
            return f"{x:,.0f}".replace(",", " ")
        print(f"| {name} | {g(d['value'])}{ok} | {d['ms_per_step'] * 1e3:.1f} "
              f"({d.get('ms_per_step_without_kernel_events', d['ms_per_step']) * 1e3:.1f}) | "
              f"`{r['kernel'].replace('_kernel', '')}` {r['avg_launch_us']:.1f} µs | {g(r['achieved'])} GB/s | "
              f"{r['frac']:.2f} | {r.get('step_frac', float('nan')):.2f} | {traffic} |")


if __name__ == "__main__":
    main(*sys.argv[1:])


def pcie(root="profiles"):
    """The PCIe-inclusive table (Mmsgs/s): staged serialised / pipelined,
    zero copy, the vectored encode's three legs, the CPU baseline."""
    def v(x):
        return f"{x['value']:.1f}" if isinstance(x, dict) and x.get("value") and x.get("validated") else "—"
    print("| Workload | staged, serialised | staged, pipelined | zero copy | vectored: serialised / pipelined / "
          "zero copy | CPU (oracle, 16 threads) |")
    print("|---|---|---|---|---|---|")
    for tag, iov, name in (("c2", None, "c2 (decode, 1M mixed, 1.92 GB wire)"),
                           ("default", "iov_c1", "c1 (loopback, 1M × 300 B)"),
                           ("c3", "iov_c3", "c3 (loopback, 4M × 1152 B)"),
                           ("c0", "iov_c0", "c0 (loopback, 1M × 192 B)")):
        d = line(f"{root}/bench_r06_{tag}.log")
        p = d.get("pcie_inclusive") or {}
        z = p.get("zero_copy") or {}
        zv = z.get("variants") or {}
        if tag == "c2":
            zc = f"**{v(z)}** (registered once)"
        else:
            zc = f"{v(zv.get('in_place'))} (in place) / {v(zv.get('wire_on_device'))} (wire on device)"
        if iov:
            q = line(f"{root}/bench_r06_{iov}.log").get("pcie_inclusive") or {}
            vec = f"{v(q.get('serialised'))} / {v(q.get('pipelined'))} / {v(q.get('zero_copy'))}"
        else:
            vec = "—"
        cpu = (d.get("cpu_baseline") or {}).get("value")
        print(f"| {name} | {v(p)} | {v(p.get('pipelined'))} | {zc} | {vec} | {cpu:.1f} |")
