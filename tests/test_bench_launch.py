"""bench.py's multi-GPU launcher on the CPU: `--gpus N`
without WORLD_SIZE spawns N ranks under torch.distributed.run (one process
per GPU) as a child process, and every rank checks that the process
group's world size equals --gpus. --check-launch stops after the rendezvous
(gloo backend, no GPU call)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(extra_env or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    return p


def test_gpus_n_spawns_n_ranks():
    p = _run(["--gpus", "2", "--check-launch", "--backend", "gloo"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["gpus_arg"] == 2 and r["backend"] == "gloo"
    assert [x[0] for x in r["ranks"]] == [0, 1]
    pids = {x[1] for x in r["ranks"]}
    assert len(pids) == 2 and os.getpid() not in pids


def test_single_gpu_runs_in_process():
    p = _run(["--check-launch"])
    assert p.returncode == 0, p.stderr[-2000:]
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert r["n_gpus"] == 1 and len(r["ranks"]) == 1


def test_gpus_must_match_world_size():
    p = _run(["--gpus", "2", "--check-launch"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "--gpus 2 but WORLD_SIZE=1" in p.stderr


def test_gpus_2_line_carries_cpu_baseline():
    """N > 1: rank 0 times the reference-semantics CPU baseline after every
    rank's legs (bench.finish), so a --gpus 2 line carries cpu_baseline next
    to the multi-GPU numbers (north_star: 1/2/4/8-GPU numbers next to the CPU
    path timed on the same box in the same run). CPU rehearsal: gloo, the
    closing step of a real run on an oracle-encoded sample."""
    p = _run(["--gpus", "2", "--check-launch", "--backend", "gloo", "--cpu-check-records", "3000",
              "--cpu-seconds", "0.4", "--cpu-threads", "2"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    r = json.loads(lines[0])
    cb = r["cpu_baseline"]
    assert r["n_gpus"] == 2 and cb["kind"] == "port" and cb["cores"] == 2 and cb["value"] > 0
    assert cb["sample_bit_exact_vs_gpu"] is True and "after all 2 ranks" in cb["note"]
