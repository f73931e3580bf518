"""The oracle under AddressSanitizer + UndefinedBehaviorSanitizer
(oracle/fuzz_oracle.c, `make -C oracle fuzz_asan`): the reference's two
fuzz invariants — fuzz/fuzz_targets/parse_serialise.rs:5-12 (decode ->
serialise -> decode is the identity) and fuzz/fuzz_targets/bytes.rs:8-23
(slice and Bytes decoders agree on Ok/Err and re-serialise identically) —
over generated valid messages, mutants of them and short random buffers,
each input in a heap block of exactly its length (an over-read is an ASan
report). Host code only; no GPU."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


@pytest.fixture(scope="module")
def fuzzer():
    subprocess.check_call(["make", "-C", ORACLE, "-s", "fuzz_asan"])
    return os.path.join(ORACLE, "fuzz_oracle_asan")


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_fuzz_invariants_under_sanitizers(fuzzer, seed):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([fuzzer, "60000", str(seed)], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stdout + p.stderr[-3000:]
    assert "ERROR" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-3000:]
    m = re.search(r"slice ok (\d+) err (\d+); bytes ok (\d+) err (\d+)", p.stdout)
    ok_s, err_s, ok_b, err_b = (int(x) for x in m.groups())
    # every generated message decodes; the mutants exercise the error paths
    assert ok_s >= 60000 and err_s > 10000 and ok_b == ok_s and err_b == err_s
