#!/bin/bash
# wave-specialised enc_emit: the producer also streams a quarter of each span
# (4 parts) — product for long payloads (configs[3]); p2 also for the 2 KiB
# instance (configs[1] / [4]). Emit-path tests on both, then c3 (product vs
# HEAD build/h4) and c1 / c4 (p2 vs HEAD), 3 rounds.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_emit_paths.py \
  tests/test_gpu_r03.py > gpurun_out/prod_tests.log 2>&1; rc=$?; tail -1 gpurun_out/prod_tests.log; [ $rc = 0 ] || exit $rc
(cd build/p2 && timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_emit_paths.py > ../../gpurun_out/prod_tests_p2.log 2>&1); rc=$?; tail -1 gpurun_out/prod_tests_p2.log; [ $rc = 0 ] || exit $rc
CASES="h4:build/h4 prod:." ROUNDS=3 WLS="c3" bash scripts/ab_tree.sh || exit $?
CASES="h4:build/h4 p2:build/p2" ROUNDS=3 WLS="c1 c4" bash scripts/ab_tree.sh
