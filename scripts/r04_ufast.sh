#!/bin/bash
# decode: wave-uniform fast path for waves of Calls with an empty-name
# AUTH_UNIX credential and an AUTH_NONE verifier (configs[0] / [3]): GPU
# suite, then c3 / c0 / c1 (3 rounds) and c4 (2) against HEAD (build/h4).
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/ufast_tests.log 2>&1; rc=$?; tail -1 gpurun_out/ufast_tests.log; [ $rc = 0 ] || exit $rc
CASES="h4:build/h4 ufast:." ROUNDS=3 WLS="c3 c0 c1" bash scripts/ab_tree.sh || exit $?
CASES="h4:build/h4 ufast:." ROUNDS=2 WLS="c4" bash scripts/ab_tree.sh
