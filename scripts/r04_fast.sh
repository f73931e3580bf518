#!/bin/bash
# decode: wave-uniform fast path for all-simple-Call waves (AUTH_NONE x2):
# GPU suite, then c1 / c4 / c2 / c3 / c0 against HEAD (build/h1), one box, 3 rounds.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/fast_tests.log 2>&1; rc=$?; tail -2 gpurun_out/fast_tests.log; [ $rc = 0 ] || exit $rc
CASES="h1:build/h1 fast:." ROUNDS=3 WLS="c1 c2 c3 c0" bash scripts/ab_tree.sh || exit $?
CASES="h1:build/h1 fast:." ROUNDS=2 WLS="c4" bash scripts/ab_tree.sh
