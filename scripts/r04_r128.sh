#!/bin/bash
# decode line policy: round 1 also takes at least the record's first 128
# bytes: GPU suite, then c0 / c3 / c1 / c2 against HEAD (build/h2), 3 rounds.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/r128_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r128_tests.log; [ $rc = 0 ] || exit $rc
CASES="h2:build/h2 r128:." ROUNDS=3 WLS="c0 c3 c1 c2" bash scripts/ab_tree.sh
