#!/bin/bash
# decode: a call's and an accepted reply's verifier parsed by one joined
# auth_any (mixed waves run it twice instead of three times; 25 % less code):
# GPU suite, then c2 / c1 / c3 / c0 against HEAD (build/h4), 3 rounds.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/join_tests.log 2>&1; rc=$?; tail -1 gpurun_out/join_tests.log; [ $rc = 0 ] || exit $rc
CASES="h4:build/h4 join:." ROUNDS=3 WLS="c2 c1 c3 c0" bash scripts/ab_tree.sh
