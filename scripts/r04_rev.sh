#!/bin/bash
# decode workgroups in reverse record order (the loopback's decode reads the
# lines the encode wrote last first): GPU suite, then c1 / c0 / c3 / c2 / c4
# against the HEAD tree (build/h1), one box, 3 interleaved rounds.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/rev_tests.log 2>&1; rc=$?; tail -2 gpurun_out/rev_tests.log; [ $rc = 0 ] || exit $rc
CASES="h1:build/h1 rev:." ROUNDS=3 WLS="c1 c0 c3 c2" bash scripts/ab_tree.sh || exit $?
CASES="h1:build/h1 rev:." ROUNDS=2 WLS="c4" bash scripts/ab_tree.sh
