#!/bin/bash
# wave-specialised enc_emit with the tile's descriptors kept in LDS for the
# producer's header builds (no per-span reload): emit-path tests, then c1 /
# c4 / c3 against the HEAD tree (build/h0), and (v2) the same plus the consumers
# pulling the first tile's payload lines toward L2 during the first staging; 3 rounds.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_emit_paths.py \
  > gpurun_out/desc_tests.log 2>&1; rc=$?; tail -3 gpurun_out/desc_tests.log; [ $rc = 0 ] || exit $rc
(cd build/v2 && timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_emit_paths.py > ../../gpurun_out/desc_tests_v2.log 2>&1); rc=$?; tail -1 gpurun_out/desc_tests_v2.log
[ $rc = 0 ] || exit $rc
CASES="h0:build/h0 new:. v2:build/v2" ROUNDS=3 WLS="c1 c4 c3" bash scripts/ab_tree.sh
