#!/bin/bash
# last-round split of the wave-specialised enc_emit: emit-path tests, then
# c1 / c4 against the HEAD tree (build/h0) on one box, 3 interleaved rounds.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_emit_paths.py \
  > gpurun_out/split_tests.log 2>&1; rc=$?; tail -3 gpurun_out/split_tests.log; [ $rc = 0 ] || exit $rc
CASES="h0:build/h0 new:." ROUNDS=3 WLS="c1 c4" bash scripts/ab_tree.sh
rc=$?; [ $rc = 0 ] || exit $rc
timeout -k 10 200 ./tools/dec_lab 1000000 300 > gpurun_out/lab_dec_memset.log 2>&1 || exit $?
LAB_SCRUB=read timeout -k 10 200 ./tools/dec_lab 1000000 300 > gpurun_out/lab_dec_read.log 2>&1 || exit $?
LAB_WARM=1 timeout -k 10 200 ./tools/dec_lab 1000000 300 > gpurun_out/lab_dec_warm.log 2>&1 || exit $?
grep -h product gpurun_out/lab_dec_*.log
