#!/bin/bash
# Nontemporal payload loads in enc_emit: the product now uses them for long
# payloads (a.ws == 2, configs[3]); ntws also for the wave-specialised kernel's
# 2 KiB steps (configs[1] / [4]), ntt also for the wave-per-tile kernel
# (configs[0]-shaped). Emit-path + iov tests on the product, then 3 rounds.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_emit_paths.py \
  tests/test_gpu_r03.py > gpurun_out/nt_tests.log 2>&1; rc=$?; tail -1 gpurun_out/nt_tests.log; [ $rc = 0 ] || exit $rc
CASES="new:. ntws:build/ntws" ROUNDS=3 WLS="c1 c4" bash scripts/ab_tree.sh || exit $?
CASES="new:. ntt:build/ntt" ROUNDS=3 WLS="c0" bash scripts/ab_tree.sh
