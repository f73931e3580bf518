#!/bin/bash
# configs[0]-shaped emit with a 640-chunk image (one span per 64-record tile,
# 3 waves per SIMD; build/i640) with and without the credential preload
# (variant 0x80000), against HEAD (build/h3): emit-path tests on i640, then
# c0, 3 rounds.
set -u
mkdir -p gpurun_out
(cd build/i640 && timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_emit_paths.py > ../../gpurun_out/i640_tests.log 2>&1); rc=$?; tail -1 gpurun_out/i640_tests.log; [ $rc = 0 ] || exit $rc
CASES="h3:build/h3 h3pre:build/h3:524288 i640:build/i640 i640pre:build/i640:524288" ROUNDS=3 WLS="c0" bash scripts/ab_tree.sh
