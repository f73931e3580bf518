#!/bin/bash
# GPU suite, then HEAD against the round-3 tree (build/r3) on c0 / c1 / c3,
# interleaved; c0 also without the credential preload (variant 0x80000).
set -u
mkdir -p gpurun_out
OUT=$PWD/gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
CASES="head:. r3:build/r3 headnopre:.:0x80000" ROUNDS=2 WLS="c0" bash scripts/ab_tree.sh || exit $?
CASES="head:. r3:build/r3" ROUNDS=2 WLS="c1 c3" bash scripts/ab_tree.sh
