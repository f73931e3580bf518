#!/bin/bash
# GPU suite (product default: no preload), then c1: HEAD / HEAD with the
# pipeline on every shape (no header-heavy sample) / the round-3 tree, 3
# interleaved rounds; c0 HEAD vs round 3.
set -u
mkdir -p gpurun_out
OUT=$PWD/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
CASES="head:. headpipe:.:0x10000 r3:build/r3" ROUNDS=3 WLS="c1" bash scripts/ab_tree.sh || exit $?
CASES="head:. r3:build/r3" ROUNDS=1 WLS="c0" bash scripts/ab_tree.sh
