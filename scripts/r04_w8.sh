#!/bin/bash
# decode with an 8-chunk window (8 KiB LDS per workgroup: 5 waves per SIMD
# instead of 4) — GPU suite on that tree, then c1 / c2 / c3 / c0 against
# HEAD (build/h3), 3 rounds.
set -u
mkdir -p gpurun_out
(cd build/w8 && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
  > ../../gpurun_out/w8_tests.log 2>&1); rc=$?; tail -1 gpurun_out/w8_tests.log; [ $rc = 0 ] || exit $rc
CASES="h3:build/h3 w8:build/w8" ROUNDS=3 WLS="c1 c2 c3 c0" bash scripts/ab_tree.sh
