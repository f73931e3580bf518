#!/bin/bash
# framer: the output clears in frame_guess instead of two fills (the walk
# fold into frame_chunks measured slower first): GPU suite, then c2 + framing
# against HEAD (build/h4), 3 rounds.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/walk_tests.log 2>&1; rc=$?; tail -1 gpurun_out/walk_tests.log; [ $rc = 0 ] || exit $rc
CASES="h4:build/h4 walk:." ROUNDS=3 WLS="c2" BARGS="--frame" bash scripts/ab_tree.sh
