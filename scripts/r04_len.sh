#!/bin/bash
# enc_len with one packed wave scan (lengths and header bytes) instead of two:
# emit-path tests, the kernel-choice lab (auto must stay with the better
# kernel), then c1 / c4 / c3 against HEAD (build/h2), 3 rounds.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_emit_paths.py \
  tests/test_gpu_r03.py tests/test_gpu_parity.py > gpurun_out/len_tests.log 2>&1; rc=$?; tail -1 gpurun_out/len_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/mix_lab.py 1000000 10 > gpurun_out/len_mix.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/len_mix.log; [ $rc = 0 ] || exit $rc
CASES="h2:build/h2 len:." ROUNDS=3 WLS="c1 c4 c3" bash scripts/ab_tree.sh
