#!/bin/bash
# enc_len payload totals from a u32 wave sum of header bytes (was: packed scan):
# emit-path tests, the kernel-choice lab (auto must stay with the better
# kernel), then c1 / c4 / c3 against HEAD (build/h3), 3 rounds.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_emit_paths.py \
  tests/test_gpu_r03.py tests/test_gpu_parity.py > gpurun_out/len_tests.log 2>&1; rc=$?; tail -1 gpurun_out/len_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/mix_lab.py 1000000 10 > gpurun_out/len_mix.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/len_mix.log; [ $rc = 0 ] || exit $rc
CASES="h3:build/h3 len:." ROUNDS=3 WLS="c1 c4 c3" bash scripts/ab_tree.sh
