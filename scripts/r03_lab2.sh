#!/bin/bash
# Round 3 lab 2: forced emit-path tests, re-encode timings, c1/c0 bench lines.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_emit_paths.py tests/test_gpu_r03.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_paths.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests_paths.log; [ $rc -eq 0 ] || exit $rc
for wl in c0 c1; do
  timeout -k 10 200 python -u tools/reencode_lab.py $wl 1000000 10 > gpurun_out/reencode_$wl.log 2>&1; rc=$?; echo "reencode $wl rc=$rc"; tail -3 gpurun_out/reencode_$wl.log; [ $rc -eq 0 ] || exit $rc
done
for wl in c1 c0; do
  timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --no-pcie --c4-leg off --iov-leg off > gpurun_out/bench_$wl.log 2>&1; rc=$?; echo "bench $wl rc=$rc"; python3 scripts/summ.py gpurun_out/bench_$wl.log; [ $rc -eq 0 ] || exit $rc
done
