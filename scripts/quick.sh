#!/bin/bash
# Quick GPU iteration: parity tests, then c1/c3 bench lines (no CPU baseline / PCIe legs).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for wl in ${WLS:-c1 c3}; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --no-pcie > gpurun_out/bench_$wl.log 2>&1; rc=$?; echo "bench $wl rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
