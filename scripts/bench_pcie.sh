#!/bin/bash
# Bench lines with both PCIe-inclusive legs (serialized and pipelined), no CPU baseline (dev helper).
set -u
mkdir -p gpurun_out
for wl in ${WLS:-c1 c2 c3}; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/bench_pcie_$wl.log 2>&1; rc=$?; echo "bench $wl rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
