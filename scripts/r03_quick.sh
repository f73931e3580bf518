#!/bin/bash
# Quick bench lines: the driver's default command plus the given workloads (no CPU baseline / PCIe / c4 leg).
# Each GPU step time-limited; a failure stops the script.
set -u
mkdir -p gpurun_out
TAG=${TAG:-q}
if [ -z "${NO_DEFAULT:-}" ]; then
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_default.log 2>&1; rc=$?; echo "bench default rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
for wl in ${WORKLOADS:-c0 c2}; do
  timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --no-pcie --c4-leg off --iov-leg off ${BENCH_ARGS:-} > gpurun_out/${TAG}_$wl.log 2>&1; rc=$?; echo "bench $wl rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
