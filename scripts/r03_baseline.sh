#!/bin/bash
# Round-3 first call: the driver's default bench + the configs[0] and 8M-record c1 lines on the round-2 code.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/r03_base_c1.log 2>&1; rc=$?; echo "bench c1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c0 --no-cpu-baseline --no-pcie --c4-leg off > gpurun_out/r03_base_c0.log 2>&1; rc=$?; echo "bench c0 rc=$rc"; [ $rc -eq 0 ] || exit $rc
