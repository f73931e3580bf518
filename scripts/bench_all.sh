#!/bin/bash
# All bench workloads (c1 headline, c2 decode, c3 loopback) on one GPU.
set -u
mkdir -p gpurun_out
for wl in c1 c2 c3 c0; do
  timeout -k 10 400 python bench.py --workload $wl ${BENCH_ARGS:-} > gpurun_out/bench_$wl.log 2>&1
  rc=$?; echo "bench $wl rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python bench.py --workload c2 --frame ${BENCH_ARGS:-} > gpurun_out/bench_c2f.log 2>&1; rc=$?; echo "bench c2f rc=$rc"; [ $rc -eq 0 ] || exit $rc
