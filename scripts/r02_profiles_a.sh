#!/bin/bash
# Round-2 evidence, part A: GPU tests, smoke, bench lines of every workload.
set -u
mkdir -p gpurun_out/r02
O=gpurun_out/r02
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python __graft_entry__.py smoke > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench_c1.log 2>&1; rc=$?; echo "bench c1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
for wl in c2 c3 c0; do
  timeout -k 10 300 python bench.py --workload $wl --c4-leg off > $O/bench_$wl.log 2>&1; rc=$?; echo "bench $wl rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python bench.py --workload c2 --frame --c4-leg off --no-cpu-baseline > $O/bench_c2f.log 2>&1; rc=$?; echo "bench c2f rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload c4 > $O/bench_c4.log 2>&1; rc=$?; echo "bench c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --records 8000000 --c4-leg off --no-cpu-baseline --no-pcie > $O/bench_c1_8m.log 2>&1; rc=$?; echo "bench c1 8M rc=$rc"
