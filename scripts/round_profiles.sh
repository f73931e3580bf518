#!/bin/bash
# Round-end evidence: parity tests, smoke, benches (c1 c2 c3 c2f), rocprofv3
# kernel stats of the headline bench, PMC traffic for c1/c2/c3. Each GPU step
# time-limited; a failure stops the script.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/bench_all.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie > gpurun_out/prof.log 2>&1; rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_all.sh
