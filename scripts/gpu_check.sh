#!/bin/bash
# GPU round script: parity tests, smoke, bench, rocprofv3 kernel trace.
# Each GPU step is time-limited; a crash/timeout stops the script.
set -u
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc || exit $rc
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; ok $rc || exit $rc
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; ok $rc || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie > gpurun_out/prof.log 2>&1; rc=$?; echo "rocprof rc=$rc"
fi
