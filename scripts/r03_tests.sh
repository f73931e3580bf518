#!/bin/bash
# GPU suite (one process), then the default bench line. Each GPU step time-limited; a failure stops the script.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
if [ -z "${NO_BENCH:-}" ]; then
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c1.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench_c1.log; [ $rc -eq 0 ] || exit $rc
fi
