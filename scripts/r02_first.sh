#!/bin/bash
# Round-2 first GPU pass: new tests first (fail fast), full GPU suite, smoke, default bench.
set -u
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_r02.py -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/gpu_tests_r02.log 2>&1; rc=$?; echo "pytest r02 rc=$rc"; tail -5 gpurun_out/gpu_tests_r02.log; ok $rc || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log; ok $rc || exit $rc
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; ok $rc || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench.log
