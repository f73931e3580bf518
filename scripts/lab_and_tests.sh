#!/bin/bash
# Dev loop: emit lab timings (aligned and odd payloads), then the GPU parity tests (each step time-limited).
set -u
mkdir -p gpurun_out
timeout -k 10 120 ./tools/emit_lab > gpurun_out/lab.log 2>&1; rc=$?; echo "lab rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/emit_lab 1000000 255 > gpurun_out/lab255.log 2>&1; rc=$?; echo "lab255 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; exit $rc
