#!/bin/bash
# GPU suite, then the kernel-choice lab (half/half mixes and the sweep) with
# the payload >= 4x header rule.
set -u
mkdir -p gpurun_out
OUT=$PWD/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/mix_lab.py 1000000 20 > $OUT/lab_mix.log 2>&1; rc=$?
echo "mix rc=$rc"; grep -v amdgpu.ids $OUT/lab_mix.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/mix_lab.py 1000000 10 sweep > $OUT/lab_mix_sweep.log 2>&1; rc=$?
echo "sweep rc=$rc"; grep -v amdgpu.ids $OUT/lab_mix_sweep.log; exit $rc
