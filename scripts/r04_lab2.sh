#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/mix_lab.py 1000000 10 sweep > gpurun_out/lab_mix_sweep.log 2>&1; rc=$?
echo "sweep rc=$rc"; cat gpurun_out/lab_mix_sweep.log | grep -v amdgpu.ids; exit $rc
