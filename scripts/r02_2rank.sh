#!/bin/bash
# The multi-rank bench path end to end on a 1-GPU box: 2 ranks (spawned by
# bench.py itself), both on GPU 0, gloo control plane.
set -u
mkdir -p gpurun_out/2r
export ONC_BENCH_SAME_DEVICE=1
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --no-cpu-baseline --c4-records 16000000 > gpurun_out/2r/c1.log 2>&1; rc=$?; echo "2-rank c1 rc=$rc"; tail -c 400 gpurun_out/2r/c1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --workload c4 --records 16000000 > gpurun_out/2r/c4.log 2>&1; rc=$?; echo "2-rank c4 rc=$rc"; tail -c 300 gpurun_out/2r/c4.log
