#!/bin/bash
# multi-rank GPU test, decode MLP lab, SQ counters of the product enc_emit.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_r02.py -m gpu -x -v --timeout 240 --timeout-method thread -k two_ranks > gpurun_out/gpu_tests_2r.log 2>&1; rc=$?; echo "pytest 2r rc=$rc"; tail -3 gpurun_out/gpu_tests_2r.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 ./tools/dec_lab 1000000 300 > gpurun_out/declab_300_cold.log 2>&1 || exit $?
LAB_WARM=1 timeout -k 10 120 ./tools/dec_lab 1000000 300 > gpurun_out/declab_300_warm.log 2>&1 || exit $?
timeout -k 10 120 ./tools/dec_lab 1000000 1936 > gpurun_out/declab_1936_cold.log 2>&1 || exit $?
cat gpurun_out/declab_*.log
export TMPDIR=/tmp
OUT=$PWD/gpurun_out
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/sq_$i -o run --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --c4-leg off > $OUT/sq_$i.log 2>&1
  rc=$?; echo "pmc group $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
