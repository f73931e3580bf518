#!/bin/bash
# SQ counters of the product kernels on configs[1] (two passes of 8 SQ counters, --kernel-trace only).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=$PWD/gpurun_out
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/sq_$i -o run --output-format csv -- \
      python3 bench.py --workload ${WL:-c1} --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --c4-leg off --iov-leg off > $OUT/sq_$i.log 2>&1
  rc=$?; echo "pmc group $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
