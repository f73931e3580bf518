#!/bin/bash
# SQ instruction / wait counters of the decode (and the other kernels) on c0
# and c1: two rocprofv3 --pmc passes per workload, kernel trace only.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=$PWD/gpurun_out
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY"
P2="SQ_WAVES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS"
for wl in c0 c1; do
  i=0
  for grp in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/sq_${wl}_$i -o run --output-format csv -- \
      python3 bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --c4-leg off --iov-leg off \
      --cache-leg off > $OUT/sq_${wl}_$i.log 2>&1
    rc=$?; echo "sq $wl pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 scripts/sq_json.py $OUT/sq_$wl.json "rocprofv3 --kernel-trace --pmc, 2 passes over bench.py --workload $wl --steps 3 --warmup 1" \
    $(ls $OUT/sq_${wl}_1/*counter_collection.csv) $(ls $OUT/sq_${wl}_2/*counter_collection.csv) | grep onc
done
