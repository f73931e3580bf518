#!/bin/bash
# Round 3 lab 1: re-encode-from-wire timings (c0, c1) and SQ instruction counts of the c2 decode.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=$PWD/gpurun_out
for wl in c0 c1; do
  timeout -k 10 200 python -u tools/reencode_lab.py $wl 1000000 10 > $OUT/reencode_$wl.log 2>&1; rc=$?; echo "reencode $wl rc=$rc"; cat $OUT/reencode_$wl.log | tail -12; [ $rc -eq 0 ] || exit $rc
done
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY" "SQ_WAVES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $grp -d $OUT/sq_c2_$i -o run --output-format csv -- \
      python3 bench.py --workload c2 --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --c4-leg off > $OUT/sq_c2_$i.log 2>&1
  rc=$?; echo "sq group $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/sq_json.py $OUT/sq_r03_c2.json "rocprofv3 --kernel-trace --pmc, 2 passes over bench.py --workload c2 --steps 3 --warmup 1" $(ls $OUT/sq_c2_*/*counter_collection.csv)
