#!/bin/bash
# PMC passes over the emit lab (one counter group per rocprofv3 run, --kernel-trace only).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=$PWD/gpurun_out
BIN=${LAB_BIN:-./tools/emit_lab}
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
for grp in "${@}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/pmclab_$i -o run --output-format csv -- $BIN > $OUT/pmclab_$i.log 2>&1
  rc=$?; echo "pmc group $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
