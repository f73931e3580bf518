#!/bin/bash
# FETCH_SIZE / EA read-request-size calibration on dec_lab's known access patterns
# (1 pass per counter group, --kernel-trace only).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=$PWD/gpurun_out
i=0
for grp in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_DRAM_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp -d $OUT/cal_$i -o run --output-format csv -- ./tools/dec_lab 1000000 300 > $OUT/cal_$i.log 2>&1
  rc=$?; echo "cal group $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
