#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only;
# no sys/runtime tracing) over a short bench run. Outputs gpurun_out/pmc_*.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=$PWD/gpurun_out
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
for grp in "${@}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d $OUT/pmc_$i -o run --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/pmc_$i.log 2>&1
  rc=$?; echo "pmc group $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
