#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate rocprofv3 runs, --kernel-trace only)
# over short bench runs of each workload; writes gpurun_out/traffic_<wl>.json.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=$PWD/gpurun_out
for wl in ${WORKLOADS:-c1 c2 c3 c0}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d $OUT/pmc_${wl}_$ctr -o run --output-format csv -- \
        python3 bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --c4-leg off > $OUT/pmc_${wl}_$ctr.log 2>&1
    rc=$?; echo "pmc $wl $ctr rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
  n=$(python3 -c "import json;print([json.loads(l) for l in open('$OUT/pmc_${wl}_FETCH_SIZE.log') if l.startswith('{')][-1]['config']['records_per_gpu'])")
  python3 scripts/traffic_json.py $(ls $OUT/pmc_${wl}_FETCH_SIZE/*counter_collection.csv) \
      $(ls $OUT/pmc_${wl}_WRITE_SIZE/*counter_collection.csv) $OUT/traffic_$wl.json $n $wl
  echo "traffic $wl rc=$?"
done
