#!/bin/bash
# Round-2 evidence, part B: rocprofv3 kernel stats of the headline and the
# configs[4] commands, FETCH_SIZE / WRITE_SIZE passes per workload
# (one counter per pass, --kernel-trace only).
set -u
export TMPDIR=/tmp
O=$PWD/gpurun_out/r02
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c1 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --c4-leg off > $O/prof_c1.log 2>&1; rc=$?; echo "rocprof c1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run --output-format csv -- python3 bench.py --workload c4 --steps 5 --warmup 2 > $O/prof_c4.log 2>&1; rc=$?; echo "rocprof c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
for wl in c1 c2 c3 c0 c4; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $ctr -d $O/pmc_${wl}_$ctr -o run --output-format csv -- \
        python3 bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --c4-leg off > $O/pmc_${wl}_$ctr.log 2>&1
    rc=$?; echo "pmc $wl $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  n=$(python3 -c "import json;print([json.loads(l) for l in open('$O/pmc_${wl}_FETCH_SIZE.log') if l.startswith('{')][-1]['config']['records_per_gpu'])")
  python3 scripts/traffic_json.py $(ls $O/pmc_${wl}_FETCH_SIZE/*counter_collection.csv) \
      $(ls $O/pmc_${wl}_WRITE_SIZE/*counter_collection.csv) $O/traffic_$wl.json $n $wl
  echo "traffic $wl rc=$?"
done
