#!/bin/bash
# Round-4 evidence: GPU suite, smoke, the driver's default bench line, every workload, the rocprofv3 kernel
# stats of the headline command and of configs[4], and FETCH_SIZE / WRITE_SIZE traffic per workload.
# Every GPU step time-limited; a failure stops the script.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=$PWD/gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python -u bench.py > $OUT/bench_default.log 2>&1; rc=$?; echo "bench default rc=$rc"; [ $rc -eq 0 ] || exit $rc
for wl in c2 c3 c0 c4; do
  timeout -k 10 400 python -u bench.py --workload $wl --c4-leg off > $OUT/bench_$wl.log 2>&1; rc=$?; echo "bench $wl rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python -u bench.py --workload c2 --frame --c4-leg off > $OUT/bench_c2f.log 2>&1; rc=$?; echo "bench c2f rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --iov --c4-leg off > $OUT/bench_iov.log 2>&1; rc=$?; echo "bench iov rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c1 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --c4-leg off --iov-leg off --cache-leg off > $OUT/prof_c1.log 2>&1; rc=$?; echo "rocprof c1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c4 -o run --output-format csv -- python3 bench.py --workload c4 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof_c4.log 2>&1; rc=$?; echo "rocprof c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
for wl in ${WORKLOADS:-c1 c2 c3 c0 c4}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $ctr -d $OUT/pmc_${wl}_$ctr -o run --output-format csv -- \
        python3 bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --c4-leg off --iov-leg off --cache-leg off > $OUT/pmc_${wl}_$ctr.log 2>&1
    rc=$?; echo "pmc $wl $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  n=$(python3 -c "import json;d=[json.loads(l) for l in open('$OUT/pmc_${wl}_FETCH_SIZE.log') if l.startswith('{')][-1];print(d['config'].get('records_per_gpu', d['config'].get('records_total')))")
  python3 scripts/traffic_json.py $(ls $OUT/pmc_${wl}_FETCH_SIZE/*counter_collection.csv) \
      $(ls $OUT/pmc_${wl}_WRITE_SIZE/*counter_collection.csv) $OUT/traffic_$wl.json $n $wl
  echo "traffic $wl rc=$?"
done
timeout -k 10 120 tests/cpp/test_mirror tests/golden/vectors.json > $OUT/cpp_mirror.log 2>&1; echo "cpp mirror rc=$?"
if [ -n "${AB:-}" ]; then CASES="head:. r3:build/r3 r2:build/r2" ROUNDS=3 WLS="c1" bash scripts/ab_tree.sh; fi
