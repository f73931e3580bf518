#!/bin/bash
# Round 4, first GPU call: the GPU suite on the ABI-6 library, the C++
# mirror's single-message cost, c2 cold / warm, c0, then the round-2 tree
# against HEAD on c1 (interleaved).
set -u
mkdir -p gpurun_out
OUT=$PWD/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tests/cpp/test_mirror tests/golden/vectors.json > $OUT/cpp_mirror.log 2>&1; rc=$?
echo "cpp mirror rc=$rc"; grep TIMING $OUT/cpp_mirror.log; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1],round(d['value']),d['config'].get('cache'),round(d['roofline']['avg_launch_us'],1),{k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()},{k:(round(v['Mmsgs_per_s']),round(v['avg_launch_us'],1)) for k,v in (d.get('cache_legs') or {}).items()})" $1; }
for wl in c2 c0; do
  timeout -k 10 240 python -u bench.py --workload $wl --c4-leg off --no-pcie --no-cpu-baseline > $OUT/bench_$wl.log 2>&1; rc=$?
  echo "bench $wl rc=$rc"; [ $rc -eq 0 ] || exit $rc
  summ $OUT/bench_$wl.log
done
CASES="head:. r2:build/r2 headnohh:.:0x10000" ROUNDS=3 WLS=c1 bash scripts/ab_tree.sh
