#!/bin/bash
# Round 4, first GPU call: the GPU suite on the ABI-6 library, then the
# round-2 tree against HEAD on c1 (interleaved), then c2 cold / warm.
set -u
mkdir -p gpurun_out
OUT=$PWD/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u bench.py --workload c2 --c4-leg off --no-pcie --no-cpu-baseline > $OUT/bench_c2.log 2>&1; rc=$?
echo "bench c2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.loads(open('$OUT/bench_c2.log').read().strip().splitlines()[-1]);print(round(d['value']),d['config']['cache'],round(d['roofline']['avg_launch_us'],1),{k:(round(v['Mmsgs_per_s']),round(v['avg_launch_us'],1)) for k,v in d['cache_legs'].items()})"
CASES="head:. r2:build/r2 headnohh:.:0x10000" ROUNDS=3 WLS=c1 bash scripts/ab_tree.sh
