#!/bin/bash
# Round 4, first GPU call: the GPU suite on the ABI-6 library, the C++
# mirror's single-message cost, c2 cold / warm, then the round-3 tree against
# HEAD on c0 / c1 / c3 (interleaved), and c0 with the re-planning emit.
set -u
mkdir -p gpurun_out
OUT=$PWD/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tests/cpp/test_mirror tests/golden/vectors.json > $OUT/cpp_mirror.log 2>&1; rc=$?
echo "cpp mirror rc=$rc"; grep TIMING $OUT/cpp_mirror.log; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1],round(d['value']),d['config'].get('cache'),round(d['roofline']['avg_launch_us'],1),{k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()},{k:(round(v['Mmsgs_per_s']),round(v['avg_launch_us'],1)) for k,v in (d.get('cache_legs') or {}).items()})" $1; }
timeout -k 10 240 python -u bench.py --workload c2 --c4-leg off --no-pcie --no-cpu-baseline > $OUT/bench_c2.log 2>&1; rc=$?
echo "bench c2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
summ $OUT/bench_c2.log
CASES="head:. r3:build/r3 headreplan:.:0x20000" ROUNDS=2 WLS="c0" bash scripts/ab_tree.sh || exit $?
CASES="head:. r3:build/r3" ROUNDS=2 WLS="c1 c3" bash scripts/ab_tree.sh
