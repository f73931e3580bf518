#!/bin/bash
# A/B of ONC_RPC_VARIANT bit sets on c1/c2/c3 bench lines (interleaved, 2 rounds).
set -u
mkdir -p gpurun_out/ab
VARS=${VARS:-"0 1 2 3"}
WLS=${WLS:-"c1 c2 c3"}
if [ -n "${TESTV:-}" ]; then
  ONC_RPC_VARIANT=$TESTV timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/ab/tests_v$TESTV.log 2>&1; rc=$?; echo "tests v$TESTV rc=$rc"; tail -2 gpurun_out/ab/tests_v$TESTV.log; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do for wl in $WLS; do for v in $VARS; do
  ONC_RPC_VARIANT=$v timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-pcie --c4-leg off > gpurun_out/ab/${wl}_v${v}_r$r.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], round(d['value'],1), round(d['ms_per_step']*1e3,1), {k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" gpurun_out/ab/${wl}_v${v}_r$r.log
done; done; done
