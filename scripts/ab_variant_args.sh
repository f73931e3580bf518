#!/bin/bash
# A/B of ONC_RPC_VARIANT bit sets over bench argument sets (interleaved, 2 rounds).
# VARS="0 0x200", CASES="name:args;name:args" (args with spaces), TESTV=bits to run the GPU suite first.
set -u
mkdir -p gpurun_out/ab
if [ -n "${TESTV:-}" ]; then
  ONC_RPC_VARIANT=$TESTV timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/ab/tests_v$TESTV.log 2>&1; rc=$?; echo "tests v$TESTV rc=$rc"; tail -2 gpurun_out/ab/tests_v$TESTV.log; [ $rc -eq 0 ] || exit $rc
fi
IFS=';' read -ra CS <<< "${CASES:-c1:--workload c1}"
for r in 1 2; do for cs in "${CS[@]}"; do for v in ${VARS:-0 0x200}; do
  name=${cs%%:*}; args=${cs#*:}
  ONC_RPC_VARIANT=$v timeout -k 10 200 python bench.py $args --no-cpu-baseline --no-pcie --c4-leg off > gpurun_out/ab/${name}_v${v}_r$r.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], round(d['value'],1), round(d['ms_per_step']*1e3,1), d['validated'], {k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" gpurun_out/ab/${name}_v${v}_r$r.log
done; done; done
