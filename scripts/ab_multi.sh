#!/bin/bash
# A/B over (library, ONC_RPC_VARIANT) configurations and bench argument sets
# (interleaved, 2 rounds). CFGS="name|lib|variant ...", CASES="name:args;...",
# TESTCFG="lib|variant" to run the GPU suite with that configuration first.
set -u
mkdir -p gpurun_out/ab
if [ -n "${TESTCFG:-}" ]; then
  IFS='|' read tlib tvar <<< "$TESTCFG"
  ONC_RPC_AMD_LIB=$PWD/$tlib ONC_RPC_VARIANT=$tvar timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/ab/tests_cfg.log 2>&1; rc=$?; echo "tests $TESTCFG rc=$rc"; tail -2 gpurun_out/ab/tests_cfg.log; [ $rc -eq 0 ] || exit $rc
fi
IFS=';' read -ra CS <<< "${CASES:-c1:--workload c1}"
for r in 1 2; do for cs in "${CS[@]}"; do for cfg in ${CFGS}; do
  IFS='|' read name lib var <<< "$cfg"
  cname=${cs%%:*}; args=${cs#*:}
  ONC_RPC_AMD_LIB=$PWD/$lib ONC_RPC_VARIANT=$var timeout -k 10 200 python bench.py $args --no-cpu-baseline --no-pcie --c4-leg off > gpurun_out/ab/${cname}_${name}_r$r.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], round(d['value'],1), round(d['ms_per_step']*1e3,1), d['validated'], {k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" gpurun_out/ab/${cname}_${name}_r$r.log
done; done; done
