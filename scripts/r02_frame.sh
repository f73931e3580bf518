#!/bin/bash
# Framer A/B: frame tests, then c2 --frame per CFGS entry
# name:ONC_RPC_VARIANT:ONC_RPC_FRAME_CHUNK[:library path].
set -u
O=gpurun_out/frame; mkdir -p $O
[ "${TESTS:-1}" = "1" ] && { timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k frame -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc; }
for r in 1 2; do for cfg in ${CFGS:-cur:0:65536 c32:0:32768}; do
  IFS=: read name var ch lib <<< "$cfg"
  ONC_RPC_AMD_LIB=$PWD/${lib:-onc-rpc_amd/libonc_rpc_amd.so} ONC_RPC_VARIANT=$var ONC_RPC_FRAME_CHUNK=$ch timeout -k 10 200 python bench.py --workload c2 --frame --c4-leg off --no-cpu-baseline --no-pcie > $O/c2f_${name}_r$r.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], round(d['value'],1), round(d['ms_per_step']*1e3,1), d['validated'], {k.replace('_kernel','').replace('frame_',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" $O/c2f_${name}_r$r.log
done; done
