#!/bin/bash
# Decode component lab on configs[2]: the product library against lab builds
# (-DONC_DEC_LAB=1 no AUTH_UNIX slot stores, =2 records assumed 4-byte
# aligned, =3 no parse) — interleaved, 2 rounds — then tools/line_lab.py.
# A lab build's bench fails its own validation (exit 3); anything else stops.
set -u
mkdir -p gpurun_out/declab
for r in 1 2; do for lv in base:onc-rpc_amd/libonc_rpc_amd.so ${LABS:-l1:build/lab1/libonc_rpc_amd.so l2:build/lab2/libonc_rpc_amd.so l3:build/lab3/libonc_rpc_amd.so}; do
  name=${lv%%:*}; lib=${lv#*:}
  log=gpurun_out/declab/${WL:-c2}_${name}_r$r.log
  ONC_RPC_AMD_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload ${WL:-c2} --no-cpu-baseline --no-pcie --c4-leg off > $log 2>&1
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { echo "$name rc=$rc"; tail -5 $log; exit $rc; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], round(d['value'],1), round(d['ms_per_step']*1e3,1), {k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" $log
done; done
if [ "${LINE:-1}" = "1" ]; then
  timeout -k 10 240 python -u tools/line_lab.py 1000000 20 > gpurun_out/declab/line_lab.log 2>&1; rc=$?; cat gpurun_out/declab/line_lab.log; exit $rc
fi
