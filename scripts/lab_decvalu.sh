#!/bin/bash
# decode VALU sensitivity: +256 / +512 VALU per wave (lab pad) vs product, c1 and c2.
set -u
mkdir -p gpurun_out/ab
for r in 1 2; do for wl in c1 c2; do for lv in "prev:build/prev/libonc_rpc_amd.so" "pad256:build/pad256/libonc_rpc_amd.so" "pad512:build/pad512/libonc_rpc_amd.so"; do
  name=${lv%%:*}; lib=${lv#*:}
  ONC_RPC_AMD_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-pcie --c4-leg off --iov-leg off > gpurun_out/ab/${wl}_${name}_r$r.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], round(d['value'],1), round(d['ms_per_step']*1e3,1), {k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" gpurun_out/ab/${wl}_${name}_r$r.log
done; done; done
