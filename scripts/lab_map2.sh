#!/bin/bash
# exact chunk map (ONC_GSH_MIN=0, 2048 entries) vs HEAD, after the consumer VALU trims.
set -u
mkdir -p gpurun_out/ab
for r in 1 2 3; do for wl in c1 c0 c1_8m; do for lv in "prev:build/prevh/libonc_rpc_amd.so" "map2k:build/map2k/libonc_rpc_amd.so"; do
  name=${lv%%:*}; lib=${lv#*:}
  extra=""; w=$wl; if [ "$wl" = "c1_8m" ]; then w=c1; extra="--records 8000000 --steps 10 --warmup 2"; fi
  ONC_RPC_AMD_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload $w $extra --no-cpu-baseline --no-pcie --c4-leg off --iov-leg off > gpurun_out/ab/${wl}_${name}_r$r.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], round(d['value'],1), round(d['ms_per_step']*1e3,1), d['validated'], {k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" gpurun_out/ab/${wl}_${name}_r$r.log
done; done; done
