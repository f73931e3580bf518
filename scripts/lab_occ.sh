#!/bin/bash
# wave-per-tile enc_emit register budget A/B: product (106 VGPRs, 4 waves/SIMD) vs ONC_EMIT_OCC=5 (96 VGPRs + spill, 5).
set -u
mkdir -p gpurun_out/ab
for r in 1 2; do for wv in "c0:0" "c1:0x400" "c1_8m:0"; do for lv in "prod:build/prod/libonc_rpc_amd.so" "occ5:build/occ5/libonc_rpc_amd.so"; do
  wl=${wv%%:*}; v=${wv#*:}; name=${lv%%:*}; lib=${lv#*:}
  extra=""; w=$wl; if [ "$wl" = "c1_8m" ]; then w=c1; extra="--records 8000000 --steps 10 --warmup 2 --iov-leg off"; fi
  ONC_RPC_VARIANT=$v ONC_RPC_AMD_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload $w $extra --no-cpu-baseline --no-pcie --c4-leg off --iov-leg off > gpurun_out/ab/${wl}_${name}_r$r.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], round(d['value'],1), round(d['ms_per_step']*1e3,1), {k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" gpurun_out/ab/${wl}_${name}_r$r.log
done; done; done
