#!/bin/bash
# GPU suite on the working tree, then HEAD's library (build/prevh) vs the working tree on $WLS.
set -u
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ab/tests.log; [ $rc -eq 0 ] || exit $rc
for r in ${ROUNDS:-1 2}; do for wl in ${WLS:-c1 c3 c0}; do for lv in "prev:build/prevh/libonc_rpc_amd.so" "new:onc-rpc_amd/libonc_rpc_amd.so"; do
  name=${lv%%:*}; lib=${lv#*:}
  extra=""; w=$wl; if [ "$wl" = "c1_8m" ]; then w=c1; extra="--records 8000000 --steps 10 --warmup 2"; fi
  ONC_RPC_AMD_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload $w $extra --no-cpu-baseline --no-pcie --c4-leg off --iov-leg off > gpurun_out/ab/${wl}_${name}_r$r.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], round(d['value'],1), round(d['ms_per_step']*1e3,1), d['validated'], {k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" gpurun_out/ab/${wl}_${name}_r$r.log
done; done; done
