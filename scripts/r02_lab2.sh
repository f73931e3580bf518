#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 120 ./tools/dec_lab 1000000 300 > gpurun_out/declab2_300_cold.log 2>&1 || exit $?
LAB_WARM=1 timeout -k 10 120 ./tools/dec_lab 1000000 300 > gpurun_out/declab2_300_warm.log 2>&1 || exit $?
cat gpurun_out/declab2_*.log
for ov in "" "--overlap"; do for wl in c1 c3; do
  timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-pcie --c4-leg off $ov > gpurun_out/ov_${wl}_${ov:-none}.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1], round(d['value'],1), round(d['ms_per_step']*1e3,1), {k:round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" gpurun_out/ov_${wl}_${ov:-none}.log
done; done
