#!/bin/bash
# Vectored-encode bench lines (bench.py --iov) for c1 / c3 / c0.
set -u
mkdir -p gpurun_out
for wl in ${WLS:-c1 c3 c0}; do
  timeout -k 10 300 python bench.py --workload $wl --iov --no-cpu-baseline --c4-leg off ${BARGS:-} > gpurun_out/iov_$wl.log 2>&1
  rc=$?; echo "iov $wl rc=$rc"
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print(sys.argv[1].split('/')[-1], round(d['value'],1), round(d['ms_per_step']*1e3,1), 'valid', d['validated'], r['kernel'], round(r['avg_launch_us'],1), 'frac', round(r['frac'],3), 'step_frac', round(r['step_frac'],3), {k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" gpurun_out/iov_$wl.log
  [ $rc -eq 0 ] || exit $rc
done
