#!/bin/bash
set -u
mkdir -p gpurun_out/ab
for r in 1 2; do for sh in 0 4 8 12; do
  timeout -k 10 200 python bench.py --workload c1 --no-cpu-baseline --no-pcie --c4-leg off --payload-shift $sh > gpurun_out/ab/c1_sh${sh}_r$r.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], round(d['value'],1), round(d['ms_per_step']*1e3,1), {k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" gpurun_out/ab/c1_sh${sh}_r$r.log
done; done
