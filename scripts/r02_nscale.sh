#!/bin/bash
set -u
mkdir -p gpurun_out/ns
for n in 250000 500000 1000000 2000000 4000000 8000000; do
  timeout -k 10 200 python bench.py --records $n --no-cpu-baseline --no-pcie --c4-leg off > gpurun_out/ns/c1_$n.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], round(d['value'],1), round(d['ms_per_step']*1e3,1), round(d['ms_per_step_without_kernel_events']*1e3,1), {k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" gpurun_out/ns/c1_$n.log $n
done
