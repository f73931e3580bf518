#!/bin/bash
# wave-specialised (forced, variant 0x200) vs the default wave-per-tile enc_emit at 8M and 16M records (configs[4] shards).
set -u
mkdir -p gpurun_out/ab
for r in 1 2; do for n in 8000000 16000000; do for v in 0 0x200; do
  ONC_RPC_VARIANT=$v timeout -k 10 300 python bench.py --workload c1 --records $n --steps 6 --warmup 2 --no-cpu-baseline --no-pcie --c4-leg off --iov-leg off > gpurun_out/ab/c1_${n}_v${v}_r$r.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], round(d['value'],1), round(d['ms_per_step']*1e3,1), d['validated'], {k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" gpurun_out/ab/c1_${n}_v${v}_r$r.log
done; done; done
