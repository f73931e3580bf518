#!/bin/bash
# Decode first-round policy A/B in HBM (bench.py --decode-policy), after the
# cooperative round 1: interleaved rounds, per-kernel times of each workload.
set -u
mkdir -p gpurun_out/pol
for r in $(seq 1 ${ROUNDS:-2}); do for wl in ${WLS:-c2 c0 c1 c3}; do for pol in standard line auto; do
  timeout -k 10 200 python bench.py --decode-policy $pol --workload $wl --no-cpu-baseline --no-pcie --c4-leg off \
    --iov-leg off > gpurun_out/pol/${wl}_${pol}_r$r.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], round(d['value'],1), {k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" gpurun_out/pol/${wl}_${pol}_r$r.log
done; done; done
