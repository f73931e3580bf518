#!/bin/bash
# PCIe-inclusive legs (serialised and pipelined) per workload and chunk count; no CPU baseline, no configs[4] leg.
set -u
mkdir -p gpurun_out/pcie
for wl in ${WLS:-c1 c2}; do for k in ${CHUNKS:-8 16}; do
  timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --c4-leg off --iov-leg off --pcie-chunks $k --pcie-reps ${REPS:-5} > gpurun_out/pcie/${wl}_k$k.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);p=d['pcie_inclusive'];q=p['pipelined'];print(sys.argv[1].split('/')[-1], 'serial', round(p['value'],1), 'pipelined', round(q['value'],1), round(q['pcie_GBs_per_gpu'],1), 'GB/s', q['validated'])" gpurun_out/pcie/${wl}_k$k.log
done; done
