#!/bin/bash
# full-interior stream path (variant 0) vs the interior path (0x8000): GPU suite, then c1 / c3.
set -u
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ab/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for wl in c1 c3; do for v in 0 0x8000; do
  ONC_RPC_VARIANT=$v timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-pcie --c4-leg off --iov-leg off > gpurun_out/ab/${wl}_v${v}_r$r.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], round(d['value'],1), round(d['ms_per_step']*1e3,1), d['validated'], {k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" gpurun_out/ab/${wl}_v${v}_r$r.log
done; done; done
