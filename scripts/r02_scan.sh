#!/bin/bash
set -u
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_r02.py -m gpu -x -q --timeout 200 --timeout-method thread -k scan_lengths > gpurun_out/gpu_tests_scan.log 2>&1; rc=$?; echo "pytest scan rc=$rc"; tail -3 gpurun_out/gpu_tests_scan.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for fs in 1 0; do
  ONC_RPC_FORCE_SCAN=$fs timeout -k 10 200 python bench.py --workload c2 --no-cpu-baseline --no-pcie --c4-leg off > gpurun_out/ab/c2_fs${fs}_r$r.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], round(d['value'],1), round(d['ms_per_step']*1e3,1), {k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" gpurun_out/ab/c2_fs${fs}_r$r.log
done; done
