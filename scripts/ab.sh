#!/bin/bash
# A/B of library builds and kernel-variant bits (bench.py --variant) (interleaved, ROUNDS rounds, default 2):
# CASES="name:lib[:variant] ...", WLS="c0 c1 ...", BARGS extra bench args, TESTS=1 runs the GPU suite on the in-tree library first,
# LAB=1: lab builds whose output is knowingly wrong (bench exit 3, not validated) are timed, not stopped at.
set -u
mkdir -p gpurun_out/ab
if [ "${TESTS:-0}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ab/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 ${ROUNDS:-2}); do for wl in ${WLS:-c0 c1}; do for cs in ${CASES}; do
  IFS=: read -r name lib var <<< "$cs"
  ONC_RPC_AMD_LIB=$PWD/$lib timeout -k 10 200 python bench.py --variant ${var:-0} --workload $wl --no-cpu-baseline --no-pcie --c4-leg off --iov-leg off ${BARGS:-} > gpurun_out/ab/${wl}_${name}_r$r.log 2>&1 || { rc=$?; [ $rc -eq 3 ] && [ "${LAB:-0}" = 1 ] || exit $rc; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], round(d['value'],1), round(d['ms_per_step']*1e3,1), round(d['ms_per_step_without_kernel_events']*1e3,1), 'dom', round(d['roofline']['avg_launch_us'],1), {k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" gpurun_out/ab/${wl}_${name}_r$r.log
done; done; done
