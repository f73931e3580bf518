#!/bin/bash
# A/B of two library builds (interleaved, 2 rounds) after the GPU tests of the new one.
# LIBS="name:path name:path", WLS="c1 c3 ...", TESTS=1 to run the GPU suite first.
set -u
mkdir -p gpurun_out/ab
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ab/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do for wl in ${WLS:-c1 c3}; do for lv in ${LIBS}; do
  name=${lv%%:*}; lib=${lv#*:}
  ONC_RPC_AMD_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-pcie --c4-leg off ${BARGS:-} > gpurun_out/ab/${wl}_${name}_r$r.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], round(d['value'],1), round(d['ms_per_step']*1e3,1), round(d['ms_per_step_without_kernel_events']*1e3,1), 'dom', round(d['roofline']['avg_launch_us'],1), {k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" gpurun_out/ab/${wl}_${name}_r$r.log
done; done; done
