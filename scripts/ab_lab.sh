#!/bin/bash
# Lab A/B of library builds whose results may be invalid (bench exit 3 =
# validation failed is tolerated; any other failure stops the run).
# LIBS="name:path ...", WLS="c1 ...", BARGS=extra bench args.
set -u
mkdir -p gpurun_out/ab
for r in 1 2; do for wl in ${WLS:-c1}; do for lv in ${LIBS}; do
  name=${lv%%:*}; lib=${lv#*:}
  ONC_RPC_AMD_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-pcie --c4-leg off ${BARGS:-} > gpurun_out/ab/${wl}_${name}_r$r.log 2>&1; rc=$?
  [ $rc -eq 0 ] || [ $rc -eq 3 ] || { echo "$name rc=$rc"; exit $rc; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], round(d['value'],1), round(d['ms_per_step']*1e3,1), d['validated'], {k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" gpurun_out/ab/${wl}_${name}_r$r.log
done; done; done
