#!/bin/bash
# full-interior path on the wave-per-tile enc_emit: GPU suite, then on (0) / off (0x8000) on c0, c1 at 8M, c1 forced onto wave-per-tile (0x400 / 0x8400).
set -u
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ab/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for wv in "c1_8m:0" "c1_8m:0x8000" "c0:0" "c0:0x8000" "c1:0x400" "c1:0x8400"; do
  wl=${wv%%:*}; v=${wv#*:}
  extra=""; w=$wl; if [ "$wl" = "c1_8m" ]; then w=c1; extra="--records 8000000 --steps 10 --warmup 2"; fi
  ONC_RPC_VARIANT=$v timeout -k 10 200 python bench.py --workload $w $extra --no-cpu-baseline --no-pcie --c4-leg off --iov-leg off > gpurun_out/ab/${wl}_v${v}_r$r.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], round(d['value'],1), round(d['ms_per_step']*1e3,1), d['validated'], {k.replace('_kernel',''):round(v['avg_us'],1) for k,v in d['kernels_breakdown_pass'].items()})" gpurun_out/ab/${wl}_v${v}_r$r.log
done; done
