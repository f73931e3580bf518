#!/bin/bash
# A/B of whole source trees (each with its own bench.py and built library),
# interleaved, ROUNDS rounds (default 3): CASES="name:dir[:variant] ...",
# WLS="c1 ...", BARGS extra bench args. An older round's tree is extracted with
# `git archive <rev> | tar -x -C build/<name>` and built in place.
set -u
mkdir -p gpurun_out/ab
top=$PWD
for r in $(seq 1 ${ROUNDS:-3}); do for wl in ${WLS:-c1}; do for cs in ${CASES}; do
  IFS=: read -r name dir var <<< "$cs"
  log=$top/gpurun_out/ab/${wl}_${name}_r$r.log
  (cd $dir && ONC_RPC_VARIANT=${var:-0} timeout -k 10 200 python bench.py $([ -n "${var:-}" ] && [ -f $dir/include/onc_rpc.h ] && grep -q create_ex $dir/include/onc_rpc.h && echo --variant $var) --workload $wl --no-cpu-baseline --no-pcie \
     --c4-leg off --iov-leg off ${BARGS:-} > $log 2>&1) || exit $?
  python3 scripts/summ.py $log
done; done; done
