#!/bin/bash
# A/B of whole source trees (each with its own bench.py and built library),
# interleaved, ROUNDS rounds (default 3): CASES="name:dir[:variant] ...",
# WLS="c1 ...", BARGS extra bench args (for every tree). An older round's tree
# is extracted with `git archive <rev> | tar -x -C build/<name>` and built in
# place. Variant bits go through --variant where the tree's bench has it
# (ABI 6), else through the ONC_RPC_VARIANT environment variable (ABI <= 5);
# trees whose bench has --cache-leg run without the extra cache legs.
set -u
mkdir -p gpurun_out/ab
top=$PWD
for r in $(seq 1 ${ROUNDS:-3}); do for wl in ${WLS:-c1}; do for cs in ${CASES}; do
  IFS=: read -r name dir var <<< "$cs"
  log=$top/gpurun_out/ab/${wl}_${name}_r$r.log
  extra=""
  grep -q -- "--cache-leg" $dir/bench.py && extra="--cache-leg off"
  if grep -q -- '"--variant"' $dir/bench.py; then extra="$extra --variant ${var:-0}"; envv=""; else envv="ONC_RPC_VARIANT=${var:-0}"; fi
  (cd $dir && env $envv timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-pcie \
     --c4-leg off --iov-leg off $extra ${BARGS:-} > $log 2>&1) || exit $?
  python3 scripts/summ.py $log
done; done; done
