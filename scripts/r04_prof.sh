#!/bin/bash
# enc_emit (wave-specialised) phase profile on configs[1], HEAD vs the round-2
# tree, same harness (tools/emit_prof.hip built against each tree's encode.hip
# with -DONC_EMIT_PROF), 3 interleaved rounds.
set -u
mkdir -p gpurun_out
for r in 1 2 3; do
  for t in head:. r2:build/r2; do
    IFS=: read -r name dir <<< "$t"
    echo "== $name r$r"
    (cd $dir && timeout -k 10 60 ./tools/emit_prof 1000000 c1 ws) || exit $?
  done
done
