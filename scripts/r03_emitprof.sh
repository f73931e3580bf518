#!/bin/bash
# enc_emit phase profile (tools/emit_prof, built with -DONC_EMIT_PROF) on the configs[0] / configs[1] / configs[3] shapes.
set -u
mkdir -p gpurun_out
for shape in ${SHAPES:-c0 c1}; do
  timeout -k 10 120 tools/emit_prof 1000000 $shape ${EXTRA:-} > gpurun_out/emitprof_$shape.log 2>&1; rc=$?; echo "emit_prof $shape rc=$rc"; tail -9 gpurun_out/emitprof_$shape.log; [ $rc -eq 0 ] || exit $rc
done
