#!/bin/bash
# Framer: parity tests at several chunk sizes, then a chunk-size sweep on configs[2] (dev helper)
set -u
mkdir -p gpurun_out/fr
for ch in 64 4096 65536; do
  ONC_RPC_FRAME_CHUNK=$ch timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k frame --timeout 120 --timeout-method thread > gpurun_out/fr/tests_$ch.log 2>&1; rc=$?; echo "tests $ch rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for ch in ${CHUNKS:-4096 16384 32768 65536}; do
  ONC_RPC_FRAME_CHUNK=$ch timeout -k 10 300 python bench.py --workload c2 --frame --no-cpu-baseline --no-pcie > gpurun_out/fr/c2f_$ch.log 2>&1 || exit 1
done
