#!/bin/bash
# HEAD / round-3 / round-2 trees on c1 (3 interleaved rounds), HEAD / round-3 on c4 (2 rounds), the cold lab.
set -u
mkdir -p gpurun_out
CASES="head:. r3:build/r3 r2:build/r2" ROUNDS=3 WLS="c1" bash scripts/ab_tree.sh || exit $?
CASES="head:. r3:build/r3" ROUNDS=2 WLS="c4" bash scripts/ab_tree.sh || exit $?
timeout -k 10 300 python -u tools/cold_lab.py 1000000 20 > gpurun_out/lab_cold.log 2>&1; rc=$?
echo "cold rc=$rc"; grep -v amdgpu.ids gpurun_out/lab_cold.log; exit $rc
