#!/bin/bash
# Round 3 lab 3: two waves per enc_emit tile (variant 0x20000) vs one, on c0, c1 (1M, forced wave-per-tile) and c1 at 8M.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_emit_paths.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests_paths.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests_paths.log; [ $rc -eq 0 ] || exit $rc
run() {  # name variant args...
  local name=$1 v=$2; shift 2
  ONC_RPC_VARIANT=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie --c4-leg off --iov-leg off --steps 10 "$@" > gpurun_out/lab3_$name.log 2>&1; rc=$?
  echo -n "$name v=$v rc=$rc: "; python3 scripts/summ.py gpurun_out/lab3_$name.log; [ $rc -eq 0 ] || exit $rc
}
for rep in 1 2; do
run c0_tile 0 --workload c0
run c0_split 0x20000 --workload c0
run c1_tile 0x400 --workload c1
run c1_split 0x20400 --workload c1
run c1_ws 0 --workload c1
run c1_8m_tile 0 --workload c1 --records 8000000
run c1_8m_split 0x20000 --workload c1 --records 8000000
done
