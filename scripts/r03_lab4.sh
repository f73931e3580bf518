#!/bin/bash
# Round 3 lab 4: chunked encode beyond 1M records (default) vs the whole-batch plan (0x40000): GPU suite, then benches.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # name variant args...
  local name=$1 v=$2; shift 2
  ONC_RPC_VARIANT=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie --iov-leg off --steps 10 "$@" > gpurun_out/lab4_$name.log 2>&1; rc=$?
  echo -n "$name v=$v rc=$rc: "; python3 scripts/summ.py gpurun_out/lab4_$name.log; [ $rc -eq 0 ] || exit $rc
}
for rep in 1 2; do
run c1_8m_chunk 0 --workload c1 --records 8000000 --c4-leg off
run c1_8m_whole 0x40000 --workload c1 --records 8000000 --c4-leg off
run c3_chunk 0 --workload c3 --c4-leg off
run c3_whole 0x40000 --workload c3 --c4-leg off
done
run c4_chunk 0 --workload c4
run c4_whole 0x40000 --workload c4
