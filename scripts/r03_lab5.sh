#!/bin/bash
# Round 3 lab 5: chunk size of the chunked encode (ONC_RPC_ENC_CHUNK) and nontemporal payload loads (0x80000), c1 at 8M.
set -u
mkdir -p gpurun_out
run() {  # name variant chunk args...
  local name=$1 v=$2 ch=$3; shift 3
  ONC_RPC_ENC_CHUNK=$ch ONC_RPC_VARIANT=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie --iov-leg off --c4-leg off --steps 10 "$@" > gpurun_out/lab5_$name.log 2>&1; rc=$?
  echo -n "$name v=$v chunk=$ch rc=$rc: "; python3 scripts/summ.py gpurun_out/lab5_$name.log; [ $rc -eq 0 ] || exit $rc
}
for rep in 1 2; do
run c1_8m_512k 0 524288 --workload c1 --records 8000000
run c1_8m_1m 0 0 --workload c1 --records 8000000
run c1_8m_2m 0 2097152 --workload c1 --records 8000000
run c1_8m_1m_ntld 0x80000 0 --workload c1 --records 8000000
run c1_1m_ntld 0x80000 0 --workload c1
run c1_1m 0 0 --workload c1
done
