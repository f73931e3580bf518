#!/bin/bash
# A/B bench of library variants under build/<name>/ (dev helper): VARIANTS="a b", WL=c1
set -u
mkdir -p gpurun_out/ab
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do for v in ${VARIANTS}; do
  ONC_RPC_AMD_LIB=$PWD/build/$v/libonc_rpc_amd.so timeout -k 10 200 python bench.py --workload ${WL:-c1} --no-cpu-baseline --no-pcie > gpurun_out/ab/${v}_${WL:-c1}_$r.log 2>&1 || exit 1
done; done
