#!/bin/bash
# Round-6 A/B of the decode's window loads: the library against a lab build
# B="name:dir" (a libonc_rpc_amd.so built into dir with one switch of
# decode.hip turned off, e.g. -DONC_DEC_COOP2=0; the logs name each build):
# decode parity suites on the library first (unless ZC_ONLY=1), then
# HBM-resident steps (scripts/ab.sh) and the configs[2] zero-copy decode of a
# mapped wire with each library.
set -u
mkdir -p gpurun_out
B=${B:?set B=name:dir of the lab build}
[ "${ZC_ONLY:-0}" = 1 ] || {
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_decode_lengths.py tests/test_gpu_r04.py \
  tests/test_gpu_r05.py tests/test_body_roots.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/buf_tests.log 2>&1; r=$?; tail -2 gpurun_out/buf_tests.log; [ $r -eq 0 ] || exit $r
CASES="lib:onc-rpc_amd/libonc_rpc_amd.so:0 ${B%%:*}:${B#*:}/libonc_rpc_amd.so:0" WLS="c1 c2 c0 c3" ROUNDS=2 \
  bash scripts/ab.sh > gpurun_out/ab_buf.log 2>&1; r=$?; cat gpurun_out/ab_buf.log; [ $r -eq 0 ] || exit $r
}
for r in $(seq 1 ${ZC_ROUNDS:-2}); do for cs in lib:onc-rpc_amd $B; do
  IFS=: read -r name dir <<< "$cs"
  ONC_RPC_AMD_LIB=$PWD/$dir/libonc_rpc_amd.so timeout -k 10 300 python -u bench.py --workload c2 --c4-leg off \
    --no-cpu-baseline > gpurun_out/zc_${name}_r$r.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);z=d['pcie_inclusive']['zero_copy'];print(sys.argv[1].split('/')[-1], round(z['value'],1), round(z['ms_per_step'],3), {k:round(v['ms_per_step'],3) for k,v in z['variants'].items() if k.startswith('policy')})" gpurun_out/zc_${name}_r$r.log
done; done
