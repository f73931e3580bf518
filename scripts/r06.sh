#!/bin/bash
# Round-6 GPU steps (one call runs several; every GPU step has its own
# timeout; the script stops at the first crash, abort or timeout):
#   first     the GPU suite, then (suite passed or only failed tests) the
#             look-back diagnosis and link labs
#   sqlds     LDS counters of one workload's kernels
#   8rank     the driver's 8-GPU command with 8 ranks on this one GPU
# (The producer/consumer decode A/B and its SQ passes — steps `ab` and
# `sqpc` with variant 0x80000 — ran against commit 283d487, which still had
# that lab kernel: profiles/lab_r06_decode_pc_ab.log, sq_r06_decode_pc.json.)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step=${1:-first}; shift || true
crash() { [ "$1" -gt 1 ] && [ "$1" -ne 3 ]; }     # pytest 1 = failed tests; bench 3 = not validated
case $step in
  first)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
      > gpurun_out/tests.log 2>&1; rc=$?
    grep -E "passed|failed|error" gpurun_out/tests.log | tail -3; echo "tests rc=$rc"
    crash $rc && exit $rc
    timeout -k 10 120 tools/lookback_diag > gpurun_out/lookback_diag.log 2>&1; r=$?; echo "diag rc=$r"; crash $r && exit $r
    timeout -k 10 180 tools/link_lab > gpurun_out/link_lab.log 2>&1; r=$?; echo "link rc=$r"; crash $r && exit $r
    exit $rc ;;
  sqlds)
    # LDS counters of the configs[0] encode: one --pmc pass, kernel trace only
    wl=${1:-c0}
    OUT=$PWD/gpurun_out
    P="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU"
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $P -d $OUT/sqlds_$wl -o run --output-format csv -- \
      python3 bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --c4-leg off --iov-leg off \
      --cache-leg off > $OUT/sqlds_$wl.log 2>&1; r=$?; echo "sqlds rc=$r"; [ $r -eq 0 ] || exit $r
    python3 scripts/sq_json.py $OUT/sqlds_$wl.json "rocprofv3 --kernel-trace --pmc (LDS pass) over bench.py --workload $wl --steps 3 --warmup 1" \
      $(ls $OUT/sqlds_$wl/*counter_collection.csv) | grep onc ;;
  8rank)
    # the driver's 8-GPU command rehearsed with 8 ranks on this one GPU (gloo control plane);
    # a heartbeat file shows progress while the ranks run
    (while sleep 45; do date +%T >> gpurun_out/heartbeat_8rank.log; done) & hb=$!
    s0=$(date +%s)
    ONC_BENCH_SAME_DEVICE=1 timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
      --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 8 --backend gloo \
      > gpurun_out/bench_8ranks_same_device.log 2>&1; r=$?
    kill $hb 2>/dev/null
    echo "8 ranks rc=$r wall_s=$(( $(date +%s) - s0 ))" | tee -a gpurun_out/bench_8ranks_same_device.log; exit $r ;;
esac
