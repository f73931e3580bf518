#!/bin/bash
# Round-5 GPU runs, one script with a step argument (replaces the one-off
# per-experiment launchers of rounds 3-4; those are in the history):
#   tests [FILES]  the GPU suite (or the given test files), -x, thread timeouts
#   smoke          __graft_entry__.smoke()
#   line WL [ARGS] one bench line, gpurun_out/b_<WL><TAG>.log (TAG env)
#   default        the driver's bench command (python bench.py)
#   stats [ARGS]   rocprofv3 --kernel-trace --stats of a short headline run
# Every GPU step runs under its own timeout; the script stops at the first failure.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step=${1:-tests}; shift || true
case $step in
  tests)
    files=${*:-tests}
    timeout -k 10 900 python -u -m pytest $files -m gpu -x -v --timeout 200 --timeout-method thread \
      > gpurun_out/tests.log 2>&1; rc=$?
    grep -E "passed|failed|error" gpurun_out/tests.log | tail -3; exit $rc ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
    cat gpurun_out/smoke.log | tail -3; exit $rc ;;
  line)
    wl=$1; shift
    log=gpurun_out/b_${wl}${TAG:-}.log
    timeout -k 10 600 python -u bench.py --workload $wl --c4-leg off "$@" > $log 2>&1; rc=$?
    python3 scripts/summ.py $log || true; exit $rc ;;
  default)
    timeout -k 10 900 python -u bench.py > gpurun_out/b_default.log 2>&1; rc=$?
    python3 scripts/summ.py gpurun_out/b_default.log || true; exit $rc ;;
  stats)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/stats -o run --output-format csv -- \
      python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --iov-leg off --cache-leg off "$@" \
      > gpurun_out/stats.log 2>&1; rc=$?
    find gpurun_out/stats -name "*kernel_stats.csv" | head -3; exit $rc ;;
  *) echo "unknown step $step"; exit 2 ;;
esac
