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
  sq)
    # SQ instruction / wait counters, two --pmc passes (kernel trace only) -> gpurun_out/sq_<WL>.json
    wl=$1; shift
    OUT=$PWD/gpurun_out
    P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY"
    P2="SQ_WAVES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS"
    i=0
    for grp in "$P1" "$P2"; do
      i=$((i+1))
      timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp -d $OUT/sq_${wl}_$i -o run --output-format csv -- \
        python3 bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --c4-leg off --iov-leg off \
        --cache-leg off "$@" > $OUT/sq_${wl}_$i.log 2>&1
      rc=$?; echo "sq $wl pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
    python3 scripts/sq_json.py $OUT/sq_$wl.json "rocprofv3 --kernel-trace --pmc, 2 passes over bench.py --workload $wl --steps 3 --warmup 1 $*" \
      $(ls $OUT/sq_${wl}_1/*counter_collection.csv) $(ls $OUT/sq_${wl}_2/*counter_collection.csv) | grep onc ;;
  round|benches|profs)
    # the round's evidence: default line, every workload (benches), rocprof stats of c1 and c4,
    # FETCH/WRITE traffic (profs); round = both
    OUT=$PWD/gpurun_out
    if [ $step != profs ]; then
    timeout -k 10 600 python -u bench.py > $OUT/bench_default.log 2>&1; rc=$?; echo "bench default rc=$rc"; [ $rc -eq 0 ] || exit $rc
    for wl in c2 c3 c0 c4; do
      timeout -k 10 600 python -u bench.py --workload $wl --c4-leg off > $OUT/bench_$wl.log 2>&1; rc=$?; echo "bench $wl rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
    timeout -k 10 400 python -u bench.py --workload c2 --frame --c4-leg off > $OUT/bench_c2f.log 2>&1; rc=$?; echo "bench c2f rc=$rc"; [ $rc -eq 0 ] || exit $rc
    for wl in c1 c3 c0; do
      timeout -k 10 400 python -u bench.py --workload $wl --iov --c4-leg off > $OUT/bench_iov_$wl.log 2>&1; rc=$?; echo "bench iov $wl rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
    fi
    [ $step = benches ] && exit 0
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c1 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --c4-leg off --iov-leg off --cache-leg off > $OUT/prof_c1.log 2>&1; rc=$?; echo "rocprof c1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c4 -o run --output-format csv -- python3 bench.py --workload c4 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof_c4.log 2>&1; rc=$?; echo "rocprof c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
    for wl in ${WORKLOADS:-c1 c2 c3 c0 c4}; do
      for ctr in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $ctr -d $OUT/pmc_${wl}_$ctr -o run --output-format csv -- \
            python3 bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --c4-leg off --iov-leg off --cache-leg off > $OUT/pmc_${wl}_$ctr.log 2>&1
        rc=$?; echo "pmc $wl $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
      done
      n=$(python3 -c "import json;d=[json.loads(l) for l in open('$OUT/pmc_${wl}_FETCH_SIZE.log') if l.startswith('{')][-1];print(d['config'].get('records_per_gpu', d['config'].get('records_total')))")
      python3 scripts/traffic_json.py $(ls $OUT/pmc_${wl}_FETCH_SIZE/*counter_collection.csv) \
          $(ls $OUT/pmc_${wl}_WRITE_SIZE/*counter_collection.csv) $OUT/traffic_$wl.json $n $wl
      echo "traffic $wl rc=$?"
    done ;;
  *) echo "unknown step $step"; exit 2 ;;
esac
