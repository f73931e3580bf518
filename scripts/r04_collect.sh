#!/bin/bash
# Copies the evidence scripts/r04_round.sh left under gpurun_out/ into profiles/ (round-4 names).
set -eu
O=gpurun_out; P=profiles
cp $O/gpu_tests.log $P/r04_gpu_tests.log
cp $O/smoke.log $P/r04_smoke.log
for w in default c2 c3 c0 c4 c2f iov; do cp $O/bench_$w.log $P/bench_r04_$w.log; done
cp $O/prof_c1/run_kernel_stats.csv $P/r04_kernel_stats_c1.csv
cp $O/prof_c4/run_kernel_stats.csv $P/r04_kernel_stats_c4.csv
cp $O/traffic_c1.json $P/traffic_r04.json
for w in c0 c2 c3 c4; do cp $O/traffic_$w.json $P/traffic_r04_$w.json; done
cp $O/cpp_mirror.log $P/r04_cpp_mirror.log 2>/dev/null || true
