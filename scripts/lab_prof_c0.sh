set -u
mkdir -p gpurun_out
timeout -k 10 120 ./tools/emit_prof 1000000 c0 > gpurun_out/prof_c0_wpt.log 2>&1 || exit $?
timeout -k 10 120 ./tools/emit_prof 1000000 c0 ws > gpurun_out/prof_c0_ws.log 2>&1 || exit $?
timeout -k 10 120 ./tools/emit_prof 1000000 > gpurun_out/prof_c1_wpt.log 2>&1 || exit $?
