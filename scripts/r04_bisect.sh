#!/bin/bash
# c1 enc_emit between the round-2 and round-3 trees: r2, d1444de, 90aac8d
# (ws header-heavy fallback + per-workgroup payload totals), 2279c92 (image
# swizzle), 73eec08, fb463a3 (edge chunks on the last consumer part), r3,
# HEAD, HEAD with the pipeline forced (no kernel-choice sampling); 3 rounds.
set -u
CASES="r2:build/r2 d14:build/b_d1444de a90:build/b_90aac8d s22:build/b_2279c92 p73:build/b_73eec08 fb4:build/b_fb463a3 r3:build/r3 head:. hp:.:65536" \
  ROUNDS=3 WLS="c1" bash scripts/ab_tree.sh
rc=$?; [ $rc = 0 ] || exit $rc
# decode ceilings cold after a memset scrub vs a read scrub (W = 300: configs[1])
timeout -k 10 200 ./tools/dec_lab 1000000 300 > gpurun_out/lab_dec_memset.log 2>&1 || exit $?
LAB_SCRUB=read timeout -k 10 200 ./tools/dec_lab 1000000 300 > gpurun_out/lab_dec_read.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/cold_lab.py 1000000 20 > gpurun_out/lab_cold.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/lab_dec_memset.log gpurun_out/lab_dec_read.log gpurun_out/lab_cold.log
