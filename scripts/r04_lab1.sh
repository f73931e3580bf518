#!/bin/bash
# Labs: the enc_emit choice on half/half batches (tools/mix_lab.py), and the
# decode writing aux words only for failing records (variant 0x100000) on
# c1 / c0 / c2, interleaved.
set -u
mkdir -p gpurun_out
OUT=$PWD/gpurun_out
timeout -k 10 300 python -u tools/mix_lab.py 1000000 20 > $OUT/lab_mix.log 2>&1; rc=$?
echo "mix rc=$rc"; cat $OUT/lab_mix.log | tail -3; [ $rc -eq 0 ] || exit $rc
CASES="head:. auxsparse:.:0x100000" ROUNDS=2 WLS="c1 c0 c2" bash scripts/ab_tree.sh
