#!/bin/bash
# decode lab: the product decode with each lane pulling the first line of the
# record PF_DIST tiles ahead toward the caches (tools/dec_lab_pf<D>, built from
# a copy of decode.hip outside the tree) against the product (tools/dec_lab),
# clean cold (read scrub), configs[1]-shaped (W = 300) and configs[0]-shaped wires.
set -u
mkdir -p gpurun_out
for w in 300 192; do
  for b in dec_lab dec_lab_pf1024 dec_lab_pf4096; do
    env LAB_SCRUB=read $( [ $w = 192 ] && echo LAB_UNIX=1 ) timeout -k 10 200 ./tools/$b 1000000 $w > gpurun_out/pf_${b}_$w.log 2>&1 || exit $?
    echo "$b W=$w: $(grep product gpurun_out/pf_${b}_$w.log | tr -s ' ' | tr '\n' ';')"
  done
done
