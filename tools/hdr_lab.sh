#!/bin/bash
# Lab builds of the codec library for the configs[0] enc_emit attribution
# (VERDICT r05 item 6): -DONC_LAB_HDR=1 (no header build), =2 (header
# words computed, not written to the LDS image), =3 (no credential-block load). Their output bytes are
# wrong by construction; they are timed only (scripts/ab.sh LAB=1).
set -e
cd "$(dirname "$0")/../onc-rpc_amd/csrc"
for v in 1 2 3; do
  make -s -j8 OBJDIR=../../tools/lab_hdr$v/obj OUT=../../tools/lab_hdr$v/libonc_rpc_amd.so \
    HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -DONC_LAB_HDR=$v"
done
