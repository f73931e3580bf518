#!/bin/bash
# Build the working tree's library with extra compile flags into build/<name>/
# (A/B runs: ONC_RPC_AMD_LIB=$PWD/build/<name>/libonc_rpc_amd.so ...).
# usage: scripts/build_variant_lib.sh <name> "-DFOO=1 -DBAR"
set -eu
name=$1; flags=$2
d=$(mktemp -d)
mkdir -p "$d/onc-rpc_amd" build/$name
cp -r onc-rpc_amd/csrc "$d/onc-rpc_amd/"; cp -r include "$d/"
rm -rf "$d/onc-rpc_amd/csrc/"*.o
make -s -C "$d/onc-rpc_amd/csrc" OUT=$PWD/build/$name/libonc_rpc_amd.so OBJDIR=$d/obj \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $flags" -j8
rm -rf "$d"
echo "built build/$name/libonc_rpc_amd.so ($flags)"
