#!/bin/bash
# Build libonc_rpc_amd.so of a git revision into build/<name>/ (A/B runs:
# ONC_RPC_AMD_LIB=$PWD/build/<name>/libonc_rpc_amd.so python bench.py ...).
set -eu
rev=$1; name=$2
d=$(mktemp -d)
git archive "$rev" onc-rpc_amd/csrc include | tar -x -C "$d"
mkdir -p build/$name
make -s -C "$d/onc-rpc_amd/csrc" OUT=$PWD/build/$name/libonc_rpc_amd.so OBJDIR=$d/obj -j8
rm -rf "$d"
echo "built build/$name/libonc_rpc_amd.so from $rev"
