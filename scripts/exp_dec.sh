set -u
mkdir -p gpurun_out/exp
for w in 4 6 10; do for wl in c1 c2 c3; do
  ONC_RPC_AMD_LIB=$PWD/build/w$w/libonc_rpc_amd.so timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-pcie --steps 20 > gpurun_out/exp/w${w}_$wl.log 2>&1 || exit 1
done; done
