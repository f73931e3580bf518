"""Debug: frame a configs[2] stream and compare with the oracle (dev tool)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np, torch
import _onc_pkg; _onc_pkg.load()
import oracle_ffi as O
import onc_rpc_amd.runtime as R, onc_rpc_amd.synth as S
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
hb = S.mixed(n, seed=2)
wire = O.encode_batch(hb)[0]
R.load_library(os.path.join(ROOT, "onc-rpc_amd", "libonc_rpc_amd_dbg.so"))
codec = R.Codec(0)
g = R.frame_host_stream(codec, wire)
o = O.frame_stream(wire)
print("gpu", g[1:], "oracle", o[1:], "offsets equal", np.array_equal(g[0], o[0]))
