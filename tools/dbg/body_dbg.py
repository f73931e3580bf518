"""Debug: first differing record of onc_encode_body vs the oracle, per root."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import _onc_pkg  # noqa: E402

_onc_pkg.load()
import oracle_ffi as O  # noqa: E402
import onc_rpc_amd.layout as L  # noqa: E402
import onc_rpc_amd.runtime as R  # noqa: E402
import onc_rpc_amd.synth as S  # noqa: E402

codec = R.Codec(0)
for root in range(11):
    hb = L.build_batch(S.random_messages(3000, seed=100 + root, max_payload=300))
    g = R.encode_body_host_batch(codec, root, hb)
    o = O.encode_body_batch(root, hb)
    if g[0] == o[0] and np.array_equal(g[2], o[2]):
        print(root, "ok")
        continue
    off = o[1]
    gw, ow = np.frombuffer(g[0], np.uint8), np.frombuffer(o[0], np.uint8)
    k = int(np.nonzero(gw != ow)[0][0]) if len(gw) == len(ow) else -1
    i = int(np.searchsorted(off, k, side="right") - 1)
    print(root, "first diff byte", k, "record", i, "status", g[2][i], o[2][i])
    print(" desc", hb.msgs[i], "rec_off", off[i], off[i + 1], "tile", i // 64, "lane", i % 64)
    a, b = int(off[i]), int(off[i + 1])
    print(" gpu   ", gw[a:b][:96].tobytes().hex())
    print(" oracle", ow[a:b][:96].tobytes().hex())
    bad = np.nonzero(gw != ow)[0]
    recs = np.unique(np.searchsorted(off, bad, side="right") - 1)
    print(" records with diffs:", len(recs), recs[:20])
