"""bench.py's vectored-encode validation (validate_iov) on the CPU: iovecs
and packed headers built from the oracle's contiguous wire pass; a wrong
header byte, iovec field, status or total is caught. (The GPU runs the same
function on device tensors after the timed region.)"""
import importlib.util
import os

import numpy as np
import pytest

import _onc_pkg

_onc_pkg.load()
import onc_rpc_amd.synth as S  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _case(oracle):
    import torch
    hb = S.mixed(3000, seed=31, pmin=0, pmax=200, exotic=0.0)
    wire, off, st, rec_len = oracle.encode_batch(hb)
    assert not st.any()
    n = hb.n
    plen = hb.msgs["payload_len"].astype(np.int64)
    hl = rec_len.astype(np.int64) - plen
    hoff = np.cumsum(hl) - hl
    hdr = np.concatenate([np.frombuffer(bytes(wire), np.uint8)[int(off[i]):int(off[i]) + int(hl[i])]
                          for i in range(n)])
    e = np.zeros((n, 4), np.int64)
    e[:, 0] = hoff
    e[:, 1] = hb.msgs["payload_off"].astype(np.int64)
    e[:, 2] = off[:-1].astype(np.int64)
    e[:, 3] = hl | (plen << 32)
    t = {
        "n": n, "iov": torch.from_numpy(e.copy()).view(torch.uint8).reshape(-1),
        "hdr_out": torch.from_numpy(np.concatenate([hdr, np.zeros(16, np.uint8)])),
        "iov_tot": torch.tensor([int(hl.sum()), len(wire)], dtype=torch.int64),
        "iov_status": torch.zeros(n, dtype=torch.int32),
        "wire": torch.from_numpy(np.frombuffer(bytes(wire), np.uint8).copy()),
        "rec_off": torch.from_numpy(off.astype(np.int64)),
        "hdr_len_ref": torch.from_numpy(hl), "plen": torch.from_numpy(plen),
        "hb": hb, "total_bytes": len(wire), "hdr_total": int(hl.sum()),
    }
    return t


def _validate(bm, t):
    import torch
    return bm.validate_iov(torch, t["n"], t["iov"], t["hdr_out"], t["iov_tot"], t["iov_status"], t["wire"],
                           t["rec_off"], t["hdr_len_ref"], t["plen"], t["hb"], t["total_bytes"], t["hdr_total"],
                           "cpu")


def test_validate_iov_accepts_the_packed_encode(oracle):
    assert _validate(_bench(), _case(oracle))


@pytest.mark.parametrize("corrupt", ["header_byte", "hdr_off", "payload_off", "wire_off", "hdr_len", "status",
                                     "total"])
def test_validate_iov_rejects(oracle, corrupt):
    import torch
    t = _case(oracle)
    e = t["iov"].view(torch.int64).view(t["n"], 4)
    if corrupt == "header_byte":
        t["hdr_out"][t["hdr_total"] // 2] ^= 1
    elif corrupt == "hdr_off":
        e[7, 0] += 4
    elif corrupt == "payload_off":
        e[11, 1] += 1
    elif corrupt == "wire_off":
        e[13, 2] += 4
    elif corrupt == "hdr_len":
        e[17, 3] += 4
    elif corrupt == "status":
        t["iov_status"][5] = 105
    else:
        t["iov_tot"][1] += 1
    assert not _validate(_bench(), t)
