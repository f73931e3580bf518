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


def test_iov_gather_ok_rebuilds_the_wire(oracle):
    """bench.iov_gather_ok (the host-side check of the PCIe-inclusive
    vectored legs): the writev gather of header slices + host payload slices
    equals the oracle's wire, in steps smaller than the batch; a wrong header
    byte, payload offset or wire offset is caught."""
    import onc_rpc_amd.layout as L
    bm = _bench()
    t = _case(oracle)
    e = t["iov"].numpy().view(L.IOV_DTYPE).copy()
    hdr = t["hdr_out"].numpy()
    pay = t["hb"].payload_arena
    ref = t["wire"].numpy()
    assert bm.iov_gather_ok(hdr, e, pay, ref, step=777)
    h2 = hdr.copy()
    h2[t["hdr_total"] // 3] ^= 4
    assert not bm.iov_gather_ok(h2, e, pay, ref, step=777)
    e2 = e.copy()
    e2["payload_off"][100] += 1
    assert not bm.iov_gather_ok(hdr, e2, pay, ref)
    e3 = e.copy()
    e3["wire_off"][50] += 4
    assert not bm.iov_gather_ok(hdr, e3, pay, ref)
    # a chunk of it against its slice of the wire (the pipelined leg's check)
    lo, hi = 1000, 2000
    w0, w1 = int(e["wire_off"][lo]), int(e["wire_off"][hi])
    ec = e[lo:hi].copy()
    ec["wire_off"] -= w0
    assert bm.iov_gather_ok(hdr, ec, pay, ref[w0:w1])


def test_parsed_lines_bytes():
    """The line count of the zero-copy decode's note: records of 300 bytes
    packed from 0 — a record's first 48 bytes span two 128-byte lines when
    they cross a line boundary."""
    bm = _bench()
    lens = np.full(8, 300, np.int64)
    starts = np.arange(8) * 300
    want = sum(((s + 47) // 128 - s // 128 + 1) * 128 for s in starts)
    assert bm.parsed_lines_bytes(lens) == want


def test_reduce_leg_and_best():
    """bench.reduce_leg (the over-ranks reduction of the PCIe-inclusive legs,
    here on one rank): values recomputed from ms, a failed or missing
    sub-leg is unvalidated with no value; _pick_best takes the fastest
    validated one."""
    import torch
    bm = _bench()
    res = {"serialised": {"ms_per_step": 2.0, "validated": True},
           "pipelined": {"ms_per_step": 4.0, "validated": True},
           "zero_copy": {"error": "x"}}
    res = bm.reduce_leg(torch, None, "cpu", res, ["serialised", "pipelined", "zero_copy", "missing"], 1_000_000)
    assert res["serialised"]["value"] == 500.0 and res["pipelined"]["value"] == 250.0
    assert res["zero_copy"]["value"] is None and not res["zero_copy"]["validated"]
    bm._pick_best(res, ["serialised", "pipelined", "zero_copy"])
    assert res["best"] == "serialised" and res["value"] == 500.0 and not res["validated"]
