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


def _granules_loop(wire, lens, line):
    """decode.hip stage_window's granule count, one record at a time."""
    out, s = [], 0
    be = lambda o: int.from_bytes(bytes(wire[o:o + 4]), "big")  # noqa: E731
    pad = lambda x: (4 - x % 4) % 4  # noqa: E731
    for L in (int(x) for x in lens):
        q0 = s & 15
        avail = min(10, (q0 + L + 15) >> 4)
        r44 = min(4, (q0 + min(L, 44) + 15) >> 4)
        if line:
            win = s - q0
            nch = min(min(8, max(r44, (((win | 127) + 1) - win) >> 4, (q0 + min(L, 128) + 15) >> 4)), avail)
        else:
            nch = min(r44, avail)
        need = min(L, 160)
        if L >= 36 and 16 * nch >= q0 + 36:
            mt = be(s + 8)
            if mt == 0:
                cl = be(s + 32)
                vpos = 36 + cl + pad(cl) + 4
                if cl > 200:
                    need = 36
                elif q0 + vpos + 4 <= 16 * nch and vpos + 4 <= L:
                    vl = be(s + vpos)
                    need = vpos + 4 + (vl + pad(vl) if vl <= 200 else 0)
                else:
                    need = vpos + 4 + 16
            elif mt == 1:
                vl = be(s + 20)
                need = 24 + vl + pad(vl) + 12 if vl <= 200 else 24
        out.append(max(nch, min(avail, (q0 + need + 15) >> 4)) if L else 0)
        s += L
    return out


@pytest.mark.parametrize("line", [False, True])
def test_decode_granules(oracle, line):
    """bench.decode_granules (the zero-copy leg's h2d request count) agrees
    with a per-record restatement of stage_window on a mixed Call/Reply wire
    with AUTH_UNIX credentials, short records and unaligned starts."""
    bm = _bench()
    hb = S.mixed(2000, seed=7, pmin=0, pmax=300)
    wire, off, st, rec_len = oracle.encode_batch(hb)
    assert not st.any()
    w = np.frombuffer(bytes(wire), np.uint8)[:int(off[-1])].copy()
    lens = rec_len.astype(np.int64)
    got = bm.decode_granules(w, lens, line=line)
    want = _granules_loop(w, lens, line)
    assert got.tolist() == want
    assert got.min() >= 1 and got.max() <= 10


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
