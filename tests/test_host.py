"""CPU tests: C ABI library exports, descriptor layout, host logic,
synthetic generators (no GPU compute calls)."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

import onc_rpc_amd.layout as L
import onc_rpc_amd.synth as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "onc_rpc.h")
LIB = os.path.join(ROOT, "onc-rpc_amd", "libonc_rpc_amd.so")


def header_functions():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(onc_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_header_symbol():
    assert os.path.exists(LIB), "build() must produce onc-rpc_amd/libonc_rpc_amd.so"
    lib = C.CDLL(LIB)
    funcs = header_functions()
    assert len(funcs) >= 16
    for f in funcs:
        assert hasattr(lib, f), f
    import onc_rpc_amd.runtime as R
    assert sorted(R.EXPORTED) == funcs
    lib.onc_abi_version.restype = C.c_int
    assert lib.onc_abi_version() == R.ABI_VERSION == 8
    lib.onc_status_str.restype = C.c_char_p
    assert lib.onc_status_str(1) == b"incomplete rpc message"


def test_library_reads_no_environment():
    """ABI 6: kernel choices, chunk sizes and the decode policy are explicit
    onc_codec_options; the shipping library names no environment variable
    (a stray one in a server process cannot change what it runs)."""
    blob = open(LIB, "rb").read()
    assert b"ONC_RPC_" not in blob
    assert b"getenv" not in blob


def test_codec_options_layout_matches_header():
    import onc_rpc_amd.runtime as R
    prog = r'''
#include <stdio.h>
#include <stddef.h>
#include "onc_rpc.h"
int main(void){
 printf("%zu %zu %zu %zu %zu %zu\n", sizeof(onc_codec_options), offsetof(onc_codec_options, flags),
        offsetof(onc_codec_options, decode_policy), offsetof(onc_codec_options, variant),
        offsetof(onc_codec_options, enc_chunk), offsetof(onc_codec_options, frame_chunk));
 return 0;
}
'''
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "o.c")
        open(src, "w").write(prog)
        exe = os.path.join(d, "o")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), src, "-o", exe])
        got = [int(x) for x in subprocess.check_output([exe]).split()]
    O = R.OncCodecOptions
    assert got == [C.sizeof(O), O.flags.offset, O.decode_policy.offset, O.variant.offset, O.enc_chunk.offset,
                   O.frame_chunk.offset]


def test_library_is_gfx950_code_object():
    # the fat binary embeds the offload target id (amdgcn-amd-amdhsa--gfx950)
    blob = open(LIB, "rb").read()
    assert b"gfx950" in blob
    assert b"gfx942" not in blob and b"sm_" not in blob[:0]


def test_descriptor_layout_matches_header():
    """offsetof/sizeof from the C header == numpy dtypes used by the host side."""
    prog = r'''
#include <stdio.h>
#include <stddef.h>
#include "onc_rpc.h"
int main(void){
 printf("%zu %zu %zu\n", sizeof(onc_msg), sizeof(onc_unix_params), sizeof(onc_auth));
 printf("%zu %zu %zu %zu %zu\n", offsetof(onc_msg,msg_type), offsetof(onc_msg,u), offsetof(onc_msg,payload_len),
        offsetof(onc_msg,payload_off), offsetof(onc_msg,cred));
 printf("%zu %zu %zu\n", offsetof(onc_msg,verf), offsetof(onc_unix_params,name_off), offsetof(onc_unix_params,gids));
 printf("%zu %zu %zu %zu %zu\n", sizeof(onc_iov_rec), offsetof(onc_iov_rec,payload_off), offsetof(onc_iov_rec,wire_off),
        offsetof(onc_iov_rec,hdr_len), offsetof(onc_iov_rec,payload_len));
 return 0;}
'''
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(prog)
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        vals = [int(x) for x in subprocess.check_output([exe]).split()]
    assert vals[:3] == [64, 96, 16]
    f = L.MSG_DTYPE.fields
    assert vals[3:8] == [f["msg_type"][1], f["f0"][1], f["payload_len"][1], f["payload_off"][1], f["cred_id"][1]]
    u = L.UNIX_DTYPE.fields
    assert vals[8:11] == [f["verf_id"][1], u["name_off"][1], u["gids"][1]]
    v = L.IOV_DTYPE.fields
    assert vals[11:] == [32, v["payload_off"][1], v["wire_off"][1], v["hdr_len"][1], v["payload_len"][1]]


def test_build_describe_round_trip():
    ms = S.random_messages(300, seed=5)
    hb = L.build_batch(ms)
    for i, m in enumerate(ms):
        want = dict(m)
        for k in ("cred", "verf"):
            if k in want and want[k]["kind"] == "none" and not want[k]["data"]:
                want[k] = {"kind": "none", "data": None}
        assert L.describe(hb.msgs[i], hb.unix, hb.auth_arena, hb.payload_arena) == want


@pytest.mark.parametrize("gen", ["call_none", "call_unix16", "cpu_roundtrip", "mixed", "mixed_exotic"])
def test_synth_batches_round_trip_through_oracle(oracle, gen):
    hb = {"call_none": lambda: S.call_none(300),
          "call_unix16": lambda: S.call_unix16(200),
          "cpu_roundtrip": lambda: S.cpu_roundtrip(100),
          "mixed": lambda: S.mixed(500),
          "mixed_exotic": lambda: S.mixed(500, seed=4, exotic=0.4)}[gen]()
    wire, off, st, ln = oracle.encode_batch(hb)
    assert (st == 0).all()
    w = np.frombuffer(wire + b"\0" * 16, np.uint8).copy()
    for mode in (L.DECODE_SLICE, L.DECODE_BYTES):
        msgs, unix, status, a0, a1 = oracle.decode_batch(w, off, mode)
        assert (status == 0).all()
        for i in range(hb.n):
            a = L.describe(hb.msgs[i], hb.unix, hb.auth_arena, hb.payload_arena)
            b = L.describe(msgs[i], unix, w)
            assert a == b, (gen, i)


def test_synth_record_sizes_match_survey():
    """W = 300 (configs[1]), 1152 (configs[3]), 192 (configs[0])."""
    import oracle_ffi
    for hb, w in ((S.call_none(4), 300), (S.call_unix16(4), 1152), (S.cpu_roundtrip(4), 192)):
        _, off, _, _ = oracle_ffi.encode_batch(hb)
        assert set(np.diff(off).tolist()) == {w}


def test_oracle_multithreaded_decode_matches(oracle):
    hb = S.mixed(3000, seed=9, exotic=0.2)
    wire, off, _, _ = oracle.encode_batch(hb)
    w = np.frombuffer(wire + b"\0" * 16, np.uint8).copy()
    cw, coff = S.corrupt(w, off, frac=0.3)
    a = oracle.decode_batch(cw, coff, L.DECODE_BYTES)
    b = oracle.decode_batch(cw, coff, L.DECODE_BYTES, threads=4)
    for x, y in zip(a, b):
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8))


def test_oracle_multithreaded_encode_matches(oracle):
    hb = S.mixed(3000, seed=11, exotic=0.2)
    wire, off, st, ln = oracle.encode_batch(hb)
    out, off2, st2, ln2 = oracle.encode_batch_mt(hb, threads=5)
    assert out.tobytes()[: len(wire)] == wire
    assert np.array_equal(off, off2) and np.array_equal(st, st2) and np.array_equal(ln, ln2)


def test_shard_bounds_and_bases():
    import onc_rpc_amd.shard as SH
    for n in (0, 1, 7, 1000, 64_000_000):
        for world in (1, 2, 4, 8):
            b = [SH.shard_bounds(n, world, r) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
            assert max(h - l for l, h in b) - min(h - l for l, h in b) <= 1
    base, total = SH.exclusive_bases([5, 0, 7, 3])
    assert list(base) == [0, 5, 5, 12] and total == 15


def test_expected_message_len_matches_oracle(oracle, golden):
    """onc_expected_message_len (library host function, rpc_message.rs:343-367)
    against the oracle on every golden message/error buffer and short prefixes."""
    import ctypes as C
    import onc_rpc_amd.runtime as R
    lib = oracle.load()
    bufs = [bytes.fromhex(v["hex"]) for sec in ("messages", "errors", "xdrlib", "derived_errors")
            for v in golden[sec] if "hex" in v]
    bufs += [b"", b"\x80", b"\x80\x00\x00", b"\x00\x00\x00\x08", b"\xff\xff\xff\xff"]
    assert len(bufs) > 30
    for buf in bufs:
        for cut in {len(buf), min(len(buf), 3), min(len(buf), 4)}:
            b = buf[:cut]
            w = C.c_uint32(0)
            a = np.frombuffer(b + b"\0", np.uint8)
            want = lib.oracle_expected_message_len(a.ctypes.data, len(b), C.addressof(w))
            st, got = R.expected_message_len(b)
            assert st == want, b.hex()
            if st == 0:
                assert got == w.value


def test_batch_struct_matches_ctypes():
    """onc_batch (ABI v2: arena sizes) as the ctypes binding lays it out."""
    import onc_rpc_amd.runtime as R
    prog = r'''
#include <stdio.h>
#include <stddef.h>
#include "onc_rpc.h"
int main(void){
 printf("%zu %zu %zu %zu %zu\n", sizeof(onc_batch), offsetof(onc_batch,payload_arena),
        offsetof(onc_batch,unix_count), offsetof(onc_batch,auth_len), offsetof(onc_batch,payload_len));
 return 0;}
'''
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(prog)
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        vals = [int(x) for x in subprocess.check_output([exe]).split()]
    B = R.OncBatch
    assert vals == [C.sizeof(B), B.payload_arena.offset, B.unix_count.offset, B.auth_len.offset,
                    B.payload_len.offset]
