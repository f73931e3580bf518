"""ctypes binding of the CPU oracle (oracle/liboncoracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker/baseline, never as the
product path.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboncoracle.so")
_LIB = None


def use_library(path):
    """Swap in another build of the same oracle source (bench.py's CPU
    baseline compiles oracle/onc_oracle.c with -O3 -march=native on the host
    it runs on). Returns the previous library path."""
    global _LIB, LIB_PATH
    prev = LIB_PATH
    LIB_PATH = path
    _LIB = None
    load()
    return prev


def load():
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"oracle not built: {LIB_PATH} (make -C oracle)")
    lib = C.CDLL(LIB_PATH)
    vp, u64, i32, u32 = C.c_void_p, C.c_uint64, C.c_int, C.c_uint32
    lib.oracle_decode_message.argtypes = [vp, vp, u64, i32, u64, vp, vp, vp, vp]
    lib.oracle_decode_message.restype = C.c_int32
    lib.oracle_encode_message.argtypes = [vp, vp, vp, vp, vp, u64, vp, vp]
    lib.oracle_encode_message.restype = C.c_int32
    lib.oracle_encode_batch.argtypes = [u64, vp, vp, vp, vp, vp, u64, vp, vp, vp]
    lib.oracle_encode_batch.restype = None
    lib.oracle_decode_batch.argtypes = [vp, vp, u64, i32, vp, vp, vp, vp, vp]
    lib.oracle_decode_batch.restype = None
    lib.oracle_decode_batch_mt.argtypes = [vp, vp, u64, i32, vp, vp, vp, vp, vp, i32]
    lib.oracle_decode_batch_mt.restype = None
    lib.oracle_encode_batch_mt.argtypes = [u64, vp, vp, vp, vp, vp, vp, vp, vp, i32]
    lib.oracle_encode_batch_mt.restype = None
    lib.oracle_frame_stream.argtypes = [vp, u64, vp, u64, vp]
    lib.oracle_compact.argtypes = [vp, vp, vp, u64]
    lib.oracle_compact.restype = u64
    lib.oracle_frame_stream.restype = None
    lib.oracle_expected_message_len.argtypes = [vp, u64, vp]
    lib.oracle_expected_message_len.restype = C.c_int32
    lib.oracle_auth_decode.argtypes = [vp, u64, i32, vp, vp, vp]
    lib.oracle_auth_decode.restype = C.c_int32
    lib.oracle_auth_encode.argtypes = [vp, vp, vp, vp, u64, vp]
    lib.oracle_auth_encode.restype = C.c_int32
    lib.oracle_auth_serialised_len.argtypes = [vp, vp]
    lib.oracle_auth_serialised_len.restype = u32
    lib.oracle_auth_associated_data_len.argtypes = [vp, vp]
    lib.oracle_auth_associated_data_len.restype = u32
    lib.oracle_unix_params_decode.argtypes = [vp, u64, i32, u32, vp, vp]
    lib.oracle_unix_params_decode.restype = C.c_int32
    lib.oracle_unix_params_encode.argtypes = [vp, vp, vp, u64, vp]
    lib.oracle_unix_params_encode.restype = C.c_int32
    lib.oracle_opaque_from_wire.argtypes = [vp, u64, u64, vp, vp, vp]
    lib.oracle_opaque_from_wire.restype = C.c_int32
    lib.oracle_opaque_encode.argtypes = [vp, u32, vp, u64, vp]
    lib.oracle_opaque_encode.restype = C.c_int32
    lib.oracle_pad_length.argtypes = [u32]
    lib.oracle_pad_length.restype = u32
    lib.oracle_decode_body.argtypes = [i32, vp, vp, u64, i32, u32, u64, vp, vp, vp, vp, vp]
    lib.oracle_decode_body.restype = C.c_int32
    lib.oracle_encode_body.argtypes = [i32, vp, vp, vp, vp, vp, u64, vp, vp]
    lib.oracle_encode_body.restype = C.c_int32
    lib.oracle_encode_body_batch.argtypes = [i32, u64, vp, vp, vp, vp, vp, u64, vp, vp, vp]
    lib.oracle_encode_body_batch.restype = None
    lib.oracle_decode_body_batch.argtypes = [i32, vp, vp, u64, i32, vp, vp, vp, vp, vp, vp, vp]
    lib.oracle_decode_body_batch.restype = None
    _LIB = lib
    return lib


def _p(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


def _buf(b):
    a = np.frombuffer(bytes(b) + b"\0" * 8, np.uint8).copy()
    return a


def encode_batch(hb, out_cap=None):
    """HostBatch -> (wire bytes, rec_off u64[n+1], status i32[n], rec_len u32[n])."""
    lib = load()
    n = hb.n
    rec_off = np.zeros(n + 1, np.uint64)
    status = np.zeros(max(n, 1), np.int32)
    rec_len = np.zeros(max(n, 1), np.uint32)
    if out_cap is None:
        # size pass: encode with zero capacity to learn the total
        lib.oracle_encode_batch(n, _p(hb.msgs), _p(hb.unix), _p(hb.auth_arena), _p(hb.payload_arena),
                                None, 0, _p(rec_off), _p(status), _p(rec_len))
        out_cap = int(rec_off[n])
    out = np.zeros(max(out_cap, 1), np.uint8)
    lib.oracle_encode_batch(n, _p(hb.msgs), _p(hb.unix), _p(hb.auth_arena), _p(hb.payload_arena),
                            _p(out), out_cap, _p(rec_off), _p(status), _p(rec_len))
    total = min(int(rec_off[n]), out_cap)
    return out[:total].tobytes(), rec_off, status[:n], rec_len[:n]


def encode_batch_mt(hb, threads, out=None):
    """Multi-threaded encode (CPU-baseline leg): -> (out array, rec_off, status, rec_len).
    `out` (uint8) is reused when large enough."""
    lib = load()
    n = hb.n
    rec_off = np.zeros(n + 1, np.uint64)
    status = np.zeros(max(n, 1), np.int32)
    rec_len = np.zeros(max(n, 1), np.uint32)
    if out is None:
        _, off, _, _ = encode_batch(hb)
        out = np.zeros(max(int(off[n]), 1), np.uint8)
    lib.oracle_encode_batch_mt(n, _p(hb.msgs), _p(hb.unix), _p(hb.auth_arena), _p(hb.payload_arena),
                               _p(out), _p(rec_off), _p(status), _p(rec_len), threads)
    return out, rec_off, status[:n], rec_len[:n]


def decode_batch(wire, rec_off, mode, threads=1):
    """packed wire (uint8 array) + rec_off -> (msgs, unix, status, aux0, aux1)."""
    from importlib import import_module
    L = import_module("onc_rpc_amd.layout")
    lib = load()
    n = len(rec_off) - 1
    wire = np.ascontiguousarray(wire, dtype=np.uint8)
    rec_off = np.ascontiguousarray(rec_off, dtype=np.uint64)
    msgs = np.zeros(max(n, 1), L.MSG_DTYPE)
    unix = np.zeros(max(2 * n, 1), L.UNIX_DTYPE)
    status = np.zeros(max(n, 1), np.int32)
    aux0 = np.zeros(max(n, 1), np.uint32)
    aux1 = np.zeros(max(n, 1), np.uint32)
    if threads > 1:
        lib.oracle_decode_batch_mt(_p(wire), _p(rec_off), n, mode, _p(msgs), _p(unix), _p(status),
                                   _p(aux0), _p(aux1), threads)
    else:
        lib.oracle_decode_batch(_p(wire), _p(rec_off), n, mode, _p(msgs), _p(unix), _p(status),
                                _p(aux0), _p(aux1))
    return msgs[:n], unix[:2 * n], status[:n], aux0[:n], aux1[:n]


def frame_stream(buf, max_records=None):
    """Caller's expected_message_len loop -> (rec_off u64[n+1], n, consumed, status, aux0, aux1)."""
    lib = load()
    a = np.frombuffer(bytes(buf) + b"\0" * 8, np.uint8).copy()
    n_max = len(buf) // 4 + 1 if max_records is None else max_records
    off = np.zeros(n_max + 1, np.uint64)
    res = np.zeros(5, np.uint64)
    lib.oracle_frame_stream(_p(a), len(buf), _p(off), n_max, _p(res))
    n = int(res[0])
    return off[:n + 1], n, int(res[1]), int(np.int64(res[2])), int(res[3]), int(res[4])


def compact(wire, rec_off, status):
    """oracle_compact of an encoded batch -> (bytes, rec_off u64[n+1])."""
    lib = load()
    a = np.frombuffer(bytes(wire), np.uint8).copy()
    off = np.asarray(rec_off, np.uint64).copy()
    st = np.ascontiguousarray(status, np.int32)
    total = lib.oracle_compact(_p(a), _p(off), _p(st), len(st))
    return a[:total].tobytes(), off


def decode_message(buf: bytes, mode):
    """One buffer -> (status, msg record, unix[2], aux0, aux1); offsets relative to buf."""
    from importlib import import_module
    L = import_module("onc_rpc_amd.layout")
    lib = load()
    b = _buf(buf)
    msg = np.zeros(1, L.MSG_DTYPE)
    unix = np.zeros(2, L.UNIX_DTYPE)
    a0 = np.zeros(1, np.uint32)
    a1 = np.zeros(1, np.uint32)
    st = lib.oracle_decode_message(_p(b), _p(b), len(buf), mode, 0, _p(msg), _p(unix), _p(a0), _p(a1))
    return st, msg[0], unix, int(a0[0]), int(a1[0]), b


def encode_message(hb, i=0, cap=None):
    lib = load()
    written = np.zeros(1, np.uint64)
    slen = np.zeros(1, np.uint64)
    m = hb.msgs[i:i + 1].copy()
    if cap is None:
        lib.oracle_encode_message(_p(m), _p(hb.unix), _p(hb.auth_arena), _p(hb.payload_arena), None, 0,
                                  _p(written), _p(slen))
        cap = int(slen[0])
    out = np.zeros(max(cap, 1), np.uint8)
    st = lib.oracle_encode_message(_p(m), _p(hb.unix), _p(hb.auth_arena), _p(hb.payload_arena), _p(out),
                                   cap, _p(written), _p(slen))
    return st, out[:int(written[0])].tobytes(), int(slen[0])


def encode_body_batch(root, hb, out_cap=None):
    """`root`::serialise_into of every descriptor (onc_encode_body's checker)
    -> (wire bytes, rec_off u64[n+1], status i32[n], rec_len u32[n])."""
    lib = load()
    n = hb.n
    rec_off = np.zeros(n + 1, np.uint64)
    status = np.zeros(max(n, 1), np.int32)
    rec_len = np.zeros(max(n, 1), np.uint32)
    args = (_p(hb.msgs), _p(hb.unix), _p(hb.auth_arena), _p(hb.payload_arena))
    if out_cap is None:
        lib.oracle_encode_body_batch(root, n, *args, None, 0, _p(rec_off), _p(status), _p(rec_len))
        out_cap = int(rec_off[n])
    out = np.zeros(max(out_cap, 1), np.uint8)
    lib.oracle_encode_body_batch(root, n, *args, _p(out), out_cap, _p(rec_off), _p(status), _p(rec_len))
    total = min(int(rec_off[n]), out_cap)
    return out[:total].tobytes(), rec_off, status[:n], rec_len[:n]


def decode_body_batch(root, wire, rec_off, mode, param=None):
    """`root`'s TryFrom of every record (onc_decode_body's checker)
    -> (msgs, unix, status, aux0, aux1, consumed)."""
    from importlib import import_module
    L = import_module("onc_rpc_amd.layout")
    lib = load()
    n = len(rec_off) - 1
    wire = np.ascontiguousarray(wire, dtype=np.uint8)
    rec_off = np.ascontiguousarray(rec_off, dtype=np.uint64)
    prm = None if param is None else np.ascontiguousarray(param, dtype=np.uint32)
    msgs = np.zeros(max(n, 1), L.MSG_DTYPE)
    unix = np.zeros(max(2 * n, 1), L.UNIX_DTYPE)
    status = np.zeros(max(n, 1), np.int32)
    aux0 = np.zeros(max(n, 1), np.uint32)
    aux1 = np.zeros(max(n, 1), np.uint32)
    consumed = np.zeros(max(n, 1), np.uint32)
    lib.oracle_decode_body_batch(root, _p(wire), _p(rec_off), n, mode, _p(prm), _p(msgs), _p(unix), _p(status),
                                 _p(aux0), _p(aux1), _p(consumed))
    return msgs[:n], unix[:2 * n], status[:n], aux0[:n], aux1[:n], consumed[:n]
