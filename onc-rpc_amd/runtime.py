"""ctypes binding of the gfx950 codec library (libonc_rpc_amd.so, C ABI in
include/onc_rpc.h) with torch tensors as the device memory.

This is plumbing for tests/bench: all codec work runs in the HIP kernels.
There is no CPU fallback — loading fails loudly when the library is
missing, and every call that returns a non-zero rc raises.
"""
from __future__ import annotations

import ctypes as C
import mmap
import os

import numpy as np

from . import layout as L

_LIB = None
LIB_PATH = os.environ.get("ONC_RPC_AMD_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libonc_rpc_amd.so")

K_NAMES = ["enc_len_kernel", "scan_tiles_kernel", "enc_emit_kernel", "decode_kernel",
           "len_tiles_kernel", "len_apply_kernel", "iov_len_kernel", "iov_emit_kernel",
           "frame_chunks_kernel", "frame_write_kernel", "frame_walk_kernel",
           "frame_counts_kernel", "frame_guess_kernel", "compact_kernels"]
(K_ENC_LEN, K_SCAN_TILES, K_ENC_EMIT, K_DEC_PARSE, K_LEN_TILES, K_LEN_APPLY, K_IOV_LEN,
 K_IOV_EMIT, K_FRAME, K_FRAME_WRITE, K_FRAME_WALK, K_FRAME_COUNTS, K_FRAME_GUESS, K_COMPACT) = range(14)
ABI_VERSION = 8
K_COUNT = len(K_NAMES)

# every symbol include/onc_rpc.h declares
EXPORTED = [
    "onc_abi_version", "onc_codec_create", "onc_codec_destroy", "onc_codec_set_stream",
    "onc_codec_sync", "onc_codec_reserve", "onc_codec_last_error", "onc_status_str",
    "onc_codec_enable_timing", "onc_codec_kernel_stats", "onc_codec_reset_stats",
    "onc_kernel_name", "onc_encode_lengths", "onc_encode", "onc_decode", "onc_scan_lengths",
    "onc_expected_message_len", "onc_encode_iov", "onc_frame_stream", "onc_encode_plan", "onc_encode_emit",
    "onc_decode_lengths", "onc_decode_body", "onc_encode_body", "onc_encode_body_lengths",
    "onc_codec_create_ex", "onc_codec_set_decode_policy", "onc_host_register", "onc_host_unregister",
    "onc_compact", "onc_compact_iov",
]

# onc_codec_options (include/onc_rpc.h)
DECODE_POLICY_AUTO, DECODE_POLICY_STANDARD, DECODE_POLICY_LINE = 0, 1, 2
OPT_FORCE_SCAN = 0x1
VARIANT_EMIT_WS, VARIANT_EMIT_TILE = 0x200, 0x400
VARIANT_WS_NO_INTERIOR, VARIANT_WS_NO_FULL, VARIANT_WS_PIPELINE = 0x4000, 0x8000, 0x10000
VARIANT_EMIT_REPLAN, VARIANT_WHOLE_PLAN = 0x20000, 0x40000
# options every Codec() gets unless it is given its own (bench.py --variant)
DEFAULT_OPTIONS: dict = {}


class OncBatch(C.Structure):
    _fields_ = [("n", C.c_uint64), ("msgs", C.c_void_p), ("unix_params", C.c_void_p),
                ("auth_arena", C.c_void_p), ("payload_arena", C.c_void_p),
                ("unix_count", C.c_uint64), ("auth_len", C.c_uint64), ("payload_len", C.c_uint64)]


class OncCodecOptions(C.Structure):
    _fields_ = [("size", C.c_uint32), ("flags", C.c_uint32), ("decode_policy", C.c_int32), ("variant", C.c_uint32),
                ("enc_chunk", C.c_uint64), ("frame_chunk", C.c_uint64)]


class OncDecoded(C.Structure):
    _fields_ = [("msgs", C.c_void_p), ("unix_params", C.c_void_p), ("status", C.c_void_p),
                ("aux0", C.c_void_p), ("aux1", C.c_void_p)]


class CodecError(RuntimeError):
    pass


def load_library(path=LIB_PATH):
    """Load libonc_rpc_amd.so (raises if it has not been built)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise CodecError(f"HIP codec library missing: {path} (run __graft_entry__.build())")
    lib = C.CDLL(path)
    vp, u64, i32 = C.c_void_p, C.c_uint64, C.c_int
    lib.onc_abi_version.restype = i32
    lib.onc_codec_create.argtypes = [C.POINTER(vp), i32, vp]
    lib.onc_codec_create_ex.argtypes = [C.POINTER(vp), i32, vp, C.POINTER(OncCodecOptions)]
    lib.onc_codec_set_decode_policy.argtypes = [vp, i32]
    lib.onc_codec_destroy.argtypes = [vp]
    lib.onc_codec_set_stream.argtypes = [vp, vp]
    lib.onc_codec_sync.argtypes = [vp]
    lib.onc_codec_reserve.argtypes = [vp, u64]
    lib.onc_codec_last_error.argtypes = [vp]
    lib.onc_codec_last_error.restype = C.c_char_p
    lib.onc_status_str.argtypes = [C.c_int32]
    lib.onc_status_str.restype = C.c_char_p
    lib.onc_codec_enable_timing.argtypes = [vp, i32]
    lib.onc_codec_kernel_stats.argtypes = [vp, vp, vp]
    lib.onc_codec_reset_stats.argtypes = [vp]
    lib.onc_kernel_name.argtypes = [i32]
    lib.onc_kernel_name.restype = C.c_char_p
    lib.onc_encode_lengths.argtypes = [vp, C.POINTER(OncBatch), vp, vp]
    lib.onc_encode.argtypes = [vp, C.POINTER(OncBatch), vp, u64, vp, vp, vp]
    lib.onc_encode_plan.argtypes = [vp, C.POINTER(OncBatch), vp, vp]
    lib.onc_encode_emit.argtypes = [vp, C.POINTER(OncBatch), vp, u64, vp, vp]
    lib.onc_decode.argtypes = [vp, vp, vp, u64, i32, C.POINTER(OncDecoded)]
    lib.onc_decode_lengths.argtypes = [vp, vp, vp, u64, u64, i32, vp, C.POINTER(OncDecoded)]
    lib.onc_scan_lengths.argtypes = [vp, vp, u64, u64, vp]
    lib.onc_frame_stream.argtypes = [vp, vp, u64, vp, u64, vp]
    lib.onc_encode_iov.argtypes = [vp, C.POINTER(OncBatch), vp, u64, vp, vp, vp]
    lib.onc_expected_message_len.argtypes = [C.c_char_p, u64, C.POINTER(C.c_uint32)]
    lib.onc_expected_message_len.restype = C.c_int32
    lib.onc_decode_body.argtypes = [vp, i32, vp, vp, u64, i32, vp, C.POINTER(OncDecoded), vp]
    lib.onc_encode_body.argtypes = [vp, i32, C.POINTER(OncBatch), vp, u64, vp, vp, vp]
    lib.onc_encode_body_lengths.argtypes = [vp, i32, C.POINTER(OncBatch), vp, vp]
    lib.onc_host_register.argtypes = [vp, vp, u64, C.POINTER(vp)]
    lib.onc_host_unregister.argtypes = [vp, vp]
    lib.onc_compact.argtypes = [vp, vp, vp, vp, u64, C.POINTER(C.c_uint64)]
    lib.onc_compact_iov.argtypes = [vp, vp, vp, u64, vp]
    for name in EXPORTED:
        getattr(lib, name).restype = getattr(lib, name).restype or i32
    # a stale library would read a differently laid out onc_batch and label
    # the kernel timings wrongly: refuse it
    abi = lib.onc_abi_version()
    if abi != ABI_VERSION:
        raise CodecError(f"{path}: ABI {abi}, this binding expects {ABI_VERSION} (rebuild: __graft_entry__.build())")
    _LIB = lib
    return lib


def expected_message_len(buf: bytes):
    """expected_message_len (src/rpc_message.rs:343-367) -> (status, length)."""
    lib = load_library()
    out = C.c_uint32(0)
    st = lib.onc_expected_message_len(buf, len(buf), C.byref(out))
    return st, out.value


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _torch():
    import torch
    return torch


def to_device(arr, device):
    """numpy array -> uint8 CUDA tensor holding its bytes."""
    torch = _torch()
    raw = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
    if raw.size == 0:
        raw = np.zeros(16, np.uint8)
    return torch.from_numpy(raw.copy()).to(device)


class DeviceBatch:
    """Descriptor batch resident in HBM (torch uint8 tensors). The arena
    sizes handed to the codec (onc_batch bounds) are the tensors' sizes
    unless given."""

    def __init__(self, n, msgs, unix, auth_arena, payload_arena, unix_count=None, auth_len=None,
                 payload_len=None):
        self.n = n
        self.msgs = msgs
        self.unix = unix
        self.auth_arena = auth_arena
        self.payload_arena = payload_arena
        self.unix_count = unix.numel() // 96 if unix_count is None else unix_count
        self.auth_len = auth_arena.numel() if auth_len is None else auth_len
        self.payload_len = payload_arena.numel() if payload_len is None else payload_len

    @classmethod
    def from_host(cls, hb: L.HostBatch, device="cuda"):
        return cls(hb.n, to_device(hb.msgs, device), to_device(hb.unix, device),
                   to_device(hb.auth_arena, device), to_device(hb.payload_arena, device))

    def c_struct(self):
        return OncBatch(self.n, self.msgs.data_ptr(), self.unix.data_ptr(),
                        self.auth_arena.data_ptr(), self.payload_arena.data_ptr(),
                        self.unix_count, self.auth_len, self.payload_len)


def codec_options(variant=0, force_scan=False, enc_chunk=0, frame_chunk=0, decode_policy=DECODE_POLICY_AUTO):
    """onc_codec_options (include/onc_rpc.h) from keyword arguments."""
    return OncCodecOptions(C.sizeof(OncCodecOptions), OPT_FORCE_SCAN if force_scan else 0, decode_policy, variant,
                           enc_chunk, frame_chunk)


class Codec:
    """One onc_codec handle bound to a device and (by default) torch's
    current stream on that device. `options`: keyword arguments of
    codec_options (default: DEFAULT_OPTIONS)."""

    def __init__(self, device=0, stream=None, **options):
        torch = _torch()
        self.lib = load_library()
        self.device = device
        if stream is None:
            stream = torch.cuda.current_stream(device).cuda_stream
        self.stream = stream
        h = C.c_void_p()
        opt = codec_options(**(options or DEFAULT_OPTIONS))
        rc = self.lib.onc_codec_create_ex(C.byref(h), device, C.c_void_p(stream), C.byref(opt))
        if rc != 0:
            raise CodecError(f"onc_codec_create_ex rc={rc}")
        self.h = h

    def set_stream(self, stream):
        """Bind the handle to another HIP stream (an int hipStream_t or a torch stream)."""
        self.stream = getattr(stream, "cuda_stream", stream)
        self._check(self.lib.onc_codec_set_stream(self.h, C.c_void_p(self.stream)), "onc_codec_set_stream")

    def set_decode_policy(self, policy):
        self._check(self.lib.onc_codec_set_decode_policy(self.h, policy), "onc_codec_set_decode_policy")

    def close(self):
        if self.h:
            self.lib.onc_codec_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            err = self.lib.onc_codec_last_error(self.h).decode()
            raise CodecError(f"{what} rc={rc} {err}")

    def sync(self):
        self._check(self.lib.onc_codec_sync(self.h), "onc_codec_sync")

    def reserve(self, n):
        self._check(self.lib.onc_codec_reserve(self.h, n), "onc_codec_reserve")

    def enable_timing(self, on=True, kernels=None):
        """Bracket launches with HIP events: every kernel (on=True), none
        (on=False), or only the ids in `kernels` (K_* constants)."""
        mask = -1 if on else 0
        if on and kernels is not None:
            mask = 0
            for k in kernels:
                mask |= 1 << k
        self._check(self.lib.onc_codec_enable_timing(self.h, mask), "enable_timing")

    def kernel_stats(self):
        ms = (C.c_double * K_COUNT)()
        cnt = (C.c_uint64 * K_COUNT)()
        self._check(self.lib.onc_codec_kernel_stats(self.h, C.cast(ms, C.c_void_p), C.cast(cnt, C.c_void_p)),
                    "kernel_stats")
        return {K_NAMES[k]: (ms[k], cnt[k]) for k in range(K_COUNT)}

    def reset_stats(self):
        self._check(self.lib.onc_codec_reset_stats(self.h), "reset_stats")

    # -- encode -----------------------------------------------------------
    def encode_lengths(self, batch: DeviceBatch, rec_len, status):
        b = batch.c_struct()
        self._check(self.lib.onc_encode_lengths(self.h, C.byref(b), _ptr(rec_len), _ptr(status)),
                    "onc_encode_lengths")

    def encode(self, batch: DeviceBatch, out, rec_off, status, rec_len=None, out_cap=None):
        b = batch.c_struct()
        cap = out.numel() if out_cap is None else out_cap
        self._check(self.lib.onc_encode(self.h, C.byref(b), _ptr(out), cap, _ptr(rec_off), _ptr(status),
                                        _ptr(rec_len)), "onc_encode")

    def encode_plan(self, batch: DeviceBatch, status, rec_len=None):
        """Phase 1 of onc_encode (enc_len): lengths, validation, placement totals."""
        b = batch.c_struct()
        self._check(self.lib.onc_encode_plan(self.h, C.byref(b), _ptr(status), _ptr(rec_len)), "onc_encode_plan")

    def encode_emit(self, batch: DeviceBatch, out, rec_off, status, out_cap=None):
        """Phase 2 of onc_encode (enc_emit) of the batch last planned on this handle."""
        b = batch.c_struct()
        cap = out.numel() if out_cap is None else out_cap
        self._check(self.lib.onc_encode_emit(self.h, C.byref(b), _ptr(out), cap, _ptr(rec_off), _ptr(status)),
                    "onc_encode_emit")

    def encode_iov(self, batch: DeviceBatch, hdr_out, iov, status, totals=None, hdr_cap=None):
        """Vectored encode: headers into hdr_out, one onc_iov_rec (32 B) per record in iov."""
        b = batch.c_struct()
        cap = hdr_out.numel() if hdr_cap is None else hdr_cap
        self._check(self.lib.onc_encode_iov(self.h, C.byref(b), _ptr(hdr_out), cap, _ptr(iov), _ptr(status),
                                            _ptr(totals)), "onc_encode_iov")

    def frame_stream(self, wire, length, rec_off, max_records, result):
        """Frame a stream of back-to-back records (device buffers)."""
        self._check(self.lib.onc_frame_stream(self.h, _ptr(wire), length, _ptr(rec_off), max_records,
                                              _ptr(result)), "onc_frame_stream")

    # -- decode -----------------------------------------------------------
    def decode(self, wire, rec_off, n, mode, msgs, unix, status, aux0, aux1):
        d = OncDecoded(msgs.data_ptr(), unix.data_ptr(), status.data_ptr(), aux0.data_ptr(),
                       aux1.data_ptr())
        self._check(self.lib.onc_decode(self.h, _ptr(wire), _ptr(rec_off), n, mode, C.byref(d)),
                    "onc_decode")

    def decode_lengths(self, wire, rec_len, n, base, mode, msgs, unix, status, aux0, aux1, rec_off=None):
        """onc_decode_lengths: offsets from rec_len inside the decode (rec_off
        optional: receives them, n + 1 entries)."""
        d = OncDecoded(msgs.data_ptr(), unix.data_ptr(), status.data_ptr(), aux0.data_ptr(),
                       aux1.data_ptr())
        self._check(self.lib.onc_decode_lengths(self.h, _ptr(wire), _ptr(rec_len), n, base, mode,
                                                _ptr(rec_off) if rec_off is not None else None, C.byref(d)),
                    "onc_decode_lengths")

    # -- body-level roots (ONC_ROOT_*) ---------------------------------------
    def decode_body(self, root, wire, rec_off, n, mode, msgs, unix, status, aux0, aux1, param=None, consumed=None):
        """onc_decode_body: each record decoded as `root`'s TryFrom."""
        d = OncDecoded(msgs.data_ptr(), unix.data_ptr(), status.data_ptr(), aux0.data_ptr(),
                       aux1.data_ptr())
        self._check(self.lib.onc_decode_body(self.h, root, _ptr(wire), _ptr(rec_off), n, mode, _ptr(param),
                                             C.byref(d), _ptr(consumed)), "onc_decode_body")

    def encode_body_lengths(self, root, batch: DeviceBatch, rec_len, status):
        b = batch.c_struct()
        self._check(self.lib.onc_encode_body_lengths(self.h, root, C.byref(b), _ptr(rec_len), _ptr(status)),
                    "onc_encode_body_lengths")

    def encode_body(self, root, batch: DeviceBatch, out, rec_off, status, rec_len=None, out_cap=None):
        b = batch.c_struct()
        cap = out.numel() if out_cap is None else out_cap
        self._check(self.lib.onc_encode_body(self.h, root, C.byref(b), _ptr(out), cap, _ptr(rec_off), _ptr(status),
                                             _ptr(rec_len)), "onc_encode_body")

    def compact(self, out, rec_off, status, n):
        """onc_compact: the extents of records with status != OK dropped from
        an encoded buffer in place (rec_off rewritten); returns the new
        rec_off[n]."""
        total = C.c_uint64(0)
        self._check(self.lib.onc_compact(self.h, _ptr(out), _ptr(rec_off), _ptr(status), n, C.byref(total)),
                    "onc_compact")
        return total.value

    def compact_iov(self, iov, status, n, totals=None):
        """onc_compact_iov: failing records' iovecs emptied, wire_off re-placed."""
        self._check(self.lib.onc_compact_iov(self.h, _ptr(iov), _ptr(status), n, _ptr(totals)), "onc_compact_iov")

    def scan_lengths(self, rec_len, n, base, rec_off):
        self._check(self.lib.onc_scan_lengths(self.h, _ptr(rec_len), n, base, _ptr(rec_off)),
                    "onc_scan_lengths")


class HostMapped:
    """A host buffer the kernels read and write in place (onc_host_register):
    page-aligned anonymous memory, as a socket buffer would be. `host` is its
    numpy byte view (typed views: view(dtype)); data_ptr() is the device
    address, so it goes wherever a device tensor goes in this binding
    (Codec calls, DeviceBatch fields). close() unregisters it."""

    # bytes registered through HostMapped in this process, now and at most
    # (bench.py reports the pinned host memory a run holds)
    live_bytes = 0
    peak_bytes = 0

    def __init__(self, codec: "Codec", nbytes: int):
        self.nbytes = int(nbytes)
        self._dev = None
        self._mm = mmap.mmap(-1, max(self.nbytes, 4096))
        self.host = np.frombuffer(self._mm, np.uint8, count=self.nbytes)
        self._addr = self.host.ctypes.data if self.nbytes else np.frombuffer(self._mm, np.uint8).ctypes.data
        self._codec = codec
        dev = C.c_void_p()
        codec._check(codec.lib.onc_host_register(codec.h, C.c_void_p(self._addr), max(self.nbytes, 4096),
                                                  C.byref(dev)), "onc_host_register")
        self._dev = dev.value
        HostMapped.live_bytes += max(self.nbytes, 4096)
        HostMapped.peak_bytes = max(HostMapped.peak_bytes, HostMapped.live_bytes)

    @classmethod
    def from_array(cls, codec, arr):
        """A mapped copy of a numpy array's bytes."""
        raw = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
        m = cls(codec, raw.size)
        m.host[:] = raw
        return m

    def data_ptr(self):
        return self._dev

    def numel(self):
        return self.nbytes

    def element_size(self):
        return 1

    def view(self, dtype):
        return self.host.view(dtype)

    def close(self):
        # unregistered whether or not its codec is still open (a pinned range
        # belongs to the process: onc_host_unregister takes a NULL codec), so
        # the pages are unpinned before the mapping is freed
        if self._dev is not None:
            self._codec.lib.onc_host_unregister(self._codec.h or None, C.c_void_p(self._addr))
            HostMapped.live_bytes -= max(self.nbytes, 4096)
        self._dev = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def host_device_pointer(codec: "Codec", t):
    """Device address of a pinned host tensor (torch pin_memory =
    hipHostMalloc): onc_host_register maps it without registering it again."""
    dev = C.c_void_p()
    codec._check(codec.lib.onc_host_register(codec.h, C.c_void_p(t.data_ptr()), t.numel() * t.element_size(),
                                             C.byref(dev)), "onc_host_register")
    return dev.value


class MappedHostBatch:
    """A HostBatch whose arrays live in mapped host memory (HostMapped): an
    onc_batch the kernels read in place — descriptors, AUTH_UNIX table and
    arenas never copied to the device."""

    def __init__(self, codec, hb: L.HostBatch):
        self.n = hb.n
        self.msgs = HostMapped.from_array(codec, hb.msgs)
        self.unix = HostMapped.from_array(codec, hb.unix if hb.unix.size else np.zeros(1, L.UNIX_DTYPE))
        self.auth_arena = HostMapped.from_array(codec, hb.auth_arena if hb.auth_arena.size else np.zeros(16, np.uint8))
        self.payload_arena = HostMapped.from_array(codec, hb.payload_arena if hb.payload_arena.size
                                                   else np.zeros(16, np.uint8))
        self.unix_count = hb.unix.size
        self.auth_len = hb.auth_arena.size
        self.payload_len = hb.payload_arena.size

    def c_struct(self):
        return OncBatch(self.n, self.msgs.data_ptr(), self.unix.data_ptr(), self.auth_arena.data_ptr(),
                        self.payload_arena.data_ptr(), self.unix_count, self.auth_len, self.payload_len)

    def close(self):
        for m in (self.msgs, self.unix, self.auth_arena, self.payload_arena):
            m.close()


class DecodeBuffers:
    """Device output buffers for a decode of n records."""

    def __init__(self, n, device="cuda"):
        torch = _torch()
        self.n = n
        m = max(n, 1)
        self.msgs = torch.empty(m * 64, dtype=torch.uint8, device=device)
        self.unix = torch.empty(2 * m * 96, dtype=torch.uint8, device=device)
        self.status = torch.empty(m, dtype=torch.int32, device=device)
        self.aux0 = torch.empty(m, dtype=torch.int32, device=device)
        self.aux1 = torch.empty(m, dtype=torch.int32, device=device)

    def to_host(self):
        msgs = self.msgs.cpu().numpy().view(L.MSG_DTYPE)[: self.n]
        unix = self.unix.cpu().numpy().view(L.UNIX_DTYPE)[: 2 * self.n]
        return (msgs, unix, self.status.cpu().numpy()[: self.n].copy(),
                self.aux0.cpu().numpy().view(np.uint32)[: self.n].copy(),
                self.aux1.cpu().numpy().view(np.uint32)[: self.n].copy())


def encode_host_batch(codec: Codec, hb: L.HostBatch, device="cuda", out_cap=None):
    """Convenience: host batch -> GPU encode -> (wire bytes, rec_off, status, rec_len) on host."""
    torch = _torch()
    db = DeviceBatch.from_host(hb, device)
    n = hb.n
    lens = codec_lengths(codec, db)
    total = int(lens.sum())
    cap = total if out_cap is None else out_cap
    out = torch.zeros(max(16, (cap + 15) // 16 * 16), dtype=torch.uint8, device=device)
    rec_off = torch.empty(n + 1, dtype=torch.int64, device=device)
    status = torch.empty(max(n, 1), dtype=torch.int32, device=device)
    rec_len = torch.empty(max(n, 1), dtype=torch.int32, device=device)
    codec.encode(db, out, rec_off, status, rec_len, out_cap=cap)
    codec.sync()
    return (out.cpu().numpy()[:min(total, cap)].tobytes(), rec_off.cpu().numpy().view(np.uint64).copy(),
            status.cpu().numpy()[:n].copy(), rec_len.cpu().numpy().view(np.uint32)[:n].copy())


def frame_host_stream(codec: Codec, buf: bytes, max_records=None, device="cuda"):
    """Convenience: host stream bytes -> GPU framing -> (rec_off[n+1], n, consumed, status, aux0, aux1)."""
    torch = _torch()
    w = to_device(np.frombuffer(bytes(buf) + b"\0" * 16, np.uint8), device)
    m = len(buf) // 4 + 1 if max_records is None else max_records
    off = torch.zeros(m + 1, dtype=torch.int64, device=device)
    res = torch.zeros(5, dtype=torch.int64, device=device)
    codec.frame_stream(w, len(buf), off, m, res)
    codec.sync()
    r = res.cpu().numpy()
    n = int(r[0])
    return (off.cpu().numpy().view(np.uint64)[:n + 1].copy(), n, int(r[1]), int(r[2]), int(np.uint32(r[3])),
            int(np.uint32(r[4])))


def codec_lengths(codec: Codec, db: DeviceBatch):
    torch = _torch()
    n = db.n
    rec_len = torch.empty(max(n, 1), dtype=torch.int32, device=db.msgs.device)
    status = torch.empty(max(n, 1), dtype=torch.int32, device=db.msgs.device)
    if n:
        codec.encode_lengths(db, rec_len, status)
        codec.sync()
    return rec_len.cpu().numpy().view(np.uint32)[:n].astype(np.uint64)


def decode_host_wire(codec: Codec, wire: np.ndarray, rec_off: np.ndarray, mode, device="cuda"):
    """Convenience: packed wire + offsets (host) -> GPU decode -> host arrays."""
    torch = _torch()
    n = len(rec_off) - 1
    w = to_device(wire, device)
    off = torch.from_numpy(rec_off.astype(np.uint64).view(np.int64).copy()).to(device)
    bufs = DecodeBuffers(n, device)
    codec.decode(w, off, n, mode, bufs.msgs, bufs.unix, bufs.status, bufs.aux0, bufs.aux1)
    codec.sync()
    return bufs.to_host()


def encode_body_host_batch(codec: Codec, root, hb: L.HostBatch, device="cuda", out_cap=None):
    """Convenience: host batch -> GPU onc_encode_body -> (wire bytes, rec_off, status, rec_len) on host."""
    torch = _torch()
    db = DeviceBatch.from_host(hb, device)
    n = hb.n
    rec_len = torch.empty(max(n, 1), dtype=torch.int32, device=device)
    status = torch.empty(max(n, 1), dtype=torch.int32, device=device)
    if n:
        codec.encode_body_lengths(root, db, rec_len, status)
        codec.sync()
    total = int(rec_len.cpu().numpy().view(np.uint32)[:n].astype(np.uint64).sum())
    cap = total if out_cap is None else out_cap
    out = torch.zeros(max(16, (cap + 15) // 16 * 16), dtype=torch.uint8, device=device)
    rec_off = torch.empty(n + 1, dtype=torch.int64, device=device)
    codec.encode_body(root, db, out, rec_off, status, rec_len, out_cap=cap)
    codec.sync()
    return (out.cpu().numpy()[:min(total, cap)].tobytes(), rec_off.cpu().numpy().view(np.uint64).copy(),
            status.cpu().numpy()[:n].copy(), rec_len.cpu().numpy().view(np.uint32)[:n].copy())


def decode_body_host_wire(codec: Codec, root, wire: np.ndarray, rec_off: np.ndarray, mode, param=None, device="cuda"):
    """Convenience: packed records + offsets (host) -> GPU onc_decode_body ->
    (msgs, unix, status, aux0, aux1, consumed) on host."""
    torch = _torch()
    n = len(rec_off) - 1
    w = to_device(wire, device)
    off = torch.from_numpy(rec_off.astype(np.uint64).view(np.int64).copy()).to(device)
    bufs = DecodeBuffers(n, device)
    prm = None if param is None else torch.from_numpy(np.asarray(param, np.uint32).view(np.int32).copy()).to(device)
    consumed = torch.empty(max(n, 1), dtype=torch.int32, device=device)
    codec.decode_body(root, w, off, n, mode, bufs.msgs, bufs.unix, bufs.status, bufs.aux0, bufs.aux1,
                      param=prm, consumed=consumed)
    codec.sync()
    return bufs.to_host() + (consumed.cpu().numpy().view(np.uint32)[:n].copy(),)
