"""onc_rpc_amd — MI355X (gfx950) batch ONC-RPC / XDR codec.

Drop-in batch path for domodwyer/onc-rpc's RpcMessage::serialise_into and
RpcMessage::try_from (see include/onc_rpc.h for the C ABI and DESIGN.md).
The Python package is host plumbing for tests and the bench; all codec work
runs in the hand-written HIP kernels of libonc_rpc_amd.so.

The directory is named ``onc-rpc_amd`` (not importable by plain ``import``);
repo entry points register it as ``onc_rpc_amd`` via ``_onc_pkg.load()``.
"""
from . import layout  # noqa: F401
from .layout import (MSG_DTYPE, UNIX_DTYPE, HostBatch, build_batch, describe,  # noqa: F401
                     DECODE_SLICE, DECODE_BYTES)

__all__ = ["layout", "MSG_DTYPE", "UNIX_DTYPE", "HostBatch", "build_batch", "describe",
           "DECODE_SLICE", "DECODE_BYTES", "runtime", "synth", "shard"]


def __getattr__(name):
    # runtime/synth/shard import torch/numpy-heavy pieces lazily
    import importlib
    if name in ("runtime", "synth", "shard"):
        return importlib.import_module(f"{__name__}.{name}")
    raise AttributeError(name)
