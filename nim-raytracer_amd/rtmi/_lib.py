"""Loader for librtmi.so (the C-ABI of include/rtmi.h).

There is no fallback: if the native library is missing or lacks a symbol the
header declares, importing the renderer raises. Build it with
`make -C nim-raytracer_amd` or `python -c "import __graft_entry__ as g; g.build()"`.
"""
import ctypes as C
import os

from . import abi

LIB_PATH = os.environ.get("RTMI_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "librtmi.so")

_lib = None


class RtmiError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"rtmi error {code}: {msg}")
        self.code = code


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built (make -C nim-raytracer_amd)")
        # One HIP runtime per process: when PyTorch is importable, load it
        # first so librtmi.so binds to the same libamdhip64.so.7 torch uses
        # (device buffers and RCCL collectives come from torch). Loading the
        # system runtime first and torch's second leaves two runtimes that
        # do not see each other's devices.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        _lib = abi.bind(C.CDLL(LIB_PATH))
        if _lib.rt_version() != abi.RTMI_ABI_VERSION:
            raise ImportError(f"librtmi.so ABI {_lib.rt_version()} != {abi.RTMI_ABI_VERSION}")
    return _lib


def check(rc):
    if rc != abi.RT_OK:
        raise RtmiError(rc, lib().rt_last_error().decode(errors="replace"))
    return rc


def kernel_source_hash():
    """sha256 (first 16 hex digits) of the native sources (csrc/, the
    Makefile, include/rtmi.h): PMC summaries record it, and bench.py uses a
    committed summary only for the sources it was measured on."""
    from .srchash import source_hash
    return source_hash()


def library_source_hash():
    """The source hash librtmi.so was built from (rt_build_source_hash)."""
    return lib().rt_build_source_hash().decode()
