"""ctypes binding of ``libtonehip.so`` (the C ABI declared in ``include/tonehip.h``).

The library is built in-tree (``t-one_amd/libtonehip.so``, see ``t-one_amd/csrc/Makefile``).  There is
no fallback: if the library is missing or fails to load, every entry point raises.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("TONEHIP_LIB", PKG_DIR / "libtonehip.so"))

# every symbol include/tonehip.h declares, with its ctypes signature
_c_void_p, _c_int, _c_int64, _c_double, _c_char_p = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_double, ctypes.c_char_p
SIGNATURES = {
    "tone_abi_version": (_c_int, []),
    "tone_last_error": (_c_char_p, []),
    "tone_session_create": (_c_int, [ctypes.POINTER(_c_void_p), _c_int, _c_int, _c_int]),
    "tone_session_destroy": (_c_int, [_c_void_p]),
    "tone_session_set_weight": (_c_int, [_c_void_p, _c_char_p, _c_void_p, _c_int64]),
    "tone_session_finalize": (_c_int, [_c_void_p]),
    "tone_session_set_graph": (_c_int, [_c_void_p, _c_int]),
    "tone_session_set_chunk": (_c_int, [_c_void_p, _c_int]),
    "tone_session_frames_per_chunk": (_c_int, [_c_void_p]),
    "tone_session_set_frame_info": (_c_int, [_c_void_p, _c_void_p]),
    "tone_session_run": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_int64, _c_void_p]),
    "tone_session_run_slots": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int64, _c_void_p, _c_int, _c_void_p]),
    "tone_session_run_rows": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int64, _c_void_p, _c_int, _c_void_p]),
    "tone_session_run_ring": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int64, _c_void_p, _c_void_p,
                                       _c_void_p, _c_int, _c_void_p]),
    "tone_session_ring_import": (_c_int, [_c_void_p, _c_void_p, _c_int64, _c_void_p, _c_int64, _c_void_p, _c_void_p,
                                          _c_void_p, _c_int, _c_void_p]),
    "tone_session_ring_export": (_c_int, [_c_void_p, _c_void_p, _c_int64, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                          _c_int64, _c_int, _c_void_p]),
    "tone_session_ring_elems": (_c_int64, []),
    "tone_session_device_bytes": (_c_int64, [_c_void_p]),
    "tone_session_set_timing": (_c_int, [_c_void_p, _c_int]),
    "tone_session_kernel_us": (_c_double, [_c_void_p, _c_char_p, ctypes.POINTER(_c_int64)]),
    "tone_session_debug_stop": (_c_int, [_c_void_p, _c_int]),
    "tone_session_debug_read": (_c_int, [_c_void_p, _c_char_p, _c_void_p, _c_int64]),
}
ABI_VERSION = 1

# "fp32": fp32 GEMMs as exact 3-way bf16 splits on the bf16 MFMA (fp32-accurate; the default fp32 path);
# "fp32-mfma": fp32 GEMMs on the exact-fp32 MFMA; "bf16": bf16 GEMM operands, fp32 accumulate
PRECISION = {"fp32": 0, "bf16": 1, "fp32-mfma": 2, "fp8": 3}

_lib = None


class ToneHipError(RuntimeError):
    """A libtonehip call returned a non-zero status."""


def load() -> ctypes.CDLL:
    """Load libtonehip.so once; raise loudly if it is absent (no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    # torch bundles its own libamdhip64.so.7; importing it first makes libtonehip bind to that same
    # HIP runtime (same SONAME), so torch-allocated device pointers and our kernels share one
    # runtime instance in the process.
    import torch  # noqa: F401
    if not LIB_PATH.exists():
        raise ImportError(
            f"{LIB_PATH} not found: build it with `make -C t-one_amd/csrc` or __graft_entry__.build(). "
            "There is no CPU fallback for the acoustic path."
        )
    lib = ctypes.CDLL(str(LIB_PATH))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.tone_abi_version() != ABI_VERSION:
        raise ImportError(f"libtonehip ABI {lib.tone_abi_version()} != expected {ABI_VERSION}")
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().tone_last_error().decode(errors="replace")
        raise ToneHipError(f"{what} failed ({rc}): {msg}")
