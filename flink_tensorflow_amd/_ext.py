"""Loading of the in-tree native extensions (`_native` host runtime, `_hip` GPU kernels).

Policy (see README "native code"):
* ``native()`` builds the host extension on first use when it is missing (g++ is always
  present in this image) — CPU tests never silently skip the C++ paths.
* ``hip()`` never falls back.  On a machine with a GPU a missing or stale ``_hip`` library
  is an error, so a GPU run can not quietly execute a PyTorch fallback instead of the
  hand-written kernels.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import threading

from . import _build

_lock = threading.Lock()
_native_mod = None
_hip_mod = None


def native(required: bool = True):
    global _native_mod
    if _native_mod is not None:
        return _native_mod
    with _lock:
        if _native_mod is None:
            try:
                override = os.environ.get("FTM_NATIVE_LIB")  # e.g. a sanitizer build
                if override:
                    spec = importlib.util.spec_from_file_location("flink_tensorflow_amd._native", override)
                    _native_mod = importlib.util.module_from_spec(spec)
                    spec.loader.exec_module(_native_mod)
                    return _native_mod
                if os.environ.get("FTM_NO_AUTOBUILD") != "1":
                    _build.build_native()
                _native_mod = importlib.import_module("flink_tensorflow_amd._native")
            except Exception:
                if required:
                    raise
                return None
    return _native_mod


def hip(required: bool = True):
    """Returns the `_hip` kernel module.  Imports torch first so the process shares
    torch's HIP runtime (same SONAME ``libamdhip64.so.7``)."""
    global _hip_mod
    if _hip_mod is not None:
        return _hip_mod
    with _lock:
        if _hip_mod is None:
            import torch  # noqa: F401  (must be loaded before the kernel library)

            try:
                if os.environ.get("FTM_AUTOBUILD_HIP") == "1":
                    _build.build_hip()
                if not _build.hip_lib_path().exists():
                    raise ImportError(
                        f"HIP kernel library {_build.hip_lib_path()} is missing: run "
                        "`python -m flink_tensorflow_amd._build hip` (or __graft_entry__.build())")
                _hip_mod = importlib.import_module("flink_tensorflow_amd._hip")
            except Exception:
                if required:
                    raise
                return None
    return _hip_mod


_rccl_mod = None


def rccl():
    """Returns the `_rccl` RCCL binding (never a fallback: collectives have no other
    product path).  Imports torch first so the binding resolves ``librccl.so.1`` to the
    RCCL torch already mapped (one RCCL instance per process)."""
    global _rccl_mod
    if _rccl_mod is not None:
        return _rccl_mod
    with _lock:
        if _rccl_mod is None:
            import torch  # noqa: F401

            if os.environ.get("FTM_AUTOBUILD_HIP") == "1":
                _build.build_rccl()
            if not _build.rccl_lib_path().exists():
                raise ImportError(f"RCCL binding {_build.rccl_lib_path()} is missing: run "
                                  "`python -m flink_tensorflow_amd._build rccl` (or __graft_entry__.build())")
            _rccl_mod = importlib.import_module("flink_tensorflow_amd._rccl")
    return _rccl_mod


def hip_available() -> bool:
    """True when a GPU is visible AND the kernel library imports."""
    import torch

    if not torch.cuda.is_available():
        return False
    return hip(required=False) is not None
