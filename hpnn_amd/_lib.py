"""Loader of the native extension (hpnn_amd/_native*.so, links hpnn_amd/lib/libhpnn.so).

GPU entry points call `native()`; it raises if the extension is missing so that a
GPU run can never silently fall back to a different implementation."""
import importlib
import os

import torch  # noqa: F401

_NATIVE = None
_ERR = None


def native():
    global _NATIVE, _ERR
    if _NATIVE is None:
        try:
            _NATIVE = importlib.import_module("hpnn_amd._native")
        except ImportError as e:  # pragma: no cover - depends on build
            _ERR = e
            raise RuntimeError(
                "hpnn_amd native extension not built: run `make` (or __graft_entry__.build()) "
                f"in {os.path.dirname(os.path.dirname(__file__))}: {e}") from e
    return _NATIVE


def available():
    try:
        native()
        return True
    except RuntimeError:
        return False


def lib_path():
    return os.path.join(os.path.dirname(__file__), "lib", "libhpnn.so")
