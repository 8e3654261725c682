"""Utilities: file formats, synthetic data, timing/profiling helpers."""
from . import formats  # noqa: F401
