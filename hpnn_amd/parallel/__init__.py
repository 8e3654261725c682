"""Parallelism: data parallel (RCCL all-reduce) and row-sharded tensor parallel."""
from .comm import NativeComm  # noqa: F401
from .dp import DataParallel, init_from_env  # noqa: F401
from .tp import TensorParallelMLP  # noqa: F401
