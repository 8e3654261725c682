"""hpnn_amd -- MI355X-native feed-forward network framework (libhpnn capabilities).

Layers:
  hpnn_amd.capi      ctypes binding of the native C API (libhpnn.so: nn_* functions,
                     train_nn/run_nn workflows, FP64 CPU oracle, GPU online engine)
  hpnn_amd.ops       gfx950 HIP kernels (MFMA GEMMs, fused output / optimizer kernels)
  hpnn_amd.models    network definitions (ANN / SNN / LNN MLPs) and trainers
  hpnn_amd.parallel  data parallel (bucketed RCCL all-reduce overlapped with backward)
                     and row-sharded tensor parallel (reference-equivalent) modes
  hpnn_amd.utils     conf / kernel.opt / sample file formats, synthetic data, timers

torch is imported before any native module so the process shares torch's HIP runtime
(libamdhip64.so.7) with libhpnn.so.
"""
import torch  # noqa: F401  (must precede the native modules)

__version__ = "0.3.0"

from . import utils  # noqa: E402,F401
