"""ctypes binding of the native libhpnn C API (hpnn_amd/lib/libhpnn.so).

Gives Python users the reference workflow (include/libhpnn.h of ovhpa/hpnn): load a conf,
generate/load a kernel, train (online reference semantics or batched), run, dump
kernel.opt -- executed by the C++/HIP engines, not by Python.
"""
import ctypes
import os
import tempfile

import torch  # noqa: F401  (shares torch's HIP runtime with libhpnn)

from ._lib import lib_path

_LIB = None
_LIBC = None

NN_TYPE = {"ANN": 0, "LNN": 1, "SNN": 2}
NN_TRAIN = {"BP": 0, "BPM": 1, "CG": 2, "SPLX": 3}
NN_MODE = {"online": 0, "batched": 1}
NN_DTYPE = {"f64": 0, "f32": 1, "bf16": 2}
NN_DEVICE = {"auto": 0, "cpu": 1, "gpu": 2}


def lib():
    global _LIB, _LIBC
    if _LIB is None:
        path = lib_path()
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: build with `make`")
        L = ctypes.CDLL(path)
        vp, u, i, d, cp = ctypes.c_void_p, ctypes.c_uint, ctypes.c_int, ctypes.c_double, ctypes.c_char_p
        sig = {
            "nn_init_all": (i, [u]), "nn_deinit_all": (i, []),
            "nn_set_verbose": (None, [ctypes.c_short]), "nn_return_verbose": (ctypes.c_short, []),
            "nn_return_capabilities": (i, []), "nn_set_cuda_streams": (i, [u]),
            "nn_set_n_gpu": (i, [u]), "nn_get_n_gpu": (i, [ctypes.POINTER(u)]),
            "nn_set_omp_threads": (i, [u]),
            "nn_load_conf": (vp, [cp]), "nn_deinit_conf": (None, [vp]),
            "nn_dump_conf": (None, [vp, vp]), "nn_dump_kernel": (None, [vp, vp]),
            "nn_dump_kernel_exact": (None, [vp, vp]),
            "nn_train_kernel": (i, [vp]), "nn_run_kernel": (None, [vp]),
            "nn_get_n_inputs": (u, [vp]), "nn_get_n_hiddens": (u, [vp]), "nn_get_n_outputs": (u, [vp]),
            "nn_get_h_neurons": (u, [vp, u]),
            "nn_set_mode": (None, [vp, i]), "nn_set_dtype": (None, [vp, i]), "nn_set_device": (None, [vp, i]),
            "nn_set_batch": (None, [vp, u]), "nn_set_epochs": (None, [vp, u]),
            "nn_set_learning_rate": (None, [vp, d]), "nn_set_momentum": (None, [vp, d]),
            "nn_set_seed": (None, [vp, u]), "nn_return_seed": (u, [vp]),
            "nn_return_last_pass": (u, []), "nn_return_last_total": (u, []),
            "nn_return_version": (cp, []), "nn_return_type": (i, [vp]), "nn_return_train": (i, [vp]),
            "nn_dump_state": (i, [vp, cp]), "nn_load_state": (i, [vp, cp]), "nn_return_epochs_done": (u, [vp]),
            "nn_pack_samples": (i, [cp, cp]),
            "nn_pack_arrays": (i, [cp, vp, vp, u, u, u]),
            "hpnn_trace_enable": (None, [i]), "hpnn_trace_enabled": (i, []), "hpnn_trace_push": (None, [cp]),
            "hpnn_trace_pop": (None, []), "hpnn_trace_add": (None, [cp, d]), "hpnn_trace_reset": (None, []),
            "hpnn_trace_calls": (ctypes.c_uint64, [cp]), "hpnn_trace_seconds": (d, [cp]),
            "hpnn_metrics_open": (i, [cp]), "hpnn_metrics_emit": (None, [cp, cp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _LIB = L
        _LIBC = ctypes.CDLL(None)
        _LIBC.fopen.restype = vp
        _LIBC.fopen.argtypes = [cp, cp]
        _LIBC.fclose.argtypes = [vp]
    return _LIB


def init(verbose=0, streams=1):
    L = lib()
    L.nn_init_all(0)
    L.nn_set_verbose(verbose)
    L.nn_set_cuda_streams(streams)
    return L


def deinit():
    lib().nn_deinit_all()


class Network:
    """A libhpnn nn_def: conf + kernel, driven by the native engines."""

    def __init__(self, conf_path):
        self.L = lib()
        self.ptr = self.L.nn_load_conf(conf_path.encode())
        if not self.ptr:
            raise RuntimeError(f"nn_load_conf failed for {conf_path}")

    def close(self):
        if self.ptr:
            self.L.nn_deinit_conf(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # configuration
    def set(self, mode=None, dtype=None, device=None, batch=None, epochs=None, lr=None, momentum=None, seed=None):
        if mode is not None:
            self.L.nn_set_mode(self.ptr, NN_MODE[mode])
        if dtype is not None:
            self.L.nn_set_dtype(self.ptr, NN_DTYPE[dtype])
        if device is not None:
            self.L.nn_set_device(self.ptr, NN_DEVICE[device])
        if batch is not None:
            self.L.nn_set_batch(self.ptr, batch)
        if epochs is not None:
            self.L.nn_set_epochs(self.ptr, epochs)
        if lr is not None:
            self.L.nn_set_learning_rate(self.ptr, lr)
        if momentum is not None:
            self.L.nn_set_momentum(self.ptr, momentum)
        if seed is not None:
            self.L.nn_set_seed(self.ptr, seed)
        return self

    @property
    def dims(self):
        h = [self.L.nn_get_h_neurons(self.ptr, i) for i in range(self.L.nn_get_n_hiddens(self.ptr))]
        return [self.L.nn_get_n_inputs(self.ptr)] + h + [self.L.nn_get_n_outputs(self.ptr)]

    def train(self):
        return bool(self.L.nn_train_kernel(self.ptr))

    def run(self):
        self.L.nn_run_kernel(self.ptr)
        return self.L.nn_return_last_pass(), self.L.nn_return_last_total()

    def _dump(self, fn, path):
        f = _LIBC.fopen(path.encode(), b"w")
        if not f:
            raise OSError(path)
        try:
            fn(self.ptr, f)
        finally:
            _LIBC.fclose(f)

    def dump_kernel(self, path, exact=False):
        self._dump(self.L.nn_dump_kernel_exact if exact else self.L.nn_dump_kernel, path)

    def dump_conf(self, path):
        self._dump(self.L.nn_dump_conf, path)

    # exact checkpoint / resume (csrc/core/state.cpp)
    def dump_state(self, path):
        if not self.L.nn_dump_state(self.ptr, path.encode()):
            raise OSError(f"nn_dump_state({path}) failed")

    def load_state(self, path):
        if not self.L.nn_load_state(self.ptr, path.encode()):
            raise OSError(f"nn_load_state({path}) failed (missing, corrupted or mismatched)")

    @property
    def epochs_done(self):
        return self.L.nn_return_epochs_done(self.ptr)


def pack_samples(sample_dir, out_path):
    """pack a directory of sample files into one binary file (csrc/core/dataset.cpp)"""
    if not lib().nn_pack_samples(sample_dir.encode(), out_path.encode()):
        raise OSError(f"nn_pack_samples({sample_dir}) failed")


def pack_arrays(out_path, X, T):
    """write n records (X [n, n_in], T [n, n_out], anything numpy turns into float64) as a pack
    file train_nn / run_nn accept in place of a sample directory"""
    import numpy as np
    X = np.ascontiguousarray(X, dtype=np.float64)
    T = np.ascontiguousarray(T, dtype=np.float64)
    n, n_in = X.shape
    if T.shape[0] != n:
        raise ValueError("X and T need the same number of rows")
    if not lib().nn_pack_arrays(out_path.encode(), X.ctypes.data, T.ctypes.data, n, n_in, T.shape[1]):
        raise OSError(f"nn_pack_arrays({out_path}) failed")


def smoke_online():
    """One MNIST-shaped SNN sample trained online (reference semantics) by the native
    engine (GPU when present), then a kernel dump + reload round trip."""
    from .utils import formats
    import numpy as np
    init(0)
    with tempfile.TemporaryDirectory() as d:
        os.makedirs(os.path.join(d, "s"))
        rng = np.random.default_rng(0)
        x = rng.random(784)
        t = np.zeros(10)
        t[3] = 1.0
        formats.write_sample(os.path.join(d, "s", "s00001.txt"), x, t)
        conf = os.path.join(d, "nn.conf")
        formats.write_conf(conf, name="smoke", type="SNN", init="generate", seed=10958, inputs=784,
                           hiddens=[128, 64], outputs=10, train="BP", sample_dir=os.path.join(d, "s"),
                           test_dir=os.path.join(d, "s"))
        net = Network(conf)
        assert net.dims == [784, 128, 64, 10]
        assert net.train()
        kpath = os.path.join(d, "kernel.opt")
        net.dump_kernel(kpath)
        net.close()
        k = formats.read_kernel(kpath)
        assert [w.shape for w in k["weights"]] == [(128, 784), (64, 128), (10, 64)]
