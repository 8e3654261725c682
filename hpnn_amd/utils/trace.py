"""Tracing / phase timing for the Python training paths (csrc/core/observe.cpp).

`phase(name)` nests a named range: it is forwarded to roctx by libhpnn (visible with
`rocprofv3 --marker-trace`) and its host wall time lands in libhpnn's timing table;
with `device=True` the range is also timed on the GPU with a pair of hipEvents
(torch.cuda.Event) and the device time is recorded as `<name>.gpu`.  `report()` returns
the table.  Everything is a no-op unless tracing is on (HPNN_TRACE=1 or enable()).

The reference has no timers or trace hooks."""
import contextlib

from .. import capi


def enable(on=True):
    capi.lib().hpnn_trace_enable(1 if on else 0)


def enabled():
    return bool(capi.lib().hpnn_trace_enabled())


_pending = []


@contextlib.contextmanager
def phase(name, device=False):
    L = capi.lib()
    if not L.hpnn_trace_enabled():
        yield
        return
    ev = None
    if device:
        import torch
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    L.hpnn_trace_push(name.encode())
    try:
        yield
    finally:
        L.hpnn_trace_pop()
        if ev is not None:
            ev[1].record()
            _pending.append((name, ev))


def flush():
    """resolve the device timings recorded so far (synchronises the events)"""
    L = capi.lib()
    while _pending:
        name, (a, b) = _pending.pop(0)
        b.synchronize()
        L.hpnn_trace_add(f"{name}.gpu".encode(), a.elapsed_time(b) * 1e-3)


def report():
    """{name: (calls, total seconds)} of every range recorded so far"""
    flush()
    import ctypes
    import re
    import os
    import tempfile
    L = capi.lib()
    # the C table is printed by hpnn_trace_report(FILE*); read it back through a file
    libc = ctypes.CDLL(None)
    libc.fopen.restype = ctypes.c_void_p
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fclose.argtypes = [ctypes.c_void_p]
    L.hpnn_trace_report.argtypes = [ctypes.c_void_p]
    L.hpnn_trace_report.restype = ctypes.c_int
    fd, path = tempfile.mkstemp()
    os.close(fd)
    try:
        f = libc.fopen(path.encode(), b"w")
        L.hpnn_trace_report(f)
        libc.fclose(f)
        out = {}
        for ln in open(path):
            m = re.match(r"NN\(TRACE\): (\S+)\s+(\d+)\s+([\d.]+)", ln)
            if m and m.group(1) != "range":
                out[m.group(1)] = (int(m.group(2)), float(m.group(3)) * 1e-3)
        return out
    finally:
        os.unlink(path)


def reset():
    _pending.clear()
    capi.lib().hpnn_trace_reset()


def metrics_open(path):
    """JSON-lines metrics sink (same as HPNN_METRICS=path)"""
    return capi.lib().hpnn_metrics_open(path.encode() if path else None)


def metrics_emit(event, **fields):
    import json
    body = json.dumps(fields)[1:-1]
    capi.lib().hpnn_metrics_emit(event.encode(), body.encode())
