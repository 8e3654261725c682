"""Caching device allocator (csrc/core/devmem.cpp): repeated nn_train_kernel calls reuse
the device blocks of the previous call instead of hipMalloc'ing them again, the results
are unchanged, and nn_deinit_all returns the cache to the driver."""
import os

import numpy as np
import pytest

from hpnn_amd.utils import formats


@pytest.mark.gpu
def test_repeated_training_reuses_device_blocks(gpu, tmp_path, monkeypatch):
    from hpnn_amd import capi
    from hpnn_amd._lib import native
    monkeypatch.delenv("HPNN_FORCE_CPU", raising=False)
    d = str(tmp_path)
    rng = np.random.default_rng(3)
    os.makedirs(os.path.join(d, "s"))
    for i in range(256):
        t = np.zeros(10)
        t[int(rng.integers(10))] = 1.0
        formats.write_sample(os.path.join(d, "s", f"s{i:04d}.txt"), rng.random(784), t)
    formats.write_conf(os.path.join(d, "nn.conf"), name="m", type="SNN", seed=9, inputs=784, hiddens=[128, 64],
                       outputs=10, train="BPM", sample_dir=os.path.join(d, "s"), test_dir=os.path.join(d, "s"))
    capi.init(0)
    n = native()
    outs = []
    for _ in range(2):
        net = capi.Network(os.path.join(d, "nn.conf")).set(mode="batched", batch=128, epochs=1, device="gpu")
        h0 = n.devmem_stats()[2]
        assert net.train()
        p = os.path.join(d, f"k{len(outs)}.opt")
        net.dump_kernel(p, exact=True)
        outs.append(open(p).read())
        net.close()
        hits = n.devmem_stats()[2] - h0
    assert hits > 0  # second call served from the cache
    assert outs[0] == outs[1]
    in_use, cached, _, _ = n.devmem_stats()
    assert cached > 0
    capi.deinit()
    assert n.devmem_stats()[1] == 0
