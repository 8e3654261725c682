"""Network definitions and the named benchmark configurations (BASELINE.json)."""
from .mlp import MLP, reference_init, fast_init, TYPES  # noqa: F401

# name -> (layer sizes, type, default training)
CONFIGS = {
    # reference plumbing config: 4-8-4 ANN regression via train_nn on the CPU
    "ann484": ([4, 8, 4], "ANN", "BP"),
    # headline: MNIST 784-128-64-10 softmax SNN
    "mnist_snn": ([784, 128, 64, 10], "SNN", "BPM"),
    # RRUFF-XRD-shaped: 4096 inputs -> 230 -> 230 classes (tutorials/ann/tutorial.bash:135 hidden width)
    "rruff_snn": ([4096, 230, 230], "SNN", "BPM"),
    # synthetic 8 weight layers of 4096x4096 ANN (batch 8192 on 8 GPUs in BASELINE.json)
    "synth_ann_8x4096": ([4096] * 9, "ANN", "BPM"),
}


def build(name, **kw):
    sizes, typ, train = CONFIGS[name]
    kw.setdefault("momentum", train == "BPM")
    return MLP(sizes, typ, **kw)
