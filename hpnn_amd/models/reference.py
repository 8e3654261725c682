"""Plain-PyTorch reference of the libhpnn math (any dtype; FP64 = the oracle).

Mirrors csrc/cpu/cpu_engine.cpp (online step) and csrc/cpu/cpu_batched.cpp (minibatch
step) -- i.e. reference ann.c / snn.c semantics, SURVEY 2.4.
"""
import torch

TINY = 1e-14


def act(x):
    return 2.0 / (1.0 + torch.exp(-x)) - 1.0


def dact(y):
    return -0.5 * (y * y - 1.0)


def forward(weights, X, net_type):
    """X [B, n_in] -> list of activations per layer (last = network output)."""
    hs = []
    h = X
    L = len(weights)
    for l, W in enumerate(weights):
        z = h @ W.t()
        if l < L - 1 or net_type == "ANN":
            h = act(z)
        elif net_type == "SNN":
            e = torch.exp(z - 1.0)
            h = e / (TINY + e.sum(1, keepdim=True))
        else:
            h = z
        hs.append(h)
    return hs


def loss_per_sample(o, T, net_type):
    if net_type == "SNN":
        return -(T * torch.log(o + TINY) * (o > 0)).sum(1) / o.shape[1]
    return 0.5 * ((T - o) ** 2).sum(1)


def deltas(weights, hs, T, net_type):
    L = len(weights)
    o = hs[-1]
    d = [None] * L
    d[L - 1] = (T - o) * dact(o) if net_type == "ANN" else (T - o)
    for l in range(L - 2, -1, -1):
        d[l] = (d[l + 1] @ weights[l + 1]) * dact(hs[l])
    return d


def batched_step(weights, X, T, net_type, lr, momentum=None, alpha=0.2):
    """In-place minibatch step; returns the mean loss before the update.
    momentum: list of dW tensors (BPM) or None (BP)."""
    hs = forward(weights, X, net_type)
    loss = loss_per_sample(hs[-1], T, net_type).mean()
    d = deltas(weights, hs, T, net_type)
    B = X.shape[0]
    for l, W in enumerate(weights):
        hin = X if l == 0 else hs[l - 1]
        G = d[l].t() @ hin / B
        if momentum is not None:
            momentum[l] += lr * G
            W += momentum[l]
            momentum[l] *= alpha
        else:
            W += lr * G
    return loss


def online_step(weights, x, t, net_type, lr, momentum=None, alpha=0.2):
    """One reference training iteration for one sample: returns Ep - Epr."""
    X, T = x[None, :], t[None, :]
    hs = forward(weights, X, net_type)
    Ep = loss_per_sample(hs[-1], T, net_type)[0]
    d = deltas(weights, hs, T, net_type)
    for l, W in enumerate(weights):
        hin = X if l == 0 else hs[l - 1]
        G = d[l].t() @ hin
        if momentum is not None:
            momentum[l] += lr * G
            W += momentum[l]
            momentum[l] *= alpha
        else:
            W += lr * G
    hs = forward(weights, X, net_type)
    return Ep - loss_per_sample(hs[-1], T, net_type)[0], hs[-1][0]
