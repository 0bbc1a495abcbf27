"""Many-chain consumers of sample_Pnx: Wasserstein contraction coefficient and
kernel distances through a 1-Lipschitz network (reference python/utils/
lipschitz.py, used in asumptions_check.ipynb).

The samplers are the device kernels' sample_Pnx (ARWMH or ASSS, frozen
adapt state): every loss evaluation draws n_train_batches x n_points x
sample_batch_size chains in one HIP launch each, which is where the time goes
(2 min on the reference CPU for the notebook's 1-D example).  The network,
its spectral normalisation and the Adam loop are small and run in torch on the
same device.

Same functions and arguments as the reference:
  spectral_norm                    lipschitz.py:10-57
  SpectralNormDense, LipschitzNN   lipschitz.py:60-94
  compute_wasserstein_contraction  lipschitz.py:97-218
  compute_kernel_distance          lipschitz.py:221-344
  compute_kernel_distance_1d       lipschitz.py:347-494
Return values are (tau_or_rho, model, params) with params = the model's
state_dict.  Differences: the initial power-iteration vector and the network
initialisation come from torch generators (the reference uses JAX keys), so
values agree with the reference in distribution, not bit for bit.
"""
from __future__ import annotations

import math
from typing import Callable

import numpy as np
import torch
import torch.nn as nn

from kernels_amd.random import as_key, split

__all__ = ["spectral_norm", "SpectralNormDense", "LipschitzNN", "compute_wasserstein_contraction",
           "compute_kernel_distance", "compute_kernel_distance_1d"]

_THRESHOLD = 1e-10
# diagnostics: when a list, _train appends (step, loss, clipped-gradient norm)
# of every training step (tools/cell101.py logs the trajectory)
TRAIN_LOG = None


def _start_vector(W2: torch.Tensor) -> torch.Tensor:
    """The power iteration's unit start vector for W2 (see spectral_norm).  The
    seed is jnp.uint32(W[0, 0]) as XLA converts a float to uint32: truncated
    toward zero and SATURATED -- every value below 1 (negative ones included)
    and NaN give 0, values from 2^32 up give 2^32 - 1.  (Parity unpinned: JAX
    is not importable here; XLA's float-to-unsigned conversion saturates.)"""
    w = float(W2[0, 0].detach())
    seed = 0 if not w > 0.0 else min(int(math.trunc(w)), 0xFFFFFFFF)
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    u = torch.randn(W2.shape[0], generator=g, dtype=W2.dtype).to(W2.device)
    return u / torch.linalg.norm(u)


def spectral_norm(W: torch.Tensor, num_power_iters: int = 10, eps: float = 1e-10) -> torch.Tensor:
    """W / max(sigma_max(W), 1) with sigma from power iteration (lipschitz.py:10-57);
    differentiable through the iteration as in the reference."""
    shape = W.shape
    W2 = W.reshape(shape[0], -1)
    # the start vector: random.fold_in(random.PRNGKey(0), W[0, 0]) folds in
    # jnp.uint32(W[0, 0]), i.e. the weight truncated to an integer -- 0 for
    # every |W[0, 0]| < 1, so in the reference the power iteration starts from
    # the SAME vector at every training step (and the ten iterations, which
    # are differentiated through, under-estimate sigma in a way the optimiser
    # can learn to use).  The same here: the seed is the truncated,
    # saturated weight (_start_vector), not its bit pattern.
    u = _start_vector(W2)
    v = torch.zeros(W2.shape[1], dtype=W.dtype, device=W.device)
    for _ in range(num_power_iters):
        v = W2.T @ u
        v = v / (torch.linalg.norm(v) + eps)
        u = W2 @ v
        u = u / (torch.linalg.norm(u) + eps)
    sigma = u @ (W2 @ v)
    return (W2 / torch.clamp(sigma, min=1.0)).reshape(shape)


class SpectralNormDense(nn.Module):
    """flax Dense with a spectrally normalised kernel [in, out] (lecun_normal
    init, zero bias)."""

    def __init__(self, in_features: int, features: int, use_bias: bool = True, generator=None):
        super().__init__()
        std = math.sqrt(1.0 / in_features) / 0.87962566103423978
        w = torch.empty(in_features, features)
        nn.init.trunc_normal_(w, std=std, a=-2 * std, b=2 * std, generator=generator)
        self.kernel = nn.Parameter(w)
        self.bias = nn.Parameter(torch.zeros(features)) if use_bias else None

    def forward(self, x):
        x = x @ spectral_norm(self.kernel)
        return x + self.bias if self.bias is not None else x


class LipschitzNN(nn.Module):
    """Three spectrally normalised layers with leaky ReLU: 1-Lipschitz scalar f."""

    def __init__(self, dim: int, num_features: int = 32, seed: int = 0):
        super().__init__()
        g = torch.Generator(device="cpu")
        g.manual_seed(seed)
        self.l1 = SpectralNormDense(dim, num_features, generator=g)
        self.l2 = SpectralNormDense(num_features, num_features, generator=g)
        self.l3 = SpectralNormDense(num_features, 1, generator=g)

    def forward(self, x):
        x = nn.functional.leaky_relu(self.l1(x))
        x = nn.functional.leaky_relu(self.l2(x))
        return self.l3(x).squeeze(-1)


def _as_dev(X, device=None) -> torch.Tensor:
    t = X if isinstance(X, torch.Tensor) else torch.as_tensor(np.asarray(X))
    dev = device if device is not None else (t.device if t.is_cuda else torch.device("cuda", torch.cuda.current_device()))
    return t.to(device=dev, dtype=torch.float32)


def _pair_mask(X: torch.Tensor):
    n_points, dim = X.shape
    dists = torch.linalg.norm(X[:, None] - X[None, :], dim=-1)
    q = 2 * dim / n_points
    lower = torch.clamp(2 * torch.quantile(dists.reshape(-1), q), min=_THRESHOLD)
    upper = math.sqrt(dim) * lower + _THRESHOLD
    return dists, (lower <= dists) & (dists <= upper)


def _init_seed(rng_key) -> int:
    """The network's initialisation follows the key like flax's
    model.init(rng_key, ..) (lipschitz.py:137-139, :267-269, :401-403): the
    torch generator is seeded from the split key's two words, so different
    keys give different initial networks (not flax's draws)."""
    k = as_key(rng_key)
    return int(k[0]) | (int(k[1]) << 32)


def _train(model, loss_fn, rng_key, max_steps: int, lr: float):
    """Adam with element-wise gradient clipping to [-1, 1], stopped after
    max_steps or when the squared norm of the clipped gradients reaches the
    threshold (lipschitz.py:160-190)."""
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    it, grad_norm = 0, 1.0
    key = as_key(rng_key)
    while it < max_steps and grad_norm > _THRESHOLD:
        it += 1
        key, sub = split(key)
        opt.zero_grad()
        loss = loss_fn(sub)
        loss.backward()
        gn = 0.0
        for p in model.parameters():
            p.grad.clamp_(-1.0, 1.0)
            gn += float((p.grad ** 2).sum())
        grad_norm = gn
        if TRAIN_LOG is not None:
            TRAIN_LOG.append((it, float(loss.detach()), gn))
        opt.step()
    print(f"Train finished in {it} steps. Last gradient norm: {grad_norm}.")
    return key


def _mean_f(model, batch: torch.Tensor) -> torch.Tensor:
    return model(batch).mean(dim=-1)  # [n_points, n_samples, d] -> [n_points]


def compute_wasserstein_contraction(sample_Px: Callable, rng_key, X, sample_batch_size=1000, n_train_batches=10,
                                    n_eval_batches=100, alpha=10, max_steps=100, lr=0.1):
    """tau(P) = max over near pairs of |Pf(x) - Pf(y)| / |x - y| for the best
    1-Lipschitz f (lipschitz.py:97-218).  sample_Px(key, X, n) -> [n_points, n, d]."""
    X = _as_dev(X)
    dists, mask = _pair_mask(X)
    rng_key, _ = split(rng_key)
    model = LipschitzNN(X.shape[1], seed=_init_seed(rng_key)).to(X.device)

    def Pf_mean(key, n_batches):
        keys = split(key, n_batches)
        return torch.stack([_mean_f(model, sample_Px(k, X, sample_batch_size)) for k in keys]).mean(dim=0)

    def loss_fn(key):
        Pf = Pf_mean(key, n_train_batches)
        diffs = torch.abs(Pf[:, None] - Pf[None, :])
        ratios = torch.where(mask, diffs / torch.where(mask, dists, torch.ones_like(dists)), torch.zeros_like(dists))
        return -torch.logsumexp(alpha * ratios.reshape(-1), 0) / alpha

    key = _train(model, loss_fn, rng_key, max_steps, lr)
    with torch.no_grad():
        Pf = Pf_mean(key, n_eval_batches)
        diffs = torch.abs(Pf[:, None] - Pf[None, :])
        tau = torch.max(torch.where(mask, diffs / dists, torch.zeros_like(dists)))
    return float(tau), model, model.state_dict()


def compute_kernel_distance(sample_Px: Callable, sample_Qx: Callable, rng_key, X, sample_batch_size=1000,
                            n_train_batches=10, n_eval_batches=100, max_steps=100, lr=0.1, alpha=10, init_params=None):
    """rho_d(P, Q): the contraction ratio of Pf - Qf (lipschitz.py:221-344); both
    samplers get the same key per batch, as in the reference."""
    X = _as_dev(X)
    dists, mask = _pair_mask(X)
    rng_key, _ = split(rng_key)
    model = LipschitzNN(X.shape[1], seed=_init_seed(rng_key)).to(X.device)
    if init_params is not None:
        model.load_state_dict(init_params)

    def dPf_mean(key, n_batches):
        out = []
        for k in split(key, n_batches):
            out.append(_mean_f(model, sample_Px(k, X, sample_batch_size)) -
                       _mean_f(model, sample_Qx(k, X, sample_batch_size)))
        return torch.stack(out).mean(dim=0)

    def loss_fn(key):
        d = dPf_mean(key, n_train_batches)
        diffs = torch.abs(d[:, None] - d[None, :])
        ratios = torch.where(mask, diffs / torch.where(mask, dists, torch.ones_like(dists)), torch.zeros_like(dists))
        return -torch.logsumexp(alpha * ratios.reshape(-1), 0) / alpha

    key = _train(model, loss_fn, rng_key, max_steps, lr)
    with torch.no_grad():
        d = dPf_mean(key, n_eval_batches)
        diffs = torch.abs(d[:, None] - d[None, :])
        rho = torch.max(torch.where(mask, diffs / dists, torch.zeros_like(dists)))
    return float(rho), model, model.state_dict()


def compute_kernel_distance_1d(sample_Px: Callable, sample_Qx: Callable, rng_key, x, sample_batch_size=10000,
                               n_train_batches=1, n_eval_batches=100, max_steps=100, lr=0.1, ratio_rad=1,
                               init_params=None):
    """1-D variant on sorted points x (lipschitz.py:347-494): neighbours at
    distance ratio_rad in training, adjacent points in the evaluation."""
    xt = _as_dev(x).reshape(-1)
    X = xt.reshape(-1, 1)
    rng_key, _ = split(rng_key)
    model = LipschitzNN(1, seed=_init_seed(rng_key)).to(X.device)
    if init_params is not None:
        model.load_state_dict(init_params)

    def dPf_batch(key):
        kp, kq = split(key)
        return _mean_f(model, sample_Px(kp, X, sample_batch_size)) - _mean_f(model, sample_Qx(kq, X, sample_batch_size))

    def loss_fn(key):
        d = torch.stack([dPf_batch(k) for k in split(key, n_train_batches)]).mean(dim=0)
        diffs = torch.abs(d[:-ratio_rad] - d[ratio_rad:])
        dists = torch.abs(xt[:-ratio_rad] - xt[ratio_rad:])
        return -(diffs / dists).max()

    key = _train(model, loss_fn, rng_key, max_steps, lr)
    with torch.no_grad():
        d = torch.stack([dPf_batch(k) for k in split(key, n_eval_batches)]).mean(dim=0)
        tau = torch.max(torch.abs(d[1:] - d[:-1]) / torch.abs(xt[1:] - xt[:-1]))
    return float(tau), model, model.state_dict()
