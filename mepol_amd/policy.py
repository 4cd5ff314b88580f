"""GaussianPolicy with the reference's API and state-dict layout (src/policy.py:11-88).

MLP ``net = [Linear(nf,h0), act, Linear(h0,h1), act, ...]``, ``mean = Linear(h_last, a)``,
state-independent ``log_std`` parameter; keys ``net.0.*``, ``net.2.*``, ``mean.*``, ``log_std``
(loadable from / by the reference, incl. its fp32 ``pretrained/*`` files).

Parameters are float64 (the reference's dtype, src/utils/dtypes.py:3) and are initialised on
the CPU generator in the reference's order (Linear defaults, then xavier_uniform on
``mean.weight`` and the ``net`` weights, policy.py:36-41), so a given torch seed yields the
reference's initial weights; the module can then be moved to the GPU with ``.to(device)``.
The forward/backward runs on PyTorch-ROCm (hipBLASLt/rocBLAS GEMMs).
"""
import math

import torch
import torch.nn as nn

LOG_STD_EPS = 1e-7  # src/utils/dtypes.py:7, used inside get_log_p (policy.py:49)
LOG_2PI = math.log(2 * math.pi)
SPLITK_MIN_ROWS = 16384
SPLITK = 32


def _split_count(n):
    """K-slices of the split-K weight gradient: the divisor of n in [24, 48] nearest SPLITK, so
    no remainder rows are left over (a separate K < 48 remainder GEMM cost 46 us beside an
    85-us main GEMM at 25k rows); SPLITK with a remainder when n has no such divisor."""
    for dv in sorted(range(24, 49), key=lambda v: (abs(v - SPLITK), v)):
        if n % dv == 0:
            return dv
    return SPLITK


def _weight_grad(gy, x, out=None):
    """gy^T x for a tall batch (into `out` when given): f64 on the GPU runs the split-K kernel
    of csrc/wgrad.hip; otherwise a split-K batched GEMM (a plain mm with K = N = 200k runs at
    0.1-4.5 TFLOP/s in f64 on rocBLAS; K-slices as one bmm plus a reduction run at the shape's
    GEMM rate, tools/gemm_probe.py)."""
    n = gy.shape[0]
    if (gy.is_cuda and gy.dtype == torch.float64 and x.dtype == torch.float64
            and gy.is_contiguous() and x.is_contiguous() and n >= SPLITK_MIN_ROWS):
        from . import ops  # split-K on the f64 matrix cores (csrc/wgrad.hip)

        return ops.weight_grad(gy, x, out=out)
    if n < SPLITK_MIN_ROWS:
        return torch.mm(gy.t(), x, out=out) if out is not None else gy.t() @ x
    sk = _split_count(n)
    rows = n // sk
    main = rows * sk
    prod = torch.bmm(gy[:main].reshape(sk, rows, -1).transpose(1, 2),
                     x[:main].reshape(sk, rows, -1))
    out = torch.sum(prod, 0, out=out) if out is not None else prod.sum(0)
    if main < n:
        out.add_(gy[main:].t() @ x[main:])
    return out


class _Linear(torch.autograd.Function):
    """y = x W^T + b with a split-K weight gradient (same math as nn.Linear)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        return torch.addmm(bias, x, weight.t())

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        gx = gy @ weight if ctx.needs_input_grad[0] else None
        gw = _weight_grad(gy, x) if ctx.needs_input_grad[1] else None
        gb = gy.sum(0) if ctx.needs_input_grad[2] else None
        return gx, gw, gb


class _HeadLogp(torch.autograd.Function):
    """log p(a | s) from the last hidden PRE-activation z via the fused HIP head (csrc/head.hip):
    relu, mean layer, Gaussian log-density and their backward in one pass each."""

    @staticmethod
    def forward(ctx, z, w_mean, b_mean, log_std, actions):
        from . import ops

        mu, logp = ops.head_forward(z, w_mean, b_mean, log_std, actions)
        ctx.save_for_backward(z, w_mean, log_std, actions, mu)
        return logp

    @staticmethod
    def backward(ctx, g):
        from . import ops

        z, w_mean, log_std, actions, mu = ctx.saved_tensors
        dz, dw, db, dls, _ = ops.head_backward(g.contiguous(), z, w_mean, log_std, actions, mu,
                                               need_dz=ctx.needs_input_grad[0])
        return dz, dw, db, dls, None


class _TwoLayerLogp(torch.autograd.Function):
    """log p(a | s) of the reference's 2-hidden-layer ReLU policy for a large batch:

    fused    layer 1, layer 2 and the head in ONE kernel (csrc/policy_fwd.hip) when nf <= 64
             and h1 <= 320; otherwise the three steps:
    layer 1  h1 = relu(x W1^T + b1)            HIP (csrc/mlp.hip), bias + ReLU fused
    layer 2  z2 = h1 W2^T                       rocBLAS GEMM without bias
    head     logp(relu(z2 + b2) Wm^T + bm)      HIP (csrc/head.hip), b2 + ReLU folded in
    backward: head (dz2, dWm, dbm, dlog_std, db2 in one pass) -> dW2 split-K bmm, dh1 GEMM ->
    layer-1 weights (ReLU mask, dW1, db1 in one pass).  Same math as nn.Linear/ReLU."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2, Wm, bm, log_std, actions):
        from . import ops

        if ops.policy_forward_ok(x.shape[1], W2.shape[0]):  # one kernel (csrc/policy_fwd.hip)
            h1, z2, mu, logp = ops.policy_forward(x, W1, b1, W2.contiguous(), b2, Wm, bm,
                                                  log_std, actions)
        else:
            h1 = ops.layer_forward(x, W1, b1)
            z2 = torch.mm(h1, W2.t())
            mu, logp = ops.head_forward(z2, Wm, bm, log_std, actions, bz=b2)
        ctx.save_for_backward(x, h1, z2, W2, b2, Wm, log_std, actions, mu)
        return logp

    @staticmethod
    def backward(ctx, g):
        from . import ops

        x, h1, z2, W2, b2, Wm, log_std, actions, mu = ctx.saved_tensors
        dz2, dWm, dbm, dls, db2 = ops.head_backward(g.contiguous(), z2, Wm, log_std, actions, mu,
                                                    bz=b2, need_dz=True)
        dW2 = _weight_grad(dz2, h1)
        dh1 = torch.mm(dz2, W2)
        dW1, db1 = ops.layer_backward(dh1, h1, x)
        return None, dW1, db1, dW2, db2, dWm, dbm, dls, None


def _apply_linear(layer, x):
    if x.dim() == 2 and x.shape[0] >= SPLITK_MIN_ROWS and torch.is_grad_enabled():
        return _Linear.apply(x, layer.weight, layer.bias)
    return layer(x)


class GaussianPolicy(nn.Module):
    def __init__(self, hidden_sizes, num_features, action_dim, log_std_init=-0.5,
                 activation=nn.ReLU, dtype=torch.float64):
        super().__init__()
        self.activation = activation
        self.num_features = num_features
        self.action_dim = action_dim
        widths = [num_features] + list(hidden_sizes)
        layers = []
        for fan_in, fan_out in zip(widths[:-1], widths[1:]):
            layers += [nn.Linear(fan_in, fan_out, dtype=dtype), activation()]
        self.net = nn.Sequential(*layers)
        self.mean = nn.Linear(widths[-1], action_dim, dtype=dtype)
        self.log_std = nn.Parameter(torch.full((action_dim,), float(log_std_init), dtype=dtype))
        self.log_of_two_pi = LOG_2PI
        self.initialize_weights()

    def initialize_weights(self):
        nn.init.xavier_uniform_(self.mean.weight)
        for layer in self.net:
            if isinstance(layer, nn.Linear):
                nn.init.xavier_uniform_(layer.weight)

    @property
    def device(self):
        return self.log_std.device

    def mean_action(self, x):
        h = x
        for layer in self.net:
            h = _apply_linear(layer, h) if isinstance(layer, nn.Linear) else layer(h)
        return _apply_linear(self.mean, h)

    def _fused_head_ok(self, states, actions):
        return (states.is_cuda and states.dim() == 2 and states.shape[0] >= SPLITK_MIN_ROWS
                and self.activation is nn.ReLU and self.action_dim <= 32
                and self.mean.in_features <= 512 and states.dtype == torch.float64
                and actions.dtype == torch.float64)

    def get_log_p(self, states, actions):
        """sum_a -0.5 (log 2pi + 2 log_std + (a - mu)^2 / (exp(log_std) + 1e-7)^2)."""
        if self._fused_head_ok(states, actions):
            layers = [m for m in self.net if isinstance(m, nn.Linear)]
            if len(layers) == 2 and self.num_features <= 64:
                l1, l2 = layers
                return _TwoLayerLogp.apply(states.contiguous(), l1.weight.contiguous(), l1.bias,
                                           l2.weight, l2.bias, self.mean.weight.contiguous(),
                                           self.mean.bias, self.log_std, actions.contiguous())
            h = states
            for layer in layers[:-1]:
                h = torch.relu(_apply_linear(layer, h))
            z = _apply_linear(layers[-1], h).contiguous()
            return _HeadLogp.apply(z, self.mean.weight.contiguous(), self.mean.bias,
                                   self.log_std, actions.contiguous())
        mu = self.mean_action(states)
        std = torch.exp(self.log_std) + LOG_STD_EPS
        return torch.sum(-0.5 * (self.log_of_two_pi + 2 * self.log_std + (actions - mu) ** 2 / std ** 2),
                         dim=1)

    def forward(self, x, deterministic=False):
        mu = self.mean_action(x)
        if deterministic:
            return mu, mu
        noise = torch.randn(mu.size(), dtype=mu.dtype, device=mu.device)
        return mu, mu + noise * torch.exp(self.log_std)

    def predict(self, s, deterministic=False):
        """Batch-1 action for one state (policy.py:64-67); returned on the CPU as the reference."""
        with torch.no_grad():
            x = torch.as_tensor(s, dtype=self.log_std.dtype, device=self.device).unsqueeze(0)
            return self(x, deterministic=deterministic)[1][0].cpu()


def train_supervised(env, policy, train_steps=100, batch_size=5000):
    """Regress the policy mean to zero on uniform observation-space states (policy.py:70-88).

    As in the reference, every step draws 5000 fresh states (batch_size is not used,
    Appendix A.10 of SURVEY.md) and Adam(lr=2.5e-4) is used.  Sampling is vectorised on the
    policy's device when the env exposes a Box observation space.
    """
    optimizer = torch.optim.Adam(policy.parameters(), lr=0.00025)
    space = env.observation_space
    nf = env.num_features
    for _ in range(train_steps):
        optimizer.zero_grad()
        if hasattr(space, "sample_torch"):
            states = space.sample_torch(5000, policy.device)[:, :nf]
        else:
            obs = [space.sample() for _ in range(5000)]
            if isinstance(obs[0], dict):
                obs = [o["observation"] for o in obs]
            else:
                obs = [o[:nf] for o in obs]
            states = torch.as_tensor(obs, dtype=torch.float64, device=policy.device)
        mu = policy(states)[0]
        loss = torch.mean((mu - torch.zeros_like(mu)) ** 2)
        loss.backward()
        optimizer.step()
    return policy
