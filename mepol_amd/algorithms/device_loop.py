"""One off-policy iteration of MEPOL as a replayable HIP graph.

An iteration of the reference's loop (src/algorithms/mepol.py:429-439) is
``policy_update`` (entropy at theta_t, backward, optimizer step) followed by ``compute_kl``
(KL at theta_t+1).  For the reference's two-hidden-layer ReLU policy that whole sequence is a
fixed list of device launches:

    entropy_gamma -> entropy_reverse_scan                                      (dH/dlogp)
    head_backward -> dh1 GEMM -> layer_backward ; split-K dW2 (forked stream)  (dH/dtheta)
    optim_step (Adam / RMSprop)                                                (theta_t+1)
    policy_forward (layer 1 + GEMM + head, one kernel)                         (logp at t+1)
    iw_forward -> entropy_forward                     (KL at t+1, and H, dH/dW for the next)

The forward at theta_t+1, its importance weights and dH/dW are written into static buffers
that the next replay's backward reads (``_prime`` fills them before the first replay), so one
captured graph replays every iteration and the host only reads the two control scalars
(H, KL) per iteration.  The Adam/RMSprop state lives in the caller's torch optimizer
(``optimizer.state[p]``: ``step``, ``exp_avg``, ``exp_avg_sq`` / ``square_avg``), updated in
place; its per-step scalars (bias corrections, learning rate) are written to a device buffer
before each replay.  After a rejected step the caller restores theta and calls ``refresh()``.

Results equal the eager path (autograd through the same kernels) up to the optimizer's
rounding order; tests/test_gpu_device_loop.py checks both against each other and the oracle.
"""
import math
import os
import weakref

import torch
import torch.nn as nn

from .. import ops
from ..policy import GaussianPolicy

_ADAM, _RMSPROP = 0, 1


def _opt_kind(optimizer):
    if len(optimizer.param_groups) != 1:
        return None
    g = optimizer.param_groups[0]
    if isinstance(g.get("lr"), torch.Tensor) or g.get("weight_decay", 0) != 0 or g.get(
            "maximize", False) or g.get("differentiable", False) or g.get(
            "capturable", False) or g.get("fused", False):
        return None
    if type(optimizer) is torch.optim.Adam:
        if g.get("amsgrad", False) or g.get("decoupled_weight_decay", False):
            return None
        return _ADAM
    if type(optimizer) is torch.optim.RMSprop:
        if g.get("momentum", 0) != 0 or g.get("centered", False):
            return None
        return _RMSPROP
    return None


def supported(batch, behavioral_policy, target_policy, optimizer):
    """True when the iteration can run as a graph: the reference's 2-layer ReLU GaussianPolicy
    (f64, fused-head sizes), a dense particle grid, Adam/RMSprop with MEPOL's settings over
    exactly the target's parameters."""
    if os.environ.get("MEPOL_DEVICE_LOOP", "1") == "0":
        return False
    if not isinstance(target_policy, GaussianPolicy) or target_policy is behavioral_policy:
        return False
    if not (batch.dense and batch.states_flat.is_cuda):
        return False
    if not target_policy._fused_head_ok(batch.states_flat, batch.actions_flat):
        return False
    layers = [m for m in target_policy.net if isinstance(m, nn.Linear)]
    if len(layers) != 2 or target_policy.num_features > 64:
        return False
    params = list(target_policy.parameters())
    if len(params) != 7 or any(p.dtype != torch.float64 or not p.is_contiguous() or
                               p.device != batch.device for p in params):
        return False
    if _opt_kind(optimizer) is None:
        return False
    return [id(p) for p in optimizer.param_groups[0]["params"]] == [id(p) for p in params]


def _scalar_dtype():
    try:
        from torch.optim.optimizer import _get_scalar_dtype

        return _get_scalar_dtype()
    except ImportError:  # pragma: no cover
        return torch.float32


class DeviceIteration:
    """Static buffers + captured graph for one (policy, optimizer, batch shape, k, constants)."""

    def __init__(self, target_policy, optimizer, batch, k, G, B, ns, eps):
        # the cache below is keyed weakly by the target policy: a strong reference here would
        # keep every iteration (its graphs and ~1 GB of static buffers at C3) alive for good
        self._tgt_ref, self.opt = weakref.ref(target_policy), optimizer
        self.kind = _opt_kind(optimizer)
        self.params = list(target_policy.parameters())  # optimizer / state order
        l1, l2 = [m for m in target_policy.net if isinstance(m, nn.Linear)]
        self.named = (l1.weight, l1.bias, l2.weight, l2.bias, target_policy.mean.weight,
                      target_policy.mean.bias, target_policy.log_std)
        self.k, self.G, self.B, self.ns, self.eps = k, float(G), float(B), float(ns), float(eps)
        dev = batch.device
        self.device = dev
        self.N, self.nt, self.T, self.kp1 = batch.N, batch.num_traj, batch.T, batch.kp1
        W1, _, W2, _, Wm, _, _ = self.named
        f64 = dict(dtype=torch.float64, device=dev)
        self.x = torch.empty_like(batch.states_flat)
        self.act = torch.empty_like(batch.actions_flat)
        self.D = torch.empty_like(batch.D)
        self.idx32T = torch.empty_like(batch.idx32T)
        self.offsets = torch.empty_like(batch.offsets)
        self.logp_b = torch.empty((self.nt, self.T), **f64)
        off, rows = batch.csr(k)
        self.csr_off, self.csr_rows = torch.empty_like(off), torch.empty_like(rows)
        self.h1 = torch.empty((self.N, W1.shape[0]), **f64)
        self.z2 = torch.empty((self.N, W2.shape[0]), **f64)
        self.mu = torch.empty((self.N, Wm.shape[0]), **f64)
        self.logp = torch.empty(self.N, **f64)
        self.fused_fwd = (ops.policy_forward_ok(self.x.shape[1], W2.shape[0])
                          and os.environ.get("MEPOL_FUSED_FWD", "1") != "0")
        self.fused_dh1 = (ops.dh1_layer1_ok(self.x.shape[1], W2.shape[0])
                          and os.environ.get("MEPOL_FUSED_DH1", "1") != "0")
        self.neg_one = torch.full((), -1.0, **f64)
        # relu'(h1) as bits, written by the fused forward beside h1 and read by the fused dh1
        # backward in place of h1 (1/64 of the bytes its epilogue waits for)
        self.h1_mask = (ops.h1_mask_buffer(self.N, W1.shape[0], dev)
                        if self.fused_fwd and self.fused_dh1 else None)
        # W2^T only for the dh1 kernel without the mask or with an odd h0 (otherwise dh1 reads
        # W2 as stored, mepol_dh1_layer1_backward_w2)
        self.dh1_w2 = self.h1_mask is not None and W1.shape[0] % 2 == 0
        self.W2t = (torch.empty((W2.shape[1], W2.shape[0]), **f64)
                    if self.fused_dh1 and not self.dh1_w2 else None)
        # every body takes its optimizer step through _optim_step, which leaves theta_t in the
        # replay's shadow (off_policy_optimization then copies it into last_valid only when it
        # needs it, not after every accepted step)
        self.tracks_shadow = True
        # Speculative replay: replay t+1 is launched before the host
        # has read replay t's two scalars, so the GPU never idles on the host's accept/reject
        # decision.  Two captured graphs alternate; each owns its scalar in/out blocks, its
        # shadow of theta and a snapshot of the optimizer moments taken before its step, so a
        # speculative replay can be undone (cancel) when replay t turns out rejected.
        self.speculative = os.environ.get("MEPOL_SPECULATE", "1") != "0"
        self._bufs = [self._make_bufs(dev) for _ in range(2 if self.speculative else 1)]
        self._use(0)
        self._inflight = []   # parities launched and not yet returned by step(), oldest first
        self._next = 0
        self._last = 0        # parity of the replay step() returned last
        self._events = [torch.cuda.Event() for _ in self._bufs]
        self.graphs = [None] * len(self._bufs)
        self.w_cur = torch.zeros(self.N, **f64)   # importance weights of logp(theta_t)
        self.g_cur = torch.zeros(self.N, **f64)   # dH/dW at theta_t
        self.out_cur = torch.zeros(4, **f64)      # entropy_forward sums at theta_t
        # scratch owned by this graph (never the eager per-stream cache, whose buffers can be
        # replaced while a captured graph still holds their addresses)
        self.ws_head = ops.head_workspace(self.N, W2.shape[0], Wm.shape[0], dev)
        self.ws_layer = ops.layer_workspace(self.N, W1.shape[1], W1.shape[0], dev)
        self.ws_dh1 = ops.dh1_layer1_workspace(self.N, W1.shape[0], W1.shape[1], dev)
        self.ws_wgrad = ops.weight_grad_workspace(self.N, W2.shape[0], W2.shape[1], dev)
        self.graph = None
        self.fork = torch.cuda.Stream(device=dev)
        self.s_gemm = torch.cuda.Stream(device=dev)
        self._batch_id = None
        self._init_state()

    @property
    def tgt(self):
        return self._tgt_ref()

    def matches(self, target_policy, optimizer, batch, k, G, B, ns, eps):
        return (target_policy is self.tgt and optimizer is self.opt and batch.N == self.N
                and batch.num_traj == self.nt and batch.T == self.T and batch.kp1 == self.kp1
                and batch.device == self.device and (k, float(G), float(B), float(ns), float(eps))
                == (self.k, self.G, self.B, self.ns, self.eps)
                and batch.states_flat.shape == self.x.shape
                and batch.actions_flat.shape == self.act.shape
                and [p.data_ptr() for p in target_policy.parameters()]
                == [p.data_ptr() for p in self.params])

    def _make_bufs(self, dev):
        f64 = dict(dtype=torch.float64, device=dev)
        # per-replay scalars in and (H, KL) out: pinned host tensors behind graph memcpy nodes
        scal_host = torch.zeros(8, dtype=torch.float64).pin_memory()
        vals_host = torch.zeros(2, dtype=torch.float64).pin_memory()
        scal_np, vals_np = scal_host.numpy(), vals_host.numpy()
        # shadow: theta at the start of the replay = the last accepted parameters (a rejected
        # step is undone by the caller before the next one): off_policy_optimization copies it
        # into last_valid only when it needs it, not after every accepted step
        return dict(scal=torch.zeros(8, **f64), scal_host=scal_host, scal_np=scal_np,
                    vals=torch.zeros(2, **f64), vals_host=vals_host, vals_np=vals_np,
                    shadow=[torch.empty_like(p) for p in self.params], moments=[])

    def _use(self, par):
        """Point the body's scalar blocks / shadows at replay buffer set `par`."""
        b = self._bufs[par]
        self.scal, self.scal_host, self.scal_np = b["scal"], b["scal_host"], b["scal_np"]
        self.vals, self.vals_host, self.vals_np = b["vals"], b["vals_host"], b["vals_np"]
        self.shadow = b["shadow"]
        self._moments = b["moments"]

    @property
    def graph(self):
        return self.graphs[0]

    @graph.setter
    def graph(self, g):
        if g is None:
            self.graphs = [None] * len(self._bufs)
        else:
            self.graphs[0] = g

    def step_start_params(self):
        """theta at the start of the replay step() returned last (the last accepted one)."""
        return self._bufs[self._last]["shadow"]

    # -- optimizer state (kept in the torch optimizer, as torch.optim would) ------------------
    def _init_state(self):
        for p in self.params:
            st = self.opt.state[p]
            if "step" not in st:
                st["step"] = torch.tensor(0.0, dtype=_scalar_dtype())
                if self.kind == _ADAM:
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                else:
                    st["square_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        if self.kind == _ADAM:
            self.m = [self.opt.state[p]["exp_avg"] for p in self.params]
            self.v = [self.opt.state[p]["exp_avg_sq"] for p in self.params]
        else:
            self.m = None
            self.v = [self.opt.state[p]["square_avg"] for p in self.params]
        for t in (self.m or []) + self.v:
            if t.dtype != torch.float64 or not t.is_contiguous() or t.device != self.device:
                raise ValueError("optimizer state is not contiguous f64 on the policy's device")
        for b in self._bufs:
            b["moments"][:] = [torch.empty_like(t) for t in (self.m or []) + self.v]

    def _state_tensors_current(self):
        st = self.opt.state
        if self.kind == _ADAM:
            return all(st[p].get("exp_avg") is m and st[p].get("exp_avg_sq") is v
                       for p, m, v in zip(self.params, self.m, self.v))
        return all(st[p].get("square_avg") is v for p, v in zip(self.params, self.v))

    def _advance_scalars(self):
        """torch.optim's host-side step bookkeeping for one step; returns the device scalars."""
        g = self.opt.param_groups[0]
        steps = [self.opt.state[p]["step"] for p in self.params]
        torch._foreach_add_(steps, 1.0)  # one dispatch instead of one per parameter
        lr = g["lr"]
        h = self.scal_np  # numpy view of the pinned buffer: element writes without dispatch
        h[0] = 1.0
        if self.kind == _ADAM:
            beta1, beta2 = g["betas"]
            step = float(steps[0])
            bc1 = 1 - beta1 ** step
            bc2 = 1 - beta2 ** step
            h[1] = lr / bc1
            h[2] = bc2 ** 0.5
            h[3], h[4], h[5] = beta1, beta2, g["eps"]
        else:
            h[1], h[2], h[3] = lr, g["alpha"], g["eps"]

    # -- the iteration --------------------------------------------------------------------------
    def load(self, batch, logp_b=None):
        """Copy one epoch's particles and cached per-epoch tensors into the static inputs.
        Without logp_b the caller must follow with start_from_behavioral()."""
        off, rows = batch.csr(self.k)
        pairs = [(self.x, batch.states_flat), (self.act, batch.actions_flat), (self.D, batch.D),
                 (self.idx32T, batch.idx32T), (self.offsets, batch.offsets),
                 (self.csr_off, off), (self.csr_rows, rows)]
        if logp_b is not None:
            pairs.append((self.logp_b, logp_b))
        for dst, src in pairs:
            dst.copy_(src)
        self._batch_id = id(batch)

    @torch.no_grad()
    def forward(self):
        """logp of the target at its current parameters into the static buffers (h1, z2, mu
        and logp: the next replay's backward reads the activations)."""
        W1, b1, W2, b2, Wm, bm, ls = self.named
        if self.fused_fwd:  # layer 1 + z2 GEMM + head in one kernel
            ops.policy_forward(self.x, W1, b1, W2, b2, Wm, bm, ls, self.act, self.h1, self.z2,
                               self.mu, self.logp, mask_out=self.h1_mask)
            return
        ops.layer_forward(self.x, W1, b1, out=self.h1)
        torch.mm(self.h1, W2.t(), out=self.z2)
        ops.head_forward(self.z2, Wm, bm, ls, self.act, bz=b2, mu_out=self.mu,
                         logp_out=self.logp)

    def _backward(self, grad, outs=None, after_dW2=None):
        """(dW1, db1, dW2, db2, dWm, dbm, dls) from dH/dlogp: the _TwoLayerLogp backward.
        `outs`: optional tensors of those seven shapes the kernels write into (the sharded
        iteration passes views of its flat all-reduce buffer: no concatenation launch).
        `after_dW2`: optional callable issued on the dW2 stream once dW2 and the head gradients
        are written, concurrent with the dh1 / layer-1 backward (the sharded iteration starts
        that bucket's all-reduce there).

        Head backward, then dW2 (split-K f64 MFMA, csrc/wgrad.hip, forked stream) concurrent with the fused
        dh1 -> layer-1 backward (measured: faster than dh1 first with dW2 overlapping the
        layer-1 backward, and than splitting dW2 across both phases)."""
        W1, b1, W2, b2, Wm, bm, ls = self.named
        cur = torch.cuda.current_stream()
        # W2^T for the fused dh1 kernel when it cannot read W2 as stored (round 6: with the
        # forward's mask it does, mepol_dh1_layer1_backward_w2, and this copy node is gone)
        w2_direct = self.fused_dh1 and self.dh1_w2
        if self.fused_dh1 and not w2_direct:
            self.W2t.copy_(W2.t())
        W2t = self.W2t if self.fused_dh1 and not w2_direct else None
        self.fork.wait_stream(cur)
        self.s_gemm.wait_stream(cur)
        o = outs if outs is not None else (None,) * 7
        head_outs = None if outs is None else (o[4], o[5], o[6], o[3])
        # only the head's row kernel (dz2) is on the critical path: its parameter-gradient
        # reduces run on the dW2 stream after dW2, under the longer dh1 backward (round 6;
        # ahead of dW2 they delayed it behind dh1's workgroups: iteration +46 us at C3R8)
        dz2, dWm, dbm, dls, db2, head_reduce = ops.head_backward(
            grad, self.z2, Wm, ls, self.act, self.mu, bz=b2, need_dz=True, ws=self.ws_head,
            outs=head_outs, defer_reduce=True)
        e_h = torch.cuda.Event()
        e_h.record(cur)
        self.fork.wait_event(e_h)
        with torch.cuda.stream(self.fork):
            dW2 = ops.weight_grad(dz2, self.h1, out=o[2], ws=self.ws_wgrad)  # csrc/wgrad.hip
            head_reduce()
            if after_dW2 is not None:
                after_dW2()
        self.s_gemm.wait_event(e_h)
        with torch.cuda.stream(self.s_gemm):
            if self.fused_dh1:  # dh1 stays on chip (csrc/gemm.hip)
                dh1 = None
                dW1, db1 = ops.dh1_layer1_backward(dz2, W2t, self.h1, self.x, ws=self.ws_dh1,
                                                   mask=self.h1_mask,
                                                   dW_out=o[0], db_out=o[1],
                                                   w2=W2 if w2_direct else None)
            else:
                dh1 = torch.mm(dz2, W2)
                dW1, db1 = ops.layer_backward(dh1, self.h1, self.x, ws=self.ws_layer)
                if outs is not None:
                    o[0].copy_(dW1)
                    o[1].copy_(db1)
                    dW1, db1 = o[0], o[1]
        cur.wait_stream(self.fork)
        cur.wait_stream(self.s_gemm)
        del dz2, dh1
        return dW1, db1, dW2, db2, dWm, dbm, dls

    @torch.no_grad()
    def _body(self):
        W1, b1, W2, b2, Wm, bm, ls = self.named
        nt, T, N, k = self.nt, self.T, self.N, self.k
        lt = self.logp.view(nt, T)
        self._scal_in()
        # dH/dlogp at theta_t (loss.backward, mepol.py:273-278) from the importance weights and
        # dH/dW that the previous replay (or _prime) left for logp(theta_t)
        w, g = self.w_cur, self.g_cur
        gamma, partials, nparts = ops.entropy_gamma(g, w, self.csr_off, self.csr_rows)
        grad = ops.entropy_reverse_scan(gamma, w, partials, nparts, self.offsets, nt, T,
                                        self.neg_one)
        # through the policy (the _TwoLayerLogp backward)
        dW1, db1, dW2, db2, dWm, dbm, dls = self._backward(grad.view(-1))
        # optimizer.step() (mepol.py:280)
        grad_of = {id(p): g for p, g in zip(self.named, (dW1, db1, dW2, db2, dWm, dbm, dls))}
        self._optim_step([grad_of[id(p)] for p in self.params])
        # compute_kl at theta_t+1 (mepol.py:435, :157-174).  The pass with the entropy
        # constants also yields the KL sum (its terms do not depend on them) and the next
        # iteration's H(theta_t+1) and dH/dW, so each replay needs one weights pass, not two.
        # (w_cur and g_cur were last read by this replay's gamma / reverse scan, above)
        self.forward()
        ops.iw_forward(lt, self.logp_b, self.offsets, N, w_out=self.w_cur)
        # (H(theta_t), KL(theta_t+1)) into vals by the entropy pass itself, theta_t+1's sums
        # kept in out_cur for the next replay, then vals to the host
        ops.entropy_forward(self.w_cur, self.idx32T, self.D, k, self.ns, self.G, self.B,
                            self.eps, g_out=self.g_cur, out4=self.out_cur, vals=self.vals)
        ops.memcpy_async(self.vals_host, self.vals)

    def _optim_step(self, grads):
        """optimizer.step() (mepol.py:280).  The kernel also leaves theta_t in the replay's
        shadow and, when speculative, the moments before the step (cancel restores them),
        without separate copy launches."""
        nm = len(self.m) if self.m is not None else 0
        snap = (self.shadow, self._moments[:nm] if (self.speculative and nm) else None,
                self._moments[nm:] if self.speculative else None)
        ops.optim_step(self.kind, self.params, grads, self.m, self.v, self.scal, snapshot=snap)

    # The replay's scalar inputs (enable flag, lr and bias corrections) come from, and its two
    # control outputs go to, pinned host buffers through memcpy nodes of the graph itself.
    def _scal_in(self):
        ops.memcpy_async(self.scal, self.scal_host)

    def _emit(self, a, ia, b, ib, cur, nw, n):
        """vals_host <- (a[ia], b[ib]) through a memcpy node; cur[:n] <- nw[:n]."""
        if not (a is self.vals and b is self.vals and (ia, ib) == (0, 1)):
            torch.stack((a[ia], b[ib]), out=self.vals)
        cur[:n].copy_(nw[:n])
        ops.memcpy_async(self.vals_host, self.vals)

    @torch.no_grad()
    def _prime(self):
        """w, dH/dW and H for logp(theta) of the current parameters (before the first replay
        and after a rejected step restored theta)."""
        lt = self.logp.view(self.nt, self.T)
        _, _, w, _ = ops.iw_forward(lt, self.logp_b, self.offsets, self.N)
        out, _, g = ops.entropy_forward(w, self.idx32T, self.D, self.k, self.ns, self.G, self.B,
                                        self.eps)
        self.w_cur.copy_(w)
        self.g_cur.copy_(g)
        self.out_cur.copy_(out)

    def refresh(self):
        """Recompute the iteration's inputs that depend on theta: the forward (h1, z2, mu and
        logp, which the next replay's backward reads) and w, dH/dW."""
        self.forward()
        self._prime()

    def start_from_behavioral(self):
        """Epoch start with the target holding the behavioral parameters (mepol.py:409, 493):
        one forward fills h1/z2/mu/logp for the first replay's backward and is also the epoch's
        behavioral logp_b (the same parameters).  Returns logp_b [nt, T]."""
        self.forward()
        self.logp_b.view(-1).copy_(self.logp)
        self._prime()
        return self.logp_b

    def logp_of_last_step(self):
        """logp at the parameters of the last step() result's theta_t+1, i.e. the final
        accepted parameters.  Valid only when no replay is in flight and that step was the
        last one launched (no speculative replay has overwritten the forward buffers)."""
        if self._inflight or (self._last + 1) % len(self._bufs) != self._next:
            raise RuntimeError("the forward buffers do not hold the last step's parameters")
        return self.logp

    def _warmup(self):
        """One eager pass on a side stream (allocator pools, library handles, kernel code)."""
        cur = torch.cuda.current_stream()
        self._side = torch.cuda.Stream(device=self.device)
        self.scal_np[:] = 0.0  # enable = 0: the warm-up pass leaves theta and the moments alone
        self._side.wait_stream(cur)
        with torch.cuda.stream(self._side):
            self._body()
        cur.wait_stream(self._side)
        # the pass read the pinned scalar block asynchronously: it must have done so before
        # the host writes the first real step's values into it
        self._side.synchronize()

    def _capture_graph(self):
        cur = torch.cuda.current_stream()
        graphs = []
        for par in range(len(self._bufs)):
            self._use(par)
            graph = torch.cuda.CUDAGraph()
            # thread-local capture: a capture in "global" mode makes other threads' HIP calls
            # fail, and ProcessGroupNCCL's watchdog thread queries the events of earlier eager
            # collectives at any time (an error there aborts the process)
            with torch.cuda.graph(graph, stream=self._side, capture_error_mode="thread_local"):
                self._body()
            graphs.append(graph)
        cur.wait_stream(self._side)
        self._use(0)
        self.graphs = graphs

    def _capture(self):
        self._warmup()
        self._capture_graph()

    def _launch(self):
        par = self._next
        self._use(par)
        self._advance_scalars()  # into the pinned block the graph copies in
        self.graphs[par].replay()
        self._events[par].record()
        self._inflight.append(par)
        self._next = (par + 1) % len(self._bufs)

    def step(self, speculate=False):
        """policy_update + compute_kl.  Returns host floats (H(theta_t), KL(theta_t+1)
        unclamped); the target policy's parameters and the optimizer state are updated.

        speculate=True: the caller will run another step if this one is accepted, so that
        step is launched now, before this one's scalars are read; the next step() returns
        its results.  If this step is rejected instead, the caller must cancel() first."""
        if not self._inflight:
            if not self._state_tensors_current():
                self._init_state()
                self.graph = None
            if self.graph is None:
                self._capture()
            self._launch()
        par = self._inflight.pop(0)
        if speculate and self.speculative and not self._inflight:
            self._launch()
        self._events[par].synchronize()
        self._last = par
        v = self._bufs[par]["vals_np"]
        return float(v[0]), float(v[1])

    @torch.no_grad()
    def cancel(self):
        """Undo a speculative replay still in flight: wait for it and restore theta, the
        optimizer moments and the step count it advanced (as they were after the rejected
        step; the caller then restores the last accepted theta from step_start_params())."""
        while self._inflight:
            par = self._inflight.pop()
            self._events[par].synchronize()
            torch._foreach_copy_((self.m or []) + self.v, self._bufs[par]["moments"])
            torch._foreach_copy_(self.params, self._bufs[par]["shadow"])
            torch._foreach_add_([self.opt.state[p]["step"] for p in self.params], -1.0)
            self._next = par


    def release(self):
        """Wait for replays in flight and free the captured graphs (before the process group
        whose collectives a sharded graph captured is destroyed)."""
        if self._inflight:
            self.cancel()
        for g in self.graphs:
            if g is not None:
                g.reset()
        self.graph = None


_CACHE = weakref.WeakKeyDictionary()  # target policy -> DeviceIteration


def get(target_policy, optimizer, batch, k, G, B, ns, eps):
    """The cached DeviceIteration for these arguments (one per target policy)."""
    it = _CACHE.get(target_policy)
    if it is None or not it.matches(target_policy, optimizer, batch, k, G, B, ns, eps):
        it = None  # drop the old graph and buffers before allocating new ones
        _CACHE.pop(target_policy, None)
        it = DeviceIteration(target_policy, optimizer, batch, k, G, B, ns, eps)
        _CACHE[target_policy] = it
    return it


def kl_flags(H, KL):
    """(loss, loss_numeric_error, kl (clamped as torch.clamp_min), kl_numeric_error)."""
    loss = -H
    kl = KL if not (KL < 0.0) else 0.0
    return loss, not math.isfinite(loss), kl, not math.isfinite(KL)
