"""Particle-batch data parallelism over ranks (one process per GPU, RCCL over xGMI).

The reference scales the rollout with joblib worker processes (src/algorithms/mepol.py:179-187)
and the k-NN with sklearn threads (:190); everything else is one process.  Here the particle
batch is sharded by trajectory over `world` ranks (rank r owns trajectories
[r*nt/G, (r+1)*nt/G) = particles [R0, R1) in the reference's traj-major order):

  once per epoch   all-gather next-states (f32)            -> every rank holds all N candidates
                   k-NN of the rank's own queries           -> D, I for particles [R0, R1)
                   all-gather I[:, :k] (int32)              -> CSR of "who has me as neighbour"
                                                               for the rank's own particles
  per forward      sum of u: all-gather G partial sums      (fixed-order sum, identical bits)
                   all-gather w                             (N f64: the gather reads any index)
                   entropy/KL raw sums: all-gather G pairs
  per backward     all-gather g = dH/dW                      (N f64)
                   S = sum gamma_j w_j: all-gather G partials
                   policy gradients: one all-reduce of the flattened f64 grads
so every rank holds the same H, KL and parameters and takes the same accept/backtrack branch
(mepol.py:441-476).  Payloads are 1.6 MB per vector at N = 200k: latency-bound on xGMI.

The kernels come from `ops` (the HIP library).  Tests may inject another object with the same
functions to check this module's collective algebra on CPU with the gloo backend.
"""
import os
import weakref

import torch

from . import ops as _hip_ops
from .algorithms.device_loop import DeviceIteration


def prepare_nccl_env():
    """Call before init_process_group("nccl") in a process that captures collectives
    (ShardedIteration.try_capture).  ProcessGroupNCCL recycles the HIP events of finished works
    (TORCH_NCCL_CUDA_EVENT_CACHE); an event last recorded inside a graph capture can then reach
    the watchdog thread, whose query fails with hipErrorCapturedEvent and aborts the process.
    Without the cache every work gets fresh events.  A caller's explicit setting wins."""
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")


def release_graphs():
    """Free every captured sharded iteration.  Its graphs hold RCCL collectives recorded on the
    process group's communicator: they must be gone (and nothing of theirs in flight) before
    that communicator is torn down, or RCCL's threads meet a destroyed communicator."""
    its = list(_SHARDED_CACHE.values())
    if its:
        torch.cuda.synchronize()
        for it in its:
            it.release()
        torch.cuda.synchronize()
    _SHARDED_CACHE.clear()
    _GRAPH_STATE.clear()


def destroy_process_group(dist, group=None):
    """release_graphs(), then dist.destroy_process_group(group): the teardown every caller of
    the sharded path uses (CLI, bench, tests)."""
    release_graphs()
    if group is None:
        dist.destroy_process_group()
    else:
        dist.destroy_process_group(group)


class ShardedEpoch:
    def __init__(self, states, actions, real_traj_lengths, next_states_f32, k, dist, group=None,
                 ops=None):
        self.dist = dist
        self.group = group
        self.ops = ops if ops is not None else _hip_ops
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.states = states
        self.actions = actions
        self.nt, self.T = actions.shape[0], actions.shape[1]
        self.dev = states.device
        lens = real_traj_lengths.reshape(-1).to(torch.int64).cpu()
        if not bool((lens == self.T).all()):
            raise NotImplementedError("sharded epochs need full-length trajectories (ErgodicEnv)")
        self.n_local = self.nt * self.T
        self.N = self.n_local * self.world
        self.R0 = self.rank * self.n_local
        off = torch.arange(self.nt + 1, dtype=torch.int64) * self.T
        self.offsets = off.to(self.dev)
        nf = states.shape[-1]
        self.states_flat = states[:, : self.T].reshape(self.n_local, nf).contiguous()
        self.actions_flat = actions.reshape(self.n_local, -1).contiguous()
        self.next_states = next_states_f32.contiguous()
        self.k = k
        self._logp_b = None
        self._stash = None

    # -- collectives (fixed-order reductions: every rank computes bit-identical values) --------
    def _gather(self, t):
        """[world, *t.shape] stack of every rank's t (concatenated-form all_gather_into_tensor)."""
        shape = tuple(t.shape)
        flat = t.contiguous().reshape(-1)
        out = torch.empty(self.world * flat.numel(), dtype=t.dtype, device=t.device)
        self.dist.all_gather_into_tensor(out, flat, group=self.group)
        return out.reshape((self.world,) + shape)

    def _sum(self, t):
        return self._gather(t).sum(0)

    # -- per-epoch setup ------------------------------------------------------------------------
    def build_knn(self):
        cand = self._gather(self.next_states).reshape(self.N, -1)
        D, I, idx32T, check = self.ops.knn(cand, self.k + 1, query=self.next_states,
                                           defer_check=True)
        idx_all = self._gather(idx32T[: self.k].contiguous())       # [G, k, n_local]
        idx_allT = idx_all.permute(1, 0, 2).reshape(self.k, self.N).contiguous()
        csr = self.ops.csr_build(idx_allT, self.k, self.n_local, col_offset=self.R0,
                                 row_offset=0, nq=self.N)
        # The input check is read only now, with the gather and the CSR build queued behind
        # the k-NN (one host wait less in the epoch set-up).  A rejected input (a NaN / inf
        # coordinate) is rejected on every rank alike -- the check covers the gathered
        # candidates, which every rank holds -- so all ranks issued the same gather and all
        # raise here; the k-NN kernels returned early, the gathered rows are undefined and the
        # CSR build (which bounds-checks its ids) is discarded with them.  The epoch's
        # attributes are assigned only after the check passed: a caller that catches the error
        # never sees undefined neighbour tables.
        check.raise_if_invalid()
        self.D, self.I, self.idx32T, self.csr = D, I, idx32T, csr
        return self.D, self.I

    # -- policy log-probs -----------------------------------------------------------------------
    def _logp(self, policy):
        return policy.get_log_p(self.states_flat, self.actions_flat).reshape(self.nt, self.T)

    def behavioral_logp(self, policy):
        from .algorithms.particles import _param_key

        key = _param_key(policy)
        if self._logp_b is None or self._logp_b[0] != key:
            with torch.no_grad():
                self._logp_b = (key, self._logp(policy).detach())
        return self._logp_b[1]

    def seed_behavioral_logp(self, policy, logp):
        """Cache `logp` (computed at the policy's current parameters) as its behavioral
        log-probabilities (ParticleBatch.seed_behavioral_logp)."""
        from .algorithms.particles import _param_key

        with torch.no_grad():
            self._logp_b = (_param_key(policy), logp.detach().reshape(self.nt, self.T).clone())

    def _logps(self, beh, tgt):
        from .algorithms.particles import _param_key

        lb = self.behavioral_logp(beh)
        if tgt is beh:
            return lb, lb
        if torch.is_grad_enabled() and self._stash is not None:
            key, lt = self._stash
            self._stash = None
            if key == _param_key(tgt):
                return lt, lb
        return self._logp(tgt), lb

    # -- forward pieces -------------------------------------------------------------------------
    def weights(self, logp_t, logp_b):
        u, ts, _, _ = self.ops.iw_forward(logp_t.detach(), logp_b.detach(), self.offsets,
                                          self.n_local, normalize=False)
        U = self._sum(ts.sum().reshape(1)).reshape(())
        w_local = self.ops.iw_normalize(u, U)
        return w_local, self._gather(w_local).reshape(self.N)

    def entropy_sums(self, w_global, k, G, B, ns, eps):
        out4, _, g = self.ops.entropy_forward(w_global, self.idx32T, self.D, k, ns, G, B, eps,
                                              n_w=self.N)
        sums = self._sum(out4[2:4].contiguous())
        H = -sums[0] + B
        KL = sums[1] / self.N
        return H, KL, g

    # -- drop-in equivalents of the module-level functions ------------------------------------
    def _entropy(self, beh, tgt, k, G, B, ns, eps):
        lt, lb = self._logps(beh, tgt)
        return _ShardedEntropy.apply(lt, lb, self, k, G, B, ns, eps)

    def compute_entropy(self, beh, tgt, k, G, B, ns, eps):
        """H on the host, as the module-level compute_entropy returns it (mepol.py:367-368)."""
        return self._entropy(beh, tgt, k, G, B, ns, eps).cpu()

    def compute_kl_deferred(self, beh, tgt, k, eps):
        from .algorithms.particles import _param_key

        lb = self.behavioral_logp(beh)
        if tgt is beh:
            lt = lb
        elif torch.is_grad_enabled() and any(p.requires_grad for p in tgt.parameters()):
            lt = self._logp(tgt)
            self._stash = (_param_key(tgt), lt)
        else:
            with torch.no_grad():
                lt = self._logp(tgt)
        with torch.no_grad():
            _, wg = self.weights(lt, lb)
            _, KL, _ = self.entropy_sums(wg, k, 1.0, 0.0, 1.0, eps)
        kl = KL.clone()
        return torch.clamp_min(kl, 0.0), ~torch.isfinite(kl)

    def compute_kl(self, beh, tgt, k, eps):
        kl, flag = self.compute_kl_deferred(beh, tgt, k, eps)
        return kl.cpu(), bool(flag)  # host tensor, as the module-level compute_kl

    def allreduce_grads(self, params):
        grads = [p.grad for p in params if p.grad is not None]
        if not grads:
            return
        flat = torch.cat([g.reshape(-1) for g in grads])
        self.dist.all_reduce(flat, group=self.group)
        o = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[o:o + n].view_as(g))
            o += n

    def policy_update_deferred(self, optimizer, beh, tgt, k, G, B, ns, eps):
        optimizer.zero_grad()
        loss = -self._entropy(beh, tgt, k, G, B, ns, eps)
        flag = ~torch.isfinite(loss.detach())
        loss.backward()
        self.allreduce_grads(list(tgt.parameters()))
        optimizer.step()
        return loss, flag

    def policy_update(self, optimizer, beh, tgt, k, G, B, ns, eps):
        loss, flag = self.policy_update_deferred(optimizer, beh, tgt, k, G, B, ns, eps)
        return loss.detach().cpu(), bool(flag)  # host tensor, as the module-level policy_update

    def off_policy_optimization(self, optimizer, beh, tgt, last_valid, G, B, ns, eps,
                                kl_threshold, max_off_iters, use_backtracking, backtrack_coeff,
                                max_backtrack_try, original_lr, on_accept=None):
        from .algorithms.mepol import off_policy_optimization

        k = self.k

        class _Fns:
            @staticmethod
            def policy_update(opt, b, t, *a):
                return self.policy_update(opt, b, t, k, G, B, ns, eps)

            @staticmethod
            def compute_kl(b, t, *a):
                return self.compute_kl(b, t, k, eps)

            @staticmethod
            def policy_update_deferred(opt, b, t, *a):
                return self.policy_update_deferred(opt, b, t, k, G, B, ns, eps)

            @staticmethod
            def compute_kl_deferred(b, t, *a):
                return self.compute_kl_deferred(b, t, k, eps)

            @staticmethod
            def compute_entropy(b, t, *a):
                return self.compute_entropy(b, t, k, G, B, ns, eps)

            @staticmethod
            def make_device_loop(opt, b, t):
                return self.device_loop(opt, b, t, G, B, ns, eps)

            @staticmethod
            def seed_behavioral_logp(policy, logp):
                self.seed_behavioral_logp(policy, logp)

        return off_policy_optimization(optimizer, beh, tgt, last_valid, None, None, self.nt, None,
                                       None, None, k, G, B, ns, eps, kl_threshold, max_off_iters,
                                       use_backtracking, backtrack_coeff, max_backtrack_try,
                                       original_lr, on_accept, fns=_Fns)


    # -- graph-replayed iteration (the sharded form of algorithms/device_loop.py) --------------
    def device_loop(self, optimizer, beh, tgt, G, B, ns, eps):
        """A ShardedIteration ready for this epoch, or None (eager path).  Every rank takes the
        same decision: support is a function of identical arguments, and a failed graph capture
        on any rank turns the graph path off on all of them (all-reduce MIN of a flag)."""
        from .algorithms import device_loop as DL

        view = _LocalView(self)
        if not DL.supported(view, beh, tgt, optimizer) or _GRAPH_STATE.get("disabled"):
            return None
        if self.dist.get_backend(self.group) != "nccl":  # only RCCL collectives can be captured
            return None
        if self.dist is torch.distributed and os.environ.get("TORCH_NCCL_CUDA_EVENT_CACHE") != "0":
            # the group recycles events across capture and eager use (prepare_nccl_env): a
            # captured graph would put the watchdog thread at risk, so stay eager
            if not _GRAPH_STATE.get("warned"):
                import warnings

                warnings.warn("sharded iteration runs eagerly: call parallel.prepare_nccl_env() "
                              "before init_process_group('nccl') to enable graph replay")
                _GRAPH_STATE["warned"] = True
            return None
        it = _SHARDED_CACHE.get(tgt)
        if it is None or not it.matches_epoch(tgt, optimizer, self, G, B, ns, eps):
            _SHARDED_CACHE.pop(tgt, None)
            it = ShardedIteration(tgt, optimizer, self, G, B, ns, eps)
            _SHARDED_CACHE[tgt] = it
        from .algorithms.mepol import _same_params

        # At an epoch's start the target holds the behavioral parameters (mepol.py:409, 493):
        # one forward into the loop's buffers is logp_b and the first replay's activations.
        same = _same_params(tgt, beh)
        it.attach(self, None if same else self.behavioral_logp(beh))
        if same:
            self.seed_behavioral_logp(beh, it.start_from_behavioral())
        if it.graph is None and not it.try_capture():
            _GRAPH_STATE["disabled"] = True
            _SHARDED_CACHE.pop(tgt, None)
            return None
        if not same:
            it.refresh()
        return it


class _LocalView:
    """The rank's shard seen through the batch interface DeviceIteration reads."""

    def __init__(self, ep):
        self.device = ep.dev
        self.N = ep.n_local
        self.num_traj = ep.nt
        self.T = ep.T
        self.kp1 = ep.D.shape[1]
        self.states_flat = ep.states_flat
        self.actions_flat = ep.actions_flat
        self.D = ep.D
        self.idx32T = ep.idx32T
        self.offsets = ep.offsets
        self.dense = True
        self._csr = ep.csr

    def csr(self, k):
        return self._csr


_SHARDED_CACHE = weakref.WeakKeyDictionary()  # target policy -> ShardedIteration
_GRAPH_STATE = {}


class ShardedIteration(DeviceIteration):
    """policy_update + compute_kl of a ShardedEpoch as one graph with the one-rank iteration's
    single-pass structure: the forward at theta_t+1 yields KL(theta_t+1) and the next replay's
    H(theta_t+1) and dH/dW, kept in static buffers (``_prime`` fills them before the first replay
    and after a rejected step).  Collectives per replay (every rank issues the same sequence):

      1. all-gather of the gamma kernel's block partials of S = sum_j gamma_j w_j (<= 2048 f64)
      2. all-reduce of the flattened policy gradients, in two buckets: W2 / head (~0.97 MB at
         C3, issued on the dW2 stream under the dh1 backward) and W1 / b1 (~0.1 MB)
      3. all-gather of [u (n_local), trajectory sums]: weights + normaliser terms (n_local + nt)
      4. all-gather of [dH/dW (n_local), H, KL, H-sum, KL-sum]                 (n_local + 4 f64)

    Reductions over ranks are fixed-order sums of gathered values, so every rank holds the same
    bits and takes the same accept/backtrack branch (mepol.py:441-476).  The gathered blocks are
    read where they land: the weights are normalised straight out of the gather buffer
    (mepol_iw_normalize_gathered), the gamma kernel reads dH/dW there through CSR row ids
    remapped once per epoch to that layout, the reverse scan sums the gathered S partials, the
    entropy pass writes its sums into the block it sends, the backward kernels write the
    gradients into views of a persistent flat buffer that is all-reduced in place, and one
    launch (mepol_sharded_emit) forms the control scalars."""

    def __init__(self, tgt, optimizer, ep, G, B, ns, eps):
        super().__init__(tgt, optimizer, _LocalView(ep), ep.k, G, B, ns, eps)
        self.dist, self.group, self.world = ep.dist, ep.group, ep.world
        self.N_global = ep.N
        self.R0 = ep.R0
        self.ep = ep
        f64 = dict(dtype=torch.float64, device=self.device)
        n, W = self.N, self.world
        self.nparts = self.ep.ops.entropy_gamma_nparts(n)
        self.xs_all = torch.zeros(W * self.nparts, **f64)  # every rank's gamma block partials
        self.xu = torch.zeros(n + self.nt, **f64)         # [u | trajectory sums]
        self.xu_all = torch.zeros(W * (n + self.nt), **f64)
        self.xg = torch.zeros(n + 4, **f64)               # [dH/dW | H, KL, H-sum, KL-sum]
        self.xg_all = torch.zeros(W * (n + 4), **f64)     # dH/dW at theta_t of every particle
        self.w_glob = torch.zeros(self.N_global, **f64)   # importance weights at theta_t
        self.sums_cur = torch.zeros(2, **f64)             # [H-sum, KL-sum] at theta_t
        self.csr_rows_x = torch.empty_like(self.csr_rows)  # CSR ids in the xg_all layout
        # flat gradient buffer (all-reduced in place) and its per-parameter views, in the
        # optimizer's parameter order; the backward kernels write straight into the views
        sizes = [p.numel() for p in self.params]
        self.flat_grad = torch.zeros(sum(sizes), **f64)
        self.grad_views, o = [], 0
        for p, sz in zip(self.params, sizes):
            self.grad_views.append(self.flat_grad[o:o + sz].view_as(p))
            o += sz
        view_of = {id(p): v for p, v in zip(self.params, self.grad_views)}
        self.grad_outs = tuple(view_of[id(p)] for p in self.named)
        # Two all-reduce buckets when the flat layout allows: [W2, b2, Wm, bm, log_std] (ready
        # when the dW2 GEMM ends) reduced on the dW2 stream while the dh1 / layer-1 backward
        # still runs, then [W1, b1].  Needs those five as one contiguous tail of flat_grad.
        self.tail_off = None
        offs = {id(p): v.data_ptr() for p, v in zip(self.params, self.grad_views)}
        base = self.flat_grad.data_ptr()
        first_tail = min(offs[id(p)] for p in self.named[2:]) - base
        head_end = max(offs[id(p)] + p.numel() * 8 for p in self.named[:2]) - base
        if head_end <= first_tail and first_tail % 8 == 0:
            t0 = first_tail // 8
            tail_elems = sum(p.numel() for p in self.named[2:])
            if t0 + tail_elems == self.flat_grad.numel() and t0 == sum(p.numel()
                                                                      for p in self.named[:2]):
                self.tail_off = t0

    def matches_epoch(self, tgt, optimizer, ep, G, B, ns, eps):
        return (self.matches(tgt, optimizer, _LocalView(ep), ep.k, G, B, ns, eps)
                and ep.N == self.N_global and ep.world == self.world and ep.R0 == self.R0
                and ep.dist is self.dist and ep.group is self.group)

    def attach(self, ep, logp_b=None):
        self.ep = ep
        self.load(_LocalView(ep), logp_b)

    def load(self, batch, logp_b=None):
        super().load(batch, logp_b)
        # global particle id j -> its dH/dW in xg_all: rank j // n, block stride n + 4
        n, rows = self.N, self.csr_rows
        torch.add(torch.div(rows, n, rounding_mode="floor") * (n + 4), torch.remainder(rows, n),
                  out=self.csr_rows_x)

    def _gather_into(self, out, t):
        self.dist.all_gather_into_tensor(out, t, group=self.group)

    def _fwd_exchange(self):
        """Weights, dH/dW and the raw entropy / KL sums of self.logp (the last forward) over all
        ranks: collectives 3 and 4.  w_glob and xg_all are overwritten."""
        ops, n, W = self.ep.ops, self.N, self.world
        lt = self.logp.view(self.nt, self.T)
        ops.iw_forward(lt, self.logp_b, self.offsets, n, normalize=False, u_out=self.xu[:n],
                       ts_out=self.xu[n:])
        self._gather_into(self.xu_all, self.xu)
        ops.iw_normalize_gathered(self.xu_all, W, n, self.nt, self.w_glob)
        ops.entropy_forward(self.w_glob, self.idx32T, self.D, self.k, self.ns, self.G, self.B,
                            self.eps, n_w=self.N_global, g_out=self.xg[:n], out4=self.xg[n:])
        self._gather_into(self.xg_all, self.xg)

    @torch.no_grad()
    def _prime(self):
        self._fwd_exchange()
        # sums_cur <- the gathered sums (vals is rewritten by the next replay before it is read)
        self.ep.ops.sharded_emit(self.xg_all, self.world, self.N + 4, self.N + 2, self.B,
                                 self.N_global, self.sums_cur, self.vals)

    @torch.no_grad()
    def _body(self):
        self._scal_in()
        ops = self.ep.ops
        nt, T, n = self.nt, self.T, self.N
        # dH/dlogp at theta_t (_ShardedEntropy.backward) from the weights / dH/dW the previous
        # replay (or _prime) left
        w_local = self.w_glob[self.R0:self.R0 + n]
        gamma, partials, nparts = ops.entropy_gamma(self.xg_all, w_local, self.csr_off,
                                                    self.csr_rows_x)
        assert nparts == self.nparts
        # every rank's block partials of S = sum_j gamma_j w_j; the reverse scan sums all of
        # them in one fixed order (the same bits on every rank)
        self._gather_into(self.xs_all, partials[:nparts])
        grad = ops.entropy_reverse_scan(gamma, w_local, self.xs_all, self.world * nparts,
                                        self.offsets, nt, T, self.neg_one)
        # ShardedEpoch.allreduce_grads: in two buckets when the layout allows (see __init__)
        if self.tail_off is not None:
            tail = self.flat_grad[self.tail_off:]
            self._backward(grad.view(-1), outs=self.grad_outs,
                           after_dW2=lambda: self.dist.all_reduce(tail, group=self.group))
            self.dist.all_reduce(self.flat_grad[:self.tail_off], group=self.group)
        else:
            self._backward(grad.view(-1), outs=self.grad_outs)
            self.dist.all_reduce(self.flat_grad, group=self.group)
        self._optim_step(self.grad_views)
        # KL at theta_t+1 (ShardedEpoch.compute_kl); H(theta_t+1) and dH/dW for the next replay
        self.forward()
        self._fwd_exchange()
        # vals = (H(theta_t), KL(theta_t+1)), sums_cur = theta_t+1's sums, vals to the host
        ops.sharded_emit(self.xg_all, self.world, n + 4, n + 2, self.B, self.N_global,
                         self.sums_cur, self.vals)
        ops.memcpy_async(self.vals_host, self.vals)

    def step(self, speculate=False):
        H, KL = super().step(speculate)
        if os.environ.get("MEPOL_CHECK_RANKS") == "1":
            self.check_ranks_agree(H, KL)
        return H, KL

    def check_ranks_agree(self, H, KL):
        """Debug mode (MEPOL_CHECK_RANKS=1): every rank must read bit-identical (H, KL), or the
        ranks could take different accept / backtrack branches and, after a cancel(), issue
        different collective sequences.  All-gathers the bit patterns (NaN-safe) and raises."""
        bits = torch.tensor([H, KL], dtype=torch.float64, device=self.device).view(torch.int64)
        allb = torch.empty(self.world * 2, dtype=torch.int64, device=self.device)
        self.dist.all_gather_into_tensor(allb, bits, group=self.group)
        rows = allb.view(self.world, 2).cpu()
        if not bool((rows == rows[0]).all()):
            raise RuntimeError(f"ranks disagree on (H, KL): {rows.view(torch.float64).tolist()}")

    def try_capture(self):
        """Capture the iteration; all ranks agree on graph or eager.  The warm-up pass issues
        real collectives, so it runs outside the fallback: a failure there is an error on that
        rank (raised), not a reason to fall back, because the other ranks would otherwise wait
        in a collective it never joins.  Only the capture itself -- collectives are recorded,
        not executed -- may fail over to the eager path, by consensus (MIN of a flag)."""
        self._warmup()
        ok = 1
        try:
            self._capture_graph()
        except Exception as e:  # capture unsupported here: every rank falls back together
            import warnings

            warnings.warn(f"sharded iteration capture failed, running eagerly: {e!r}")
            self.graph = None
            ok = 0
            torch.cuda.synchronize()
        flag = torch.tensor([ok], dtype=torch.int32, device=self.device)
        self.dist.all_reduce(flag, op=self.dist.ReduceOp.MIN, group=self.group)
        if int(flag.item()) == 0:
            self.graph = None
            return False
        return True


class _ShardedEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logp_t, logp_b, ep, k, G, B, ns, eps):
        w_local, w_global = ep.weights(logp_t, logp_b)
        H, _, g = ep.entropy_sums(w_global, k, G, B, ns, eps)
        ctx.ep = ep
        ctx.save_for_backward(w_local, g)
        return H.clone()

    @staticmethod
    def backward(ctx, grad_H):
        ep = ctx.ep
        w_local, g = ctx.saved_tensors
        g_global = ep._gather(g).reshape(ep.N)
        off, rows = ep.csr
        gamma, partials, nparts = ep.ops.entropy_gamma(g_global, w_local, off, rows)
        S = ep._sum(partials[:nparts].sum().reshape(1)).reshape(())
        gH = grad_H.reshape(()).to(torch.float64).contiguous()
        grad = ep.ops.entropy_reverse_scan(gamma, w_local, partials, nparts, ep.offsets, ep.nt,
                                           ep.T, gH, S_ext=S)
        return grad, None, None, None, None, None, None, None
