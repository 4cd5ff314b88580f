"""Device-resident particle batch of one MEPOL epoch and its cached derived data.

The reference passes (states, actions, real_traj_lengths, distances, indices) to every
hot-path call (src/algorithms/mepol.py:142-174, 268-281) and recomputes everything each time.
These functions keep that stateless signature, but the tensors returned by
``collect_particles_and_compute_knn`` are registered here so that per-epoch invariants are
built once: flattened (state, action) rows for the batched MLP, trajectory offsets, the int32
transposed neighbour table, the CSR transpose used by the gradient, and the behavioral
policy's log-probabilities (fixed within an epoch; the reference recomputes them 2x per
iteration, mepol.py:128 via :144 and :159).
"""
import weakref

import torch

from .. import ops

# indices-tensor identity -> ParticleBatch (entries vanish with the tensor; identity, not ==)
_REGISTRY = {}


def _param_key(policy):
    return (id(policy),) + tuple((p.data_ptr(), p._version) for p in policy.parameters())


class ParticleBatch:
    def __init__(self, states, actions, real_traj_lengths, distances, indices, idx32T=None,
                 device=None, lengths=None):
        dev = device if device is not None else (
            distances.device if distances.is_cuda else torch.device("cuda"))
        self.device = dev
        self.states = states.to(dev, torch.float64)
        self.actions = actions.to(dev, torch.float64)
        self.num_traj, self.T = self.actions.shape[0], self.actions.shape[1]
        # `lengths`: the same values already on the host (the epoch path reads them before it
        # queues the k-NN, so this constructor does not wait for the k-NN to finish)
        lens = (lengths if lengths is not None
                else real_traj_lengths.reshape(-1).to(torch.int64).cpu())
        self.lengths = lens
        self.dense = bool((lens == self.T).all())
        off = torch.zeros(self.num_traj + 1, dtype=torch.int64)
        off[1:] = torch.cumsum(lens, 0)
        if lengths is not None and real_traj_lengths.is_cuda and real_traj_lengths.device == dev:
            # the same offsets formed on the device: a copy of the host tensor would be a
            # blocking transfer that waits for the k-NN queued before it
            doff = torch.zeros(self.num_traj + 1, dtype=torch.int64, device=dev)
            torch.cumsum(real_traj_lengths.reshape(-1).to(torch.int64), 0, out=doff[1:])
            self.offsets = doff
        else:
            self.offsets = off.to(dev)
        self.N = int(off[-1])
        nf = self.states.shape[-1]
        self.states_flat = self.states[:, : self.T].reshape(self.num_traj * self.T, nf).contiguous()
        self.actions_flat = self.actions.reshape(self.num_traj * self.T, -1).contiguous()
        self.D = distances.to(dev, torch.float64).contiguous()
        if idx32T is None:
            idx32T = indices.to(dev).to(torch.int32).t().contiguous()
        self.idx32T = idx32T
        self.kp1 = self.D.shape[1]
        self._csr = {}
        self._logp_b = None
        self._stash = None  # (param key, logp_t with graph) from compute_kl's forward

    def logp(self, policy):
        """log p(a|s) for all rows as a dense [num_traj, T] f64 tensor (grad if enabled)."""
        lp = policy.get_log_p(self.states_flat, self.actions_flat)
        return lp.reshape(self.num_traj, self.T)

    def behavioral_logp(self, policy):
        key = _param_key(policy)
        if self._logp_b is None or self._logp_b[0] != key:
            with torch.no_grad():
                self._logp_b = (key, self.logp(policy).detach())
        return self._logp_b[1]

    def seed_behavioral_logp(self, policy, logp):
        """Cache `logp` (computed elsewhere at the policy's current parameters) as the policy's
        behavioral log-probabilities, so behavioral_logp(policy) needs no forward pass."""
        with torch.no_grad():
            self._logp_b = (_param_key(policy),
                            logp.detach().reshape(self.num_traj, self.T).clone())

    def csr(self, k):
        if k not in self._csr:
            self._csr[k] = ops.csr_build(self.idx32T, k, self.N)
        return self._csr[k]

    # -- cross-call reuse of one MLP forward (compute_kl after a step == next policy_update) ----
    def stash_logp(self, policy, logp_t):
        self._stash = (_param_key(policy), logp_t)

    def take_logp(self, policy):
        c = self._stash
        self._stash = None
        if c is not None and c[0] == _param_key(policy):
            return c[1]
        return None


def register(indices, batch):
    key = id(indices)
    if key not in _REGISTRY:
        weakref.finalize(indices, _REGISTRY.pop, key, None)
    _REGISTRY[key] = batch
    return batch


def unregister(indices):
    """Drop the batch registered for `indices` (a rejected k-NN input: its D / I are undefined)."""
    _REGISTRY.pop(id(indices), None)


def lookup(states, actions, real_traj_lengths, distances, indices):
    """The registered batch for these tensors, or a new one built from them."""
    b = _REGISTRY.get(id(indices))
    if b is not None and b.kp1 == distances.shape[1] and b.num_traj == actions.shape[0] and (
            b.D.data_ptr() == distances.data_ptr() or torch.equal(b.D, distances.to(b.device))):
        return b
    b = ParticleBatch(states, actions, real_traj_lengths, distances, indices)
    return register(indices, b)
