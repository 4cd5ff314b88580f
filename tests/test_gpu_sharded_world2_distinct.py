"""The graph-replayed sharded iteration at world size 2 with two ranks that hold DIFFERENT
trajectories (tests/test_gpu_sharded_world2.py's twin ranks read identical
bytes from every peer block, so an offset or slot-order error in the peer-block indexing -- the CSR
remap j // n * (n + 4), the (n + nt) stride of iw_normalize_gathered, the gathered S partials, the
two-bucket all-reduce -- would still pass there).

Harness: both ranks run in ONE process and one OS thread, as two greenlets, on the same GPU, each
with its own ShardedEpoch, policies, optimizer and streams.  `_PeerDist` is a world-2 "group"
whose collectives move real peer data: a rank posts its send buffer with an event recorded behind
it, waits for the peer's post, makes its current stream wait on the peer's event and copies both
blocks (all_gather, in rank order) or adds them (all_reduce, rank 0's + rank 1's: the same bits
on both ranks), then waits on the peer's "done reading" event before going on.  A rank that waits
for a post switches to the other greenlet (saving and restoring torch's per-thread current stream
and grad mode), so all HIP calls come from one thread, as in the product's own captures (two OS
threads joining one capture crashed HIP at capture end).

Graphs: ShardedIteration._capture_graph and _launch are replaced (for _PeerDist ranks only) by a
JOINT form: rank 0 begins the capture on its side stream and rank 1 issues its body onto that
same stream, so both bodies are captured into one graph, interleaved in collective order (their
fork streams join as in a one-rank capture; the collectives' events become graph edges).  Every replay is launched by
rank 0 after both ranks wrote their per-replay scalars; rank 1's stream waits on it.  So every
collective of the sharded body replays with the peer's actual block, at its real offset.

Checked at 1e-9 (H, KL trace, final parameters) against the single-rank graph loop over the
concatenated batch (rank 0's trajectories, then rank 1's: the reference's traj-major order);
csr_rows_x against an explicit map with peer rows; both ranks bit-identical.  (The eager sharded
path is not run here: torch runs a custom Function's backward on its autograd worker thread,
outside the rank greenlets; tests/test_distributed_gloo.py covers that path's collective
algebra with distinct shards.)  Negative control: the same run with the all-gather writing the two
blocks in swapped slots must NOT match (the harness can see a slot-order error).
Reference: src/algorithms/mepol.py:179-192 (worker split), :429-476 (the off-policy loop)."""
import os

import greenlet

import numpy as np
import pytest
import scipy.special
import torch

pytestmark = pytest.mark.gpu

NT, T, NF, A, K, HID = 16, 1250, 29, 8, 10, [64, 48]  # >= 16384 rows per rank: fused path
CASES = [(10.0, 1e-3), (1e-3, 5e-2)]
WAIT_S = 120.0


class _Hub:
    """Shared state of the two ranks: posted values by key, and the switch between the two rank
    greenlets (a rank that waits for a post the peer has not made yet runs the peer)."""

    def __init__(self, swap_slots=False):
        self.box = {}
        self.failed = None
        self.swap = swap_slots
        self.seq = [0, 0]
        self.glets = [None, None]

    def put(self, key, val):
        self.box[key] = val

    def get(self, key):
        me = greenlet.getcurrent()
        r = self.glets.index(me)
        spins = 0
        while key not in self.box:
            if self.failed is not None:
                raise RuntimeError(f"peer rank failed: {self.failed!r}")
            peer = self.glets[1 - r]
            if peer is None or peer.dead:
                raise RuntimeError(f"peer finished without posting {key}")
            spins += 1
            if spins > 100000:
                raise TimeoutError(f"no peer post for {key}")
            # torch's current stream and grad mode are per thread, not per greenlet
            stream, grad = torch.cuda.current_stream(), torch.is_grad_enabled()
            peer.switch()
            torch.cuda.set_stream(stream)
            torch.set_grad_enabled(grad)
        return self.box[key]


class _PeerDist:
    class ReduceOp:
        SUM, MIN, MAX = "sum", "min", "max"

    def __init__(self, hub, rank):
        self.hub, self.rank = hub, rank

    def get_world_size(self, group=None):
        return 2

    def get_rank(self, group=None):
        return self.rank

    def get_backend(self, group=None):
        return "nccl"  # its collectives are stream operations: the graph path captures them

    def barrier(self, group=None):
        pass

    def _exchange(self, t, combine):
        """Post t, then combine(peer_t) on this rank's current stream once the peer's t is
        ready; return after the peer has finished reading t."""
        hub, r = self.hub, self.rank
        hub.seq[r] += 1
        n = hub.seq[r]
        cur = torch.cuda.current_stream()
        if os.environ.get("MEPOL_TEST_TRACE") == "1":
            import inspect
            import sys

            print(f"[rank {r}] collective {n} from {inspect.stack()[3].function}/"
                  f"{inspect.stack()[2].function} capturing={torch.cuda.is_current_stream_capturing()}",
                  file=sys.stderr, flush=True)
        ready = torch.cuda.Event()
        ready.record(cur)
        hub.put(("send", n, r), (t, ready))
        peer_t, peer_ready = hub.get(("send", n, 1 - r))
        cur.wait_event(peer_ready)
        combine(peer_t)
        done = torch.cuda.Event()
        done.record(cur)
        hub.put(("done", n, r), done)
        cur.wait_event(hub.get(("done", n, 1 - r)))

    def all_gather_into_tensor(self, out, inp, group=None):
        flat = inp.reshape(-1)
        o = out.view(2, -1)
        slot = (1 - self.rank) if self.hub.swap else self.rank

        def combine(peer):
            o[slot].copy_(flat)
            o[1 - slot].copy_(peer.reshape(-1))

        self._exchange(flat, combine)

    def all_reduce(self, t, op="sum", group=None):
        fn = {"sum": torch.add, "min": torch.minimum, "max": torch.maximum}[op]
        res = torch.empty_like(t)

        def combine(peer):
            a, b = (t, peer) if self.rank == 0 else (peer, t)
            fn(a, b, out=res)  # rank 0's operand first on both ranks: identical bits

        self._exchange(t, combine)
        t.copy_(res)


def _joint_capture_graph(self):
    """ShardedIteration._capture_graph for a _PeerDist rank: one graph holds both ranks' bodies.
    Rank 0 begins the capture on its side stream; rank 1's body is issued onto that same stream
    (its fork streams join the capture as in a one-rank capture), so the two bodies interleave
    on the capture stream in collective order and meet at the fake collectives."""
    hub, r = self.dist.hub, self.dist.rank
    cur = torch.cuda.current_stream()
    graphs = []
    for par in range(len(self._bufs)):
        self._use(par)
        if r == 0:
            # rank 1 is done with every eager wait on rank 0's events: a stream that waits on an
            # event of a stream in capture fails (hipErrorStreamCaptureIsolation)
            hub.get(("cap_ready", par))
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=self._side, capture_error_mode="relaxed"):
                hub.put(("cap_start", par), self._side)
                self._body()
                hub.get(("cap_end", par))  # rank 1 has issued all of its body
            hub.put(("cap_graph", par), g)
        else:
            hub.put(("cap_ready", par), True)
            stream = hub.get(("cap_start", par))
            with torch.cuda.stream(stream):
                self._body()
            hub.put(("cap_end", par), True)
            g = hub.get(("cap_graph", par))
        graphs.append(g)
    cur.wait_stream(self._side)
    self._use(0)
    self.graphs = graphs


def _joint_launch(self):
    """DeviceIteration._launch for a _PeerDist rank: rank 0 replays the joint graph once both
    ranks' scalars are in their pinned blocks; rank 1's stream waits on that replay."""
    hub, r = self.dist.hub, self.dist.rank
    par = self._next
    self._use(par)
    self._advance_scalars()
    self._nlaunch = getattr(self, "_nlaunch", 0) + 1
    key = ("launch", self._nlaunch)
    if r == 0:
        hub.get(key + (1,))
        self.graphs[par].replay()
        ev = torch.cuda.Event()
        ev.record()
        hub.put(key + (0,), ev)
    else:
        hub.put(key + (1,), True)
        torch.cuda.current_stream().wait_event(hub.get(key + (0,)))
    self._events[par].record()
    self._inflight.append(par)
    self._next = (par + 1) % len(self._bufs)


def _data():
    rng = np.random.default_rng(23)
    st = rng.standard_normal((2 * NT, T + 1, NF)).astype(np.float32)
    st[NT:] = 0.8 * st[NT:] + 0.3  # rank 1's trajectories from another distribution
    return st, (0.5 * rng.standard_normal((2 * NT, T, A))).astype(np.float32)


def _policies(dev, lr):
    from mepol_amd.policy import GaussianPolicy

    torch.manual_seed(5)
    beh = GaussianPolicy(HID, NF, A).to(dev)
    tgt = GaussianPolicy(HID, NF, A).to(dev)
    last = GaussianPolicy(HID, NF, A).to(dev)
    tgt.load_state_dict(beh.state_dict())
    last.load_state_dict(beh.state_dict())
    return beh, tgt, last, torch.optim.Adam(tgt.parameters(), lr=lr)


def _consts():
    return float(scipy.special.gamma(NF / 2 + 1)), float(np.log(K) - scipy.special.digamma(K))


def _params(m):
    return torch.cat([q.detach().reshape(-1) for q in m.parameters()]).cpu().numpy()


def _rank_run(hub, r, kl_threshold, lr, out):
    from mepol_amd import parallel
    from mepol_amd.parallel import ShardedEpoch

    dev = torch.device("cuda:0")
    if True:
        try:
            s = torch.cuda.Stream(device=dev)
            with torch.cuda.stream(s):
                states, actions = _data()
                sl = slice(r * NT, (r + 1) * NT)
                st = torch.as_tensor(states[sl], dtype=torch.float64, device=dev)
                ac = torch.as_tensor(actions[sl], dtype=torch.float64, device=dev)
                rtl = torch.full((NT, 1), T, dtype=torch.int64, device=dev)
                nxt = torch.as_tensor(states[sl, 1:].reshape(-1, NF), device=dev)
                beh, tgt, last, opt = _policies(dev, lr)
                G, B = _consts()
                ep = ShardedEpoch(st, ac, rtl, nxt, K, _PeerDist(hub, r))
                ep.build_knn()
                trace = []
                res = ep.off_policy_optimization(
                    opt, beh, tgt, last, G, B, NF, 0.0, kl_threshold, 6, True, 2, 4, lr,
                    on_accept=lambda n, e, kl, l: trace.append((n, float(e), float(kl), l)))
                it = parallel._SHARDED_CACHE.get(tgt)
                o = dict(H=float(res[0]), n=res[1], bt=res[2], lr=res[3], trace=trace,
                         params=_params(last), graph=it is not None and it.graph is not None)
                if o["graph"]:
                    n = NT * T
                    rows = it.csr_rows.long().cpu()
                    o["csr_remap_ok"] = bool(torch.equal(it.csr_rows_x.long().cpu(),
                                                         rows // n * (n + 4) + rows % n))
                    o["peer_rows"] = int((rows // n != r).sum())
                    if r == 1:  # rank 0's iteration owns the joint graphs (one reset)
                        it.graphs = [None] * len(it.graphs)
                torch.cuda.synchronize()
                out[r] = o
        except BaseException as e:  # wake the peer instead of leaving it waiting
            import sys
            import traceback

            if hub.failed is None:
                print(f"[rank {r}] failed:\n{traceback.format_exc()}", file=sys.stderr, flush=True)
                hub.failed = e
            out[r] = e


def _sharded(graph, kl_threshold, lr, monkeypatch, swap_slots=False):
    from mepol_amd import parallel
    from mepol_amd.parallel import ShardedIteration

    monkeypatch.setenv("MEPOL_DEVICE_LOOP", "1" if graph else "0")
    orig_cap, orig_launch = ShardedIteration._capture_graph, ShardedIteration._launch

    def cap(self):
        return (_joint_capture_graph if isinstance(self.dist, _PeerDist) else orig_cap)(self)

    def launch(self):
        return (_joint_launch if isinstance(self.dist, _PeerDist) else orig_launch)(self)

    monkeypatch.setattr(ShardedIteration, "_capture_graph", cap)
    monkeypatch.setattr(ShardedIteration, "_launch", launch)
    hub = _Hub(swap_slots)
    out = [None, None]
    hub.glets = [greenlet.greenlet(lambda r=r: _rank_run(hub, r, kl_threshold, lr, out))
                 for r in range(2)]
    cur = torch.cuda.current_stream()
    while not all(g.dead for g in hub.glets):
        for g in hub.glets:
            if not g.dead:
                g.switch()
    torch.cuda.set_stream(cur)
    try:
        for o in out:
            if isinstance(o, BaseException):
                raise o
            assert o is not None, "a rank did not finish"
    finally:
        torch.cuda.synchronize()
        parallel.release_graphs()
    return out


def _single_rank(kl_threshold, lr, monkeypatch):
    """One rank, no sharding, over the concatenated batch (traj-major)."""
    from mepol_amd.algorithms import mepol as M

    monkeypatch.setenv("MEPOL_DEVICE_LOOP", "1")
    dev = torch.device("cuda:0")
    states, actions = _data()
    st = torch.as_tensor(states, dtype=torch.float64, device=dev)
    ac = torch.as_tensor(actions, dtype=torch.float64, device=dev)
    rtl = torch.full((2 * NT, 1), T, dtype=torch.int64, device=dev)
    nxt = torch.as_tensor(states[:, 1:].reshape(-1, NF), device=dev)
    beh, tgt, last, opt = _policies(dev, lr)
    G, B = _consts()
    st_, ac_, rl_, _, D, I = M.make_particle_batch(st, ac, rtl, nxt, K)
    trace = []
    res = M.off_policy_optimization(opt, beh, tgt, last, st_, ac_, 2 * NT, rl_, D, I, K, G, B, NF,
                                    0.0, kl_threshold, 6, True, 2, 4, lr,
                                    on_accept=lambda n, e, kl, l: trace.append(
                                        (n, float(e), float(kl), l)))
    return dict(H=float(res[0]), n=res[1], bt=res[2], lr=res[3], trace=trace, params=_params(last))


def _same(a, b, rtol):
    assert (a["n"], a["bt"], a["lr"]) == (b["n"], b["bt"], b["lr"])
    assert len(a["trace"]) == len(b["trace"])
    for x, y in zip(a["trace"], b["trace"]):
        assert x[0] == y[0] and x[3] == y[3]
        np.testing.assert_allclose(x[1:3], y[1:3], rtol=rtol, atol=1e-12)
    np.testing.assert_allclose(a["H"], b["H"], rtol=rtol)
    np.testing.assert_allclose(a["params"], b["params"], rtol=1e-8, atol=1e-11)


@pytest.mark.parametrize("case", range(len(CASES)))
def test_sharded_graph_world2_distinct_shards(cuda, monkeypatch, case):
    kl_threshold, lr = CASES[case]
    g0, g1 = _sharded(True, kl_threshold, lr, monkeypatch)
    s = _single_rank(kl_threshold, lr, monkeypatch)
    assert g0["graph"] and g1["graph"], "the sharded iteration was not captured"
    for g in (g0, g1):
        assert g["csr_remap_ok"] and g["peer_rows"] > 0  # neighbours in the peer's block
    assert len(g0["trace"]) > 0 or kl_threshold < 1    # the tiny threshold rejects every step
    # both ranks hold the same bits (the same accept / backtrack branches)
    assert g0["trace"] == g1["trace"] and np.array_equal(g0["params"], g1["params"])
    _same(g0, s, 1e-9)


@pytest.mark.parametrize("fault", ["swapped_slots", "csr_stride"])
def test_sharded_world2_peer_errors_detected(cuda, monkeypatch, fault):
    """Negative controls: (a) all-gather blocks written in each other's slots, (b) the CSR remap
    of peer particle ids into the gathered dH/dW layout with a block stride of n + 3 instead of
    n + 4 -- each must change the result (the distinct-shard harness sees peer-block errors that
    the twin-rank harness cannot)."""
    from mepol_amd.parallel import ShardedIteration

    kl_threshold, lr = CASES[0]
    if fault == "csr_stride":
        orig_load = ShardedIteration.load

        def bad_load(self, batch, logp_b=None):
            orig_load(self, batch, logp_b)
            self.csr_rows_x.sub_(torch.div(self.csr_rows, self.N, rounding_mode="floor"))

        monkeypatch.setattr(ShardedIteration, "load", bad_load)
    bad0, _ = _sharded(True, kl_threshold, lr, monkeypatch, swap_slots=fault == "swapped_slots")
    monkeypatch.undo()
    s = _single_rank(kl_threshold, lr, monkeypatch)
    with pytest.raises(AssertionError):
        _same(bad0, s, 1e-9)
