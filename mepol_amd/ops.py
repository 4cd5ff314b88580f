"""Torch-facing wrappers over the C ABI (device tensors in, device tensors out, current stream).

Every function here launches HIP kernels from libmepol_amd.so; none has a CPU path.  Tensors
must live on a ROCm device; dtypes follow the reference (f64 values, int64 indices at the
API boundary; int32 indices internally).
"""
import math
import threading

import torch

from . import _lib
from ._lib import call, ptr

_WS = {}


def _stream():
    return ctypes_void(torch.cuda.current_stream().cuda_stream)


def ctypes_void(v):
    import ctypes

    return ctypes.c_void_p(v)


def _require_device(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("mepol_amd ops need ROCm device tensors (got a CPU tensor); "
                             "there is no CPU path in the product")


def _workspace(device, nbytes, tag="knn"):
    """Scratch for eager calls, one buffer per (tag, device, stream): calls on one stream are
    ordered, so they may share it; a buffer outgrown on a stream is released through the caching
    allocator, which is stream-aware.  Captured graphs (algorithms/device_loop.py) never use this
    cache: they own their scratch (see head_workspace / layer_workspace)."""
    key = (tag, device, torch.cuda.current_stream(device).cuda_stream)
    buf = _WS.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
        _WS[key] = buf
    return buf


def head_workspace(n, hidden, a, device):
    """A caller-owned scratch buffer for head_backward at these sizes."""
    import ctypes

    nbytes = ctypes.c_size_t()
    call("mepol_head_workspace_size", n, hidden, a, ctypes.byref(nbytes))
    return torch.empty(max(nbytes.value, 1), dtype=torch.uint8, device=device)


def layer_workspace(n, f, out, device):
    """A caller-owned scratch buffer for layer_backward at these sizes."""
    import ctypes

    nbytes = ctypes.c_size_t()
    call("mepol_layer_workspace_size", n, f, out, ctypes.byref(nbytes))
    return torch.empty(max(nbytes.value, 1), dtype=torch.uint8, device=device)


def dh1_layer1_workspace(n, h0, f, device):
    """A caller-owned scratch buffer for dh1_layer1_backward at these sizes."""
    import ctypes

    nbytes = ctypes.c_size_t()
    call("mepol_dh1_layer1_workspace_size", n, h0, f, ctypes.byref(nbytes))
    return torch.empty(max(nbytes.value, 1), dtype=torch.uint8, device=device)


def knn_plan(n_cand, n_query, d, kp1, split=0):
    import ctypes

    ks, lst, sp = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    call("mepol_knn_plan_info", n_cand, n_query, d, kp1, split, ctypes.byref(ks),
         ctypes.byref(lst), ctypes.byref(sp))
    # ks == 0: no f16 screen (d > 63 or k+1 > 60): every query takes the exhaustive f64 scan,
    # LIST16 is then its block-select capacity
    KS16, nh = ks.value // 10, ks.value % 10
    # MFMA products per k-step and tile (csrc/knn_select.hpp, select16_kernel: A_hi x q_hi, plus
    # A_hi x q_lo when kQueryLo = nh == 2 or KS16 >= 4, plus A_lo x q_hi when nh == 2)
    products = 0 if not ks.value else (3 if nh == 2 else (2 if KS16 >= 4 else 1))
    return {"mode": "screened" if ks.value else "exhaustive", "KS16": KS16, "nh": nh,
            "LIST16": lst.value, "split": sp.value, "mfma_products": products}


def knn_issued_mfma_flops(n_cand, n_query, plan):
    """Flops the f16 selection issues on the matrix cores: products x 2 K (K = 16 KS16) per
    32 x 32 tile pair, padded tiles included."""
    tiles = -(-n_query // 32) * -(-n_cand // 32)
    return float(plan["mfma_products"]) * 2 * 16 * plan["KS16"] * 1024 * tiles


class KnnInputCheck:
    """The input validation of a deferred k-NN call (mepol_knn_deferred): the two counts stay
    on the device, copied to pinned host memory in stream order; raise_if_invalid() waits for
    that copy only and raises what mepol_knn would have raised."""

    # Free pinned slots (a pinned allocation per call cost ~1 ms of host time).  A check holds
    # its slot until raise_if_invalid() has read it (or it is collected); with every slot held
    # a new one is allocated, so no check can read another call's counts.
    _free = []
    _lock = threading.Lock()

    def __init__(self, invalid_dev):
        cls = KnnInputCheck
        with cls._lock:
            slot = cls._free.pop() if cls._free else None
        self._host = slot if slot is not None else torch.empty(2, dtype=torch.int32,
                                                               pin_memory=True)
        memcpy_async(self._host, invalid_dev)
        self._event = torch.cuda.Event()
        self._event.record(torch.cuda.current_stream(invalid_dev.device))
        self._dev = invalid_dev
        self._nonfinite = 0

    def raise_if_invalid(self):
        """Raises sklearn's ValueError for a NaN / inf coordinate.  The second count (rows whose
        f32 squared norm overflows) is not an error: those calls were answered by the
        exhaustive f64 scan."""
        from ._lib import MepolInputError

        if self._host is not None:
            self._event.synchronize()
            self._nonfinite = int(self._host[0])
            overflow = int(self._host[1])
            self._release()
            if overflow and not self._nonfinite:
                import warnings

                warnings.warn(f"mepol_knn: {overflow} rows have a squared norm beyond f32; the f16 "
                              "screen was skipped and every query took the exhaustive f64 scan "
                              "(correct, but far slower than the screen)")
        if self._nonfinite:
            raise MepolInputError(f"mepol_knn failed (rc=1001): mepol_knn: Input contains NaN or "
                                  f"infinity ({self._nonfinite} rows)")

    def _release(self):
        """Returns the slot once its copy has landed (never while the copy may still write)."""
        host, self._host = getattr(self, "_host", None), None
        if host is not None:
            self._event.synchronize()
            with KnnInputCheck._lock:
                KnnInputCheck._free.append(host)

    def __del__(self):
        # never block in a finalizer (it runs wherever garbage collection does, and at
        # interpreter shutdown): return the slot only if its copy has already landed, else
        # drop it (the pinned block is freed with the tensor)
        try:
            host, self._host = getattr(self, "_host", None), None
            if host is not None and self._event.query():
                with KnnInputCheck._lock:
                    KnnInputCheck._free.append(host)
        except Exception:
            pass


def knn(cand, kp1, query=None, split=0, want_int64=True, return_fallback=False, defer_check=False):
    """Exact k-NN of `query` rows among `cand` rows (both f32 [*, d] on device), any d and any
    kp1 <= len(cand) (sklearn raises beyond, and so does this: MepolInputError).

    Returns (D f64 [nq, kp1], I int64 [nq, kp1] or None, I32T int32 [kp1, nq]) and, with
    return_fallback, the device int32 count of queries that took the exhaustive path.
    defer_check: no host synchronisation inside the call (mepol_knn_deferred); a KnnInputCheck
    is appended to the result and the caller must call its raise_if_invalid() before using it.
    Replaces NearestNeighbors(k+1).fit(X).kneighbors(X) (src/algorithms/mepol.py:190-192).
    """
    import ctypes

    if query is None:
        query = cand
    _require_device(cand, query)
    cand = cand.contiguous().float()
    query = query.contiguous().float()
    nc, d = cand.shape
    nq = query.shape[0]
    if query.shape[1] != d:
        raise ValueError("query/candidate dimension mismatch")
    dev = cand.device
    nbytes = ctypes.c_size_t()
    call("mepol_knn_workspace_size", nc, nq, d, kp1, split, ctypes.byref(nbytes))
    ws = _workspace(dev, nbytes.value)
    D = torch.empty((nq, kp1), dtype=torch.float64, device=dev)
    I = torch.empty((nq, kp1), dtype=torch.int64, device=dev) if want_int64 else None
    I32T = torch.empty((kp1, nq), dtype=torch.int32, device=dev)
    nfb = torch.zeros(1, dtype=torch.int32, device=dev)
    out = (D, I, I32T) + ((nfb,) if return_fallback else ())
    if defer_check:
        invalid = torch.empty(2, dtype=torch.int32, device=dev)
        call("mepol_knn_deferred", ptr(cand), nc, ptr(query), nq, d, kp1, split, ptr(D), ptr(I),
             ptr(I32T), ptr(nfb), ptr(invalid), ptr(ws), ws.numel(), _stream())
        return out + (KnnInputCheck(invalid),)
    call("mepol_knn", ptr(cand), nc, ptr(query), nq, d, kp1, split, ptr(D), ptr(I), ptr(I32T),
         ptr(nfb), ptr(ws), ws.numel(), _stream())
    return out


def knn_exact(cand, kp1, query=None, want_int64=True):
    """Exhaustive f64 k-NN (every query scanned exactly, no input validation); reference
    semantics, slower: the independent check of knn().  kp1 <= 3072."""
    if query is None:
        query = cand
    _require_device(cand, query)
    cand = cand.contiguous().float()
    query = query.contiguous().float()
    nc, d = cand.shape
    nq = query.shape[0]
    dev = cand.device
    D = torch.empty((nq, kp1), dtype=torch.float64, device=dev)
    I = torch.empty((nq, kp1), dtype=torch.int64, device=dev) if want_int64 else None
    I32T = torch.empty((kp1, nq), dtype=torch.int32, device=dev)
    call("mepol_knn_exact", ptr(cand), nc, ptr(query), nq, d, kp1, ptr(D), ptr(I), ptr(I32T),
         None, _stream())
    return D, I, I32T


def iw_forward(logp_t, logp_b, offsets, n_particles, normalize=True, w_out=None, u_out=None,
               ts_out=None):
    """u = exp(segmented cumsum(logp_t - logp_b)); w = u / sum(u).

    logp_t/logp_b: f64 [nt, T_stride]; offsets: int64 [nt+1] particle offsets.
    Returns (u [N], traj_sum [nt], w [N] or None, U 0-d or None).
    """
    _require_device(logp_t, logp_b, offsets)
    nt, Ts = logp_t.shape
    dev = logp_t.device
    lt = logp_t.contiguous()
    lb = logp_b.contiguous()
    u = u_out if u_out is not None else torch.empty(n_particles, dtype=torch.float64, device=dev)
    ts = ts_out if ts_out is not None else torch.empty(nt, dtype=torch.float64, device=dev)
    w = (w_out if w_out is not None else torch.empty(n_particles, dtype=torch.float64,
                                                     device=dev)) if normalize else None
    U = torch.empty((), dtype=torch.float64, device=dev) if normalize else None
    call("mepol_iw_forward", ptr(lt), ptr(lb), nt, Ts, ptr(offsets), n_particles, ptr(u), ptr(ts),
         ptr(w), ptr(U), _stream())
    return u, ts, w, U


def iw_normalize(u, U, out=None):
    w = out if out is not None else torch.empty_like(u)
    call("mepol_iw_normalize", ptr(u), ptr(U), u.numel(), ptr(w), _stream())
    return w


def entropy_forward(w, idxT, D, k, ns, G, B, eps, n_w=None, g_out=None, out4=None, vals=None):
    """Fused compute_entropy + compute_kl forward.

    Returns (out4 f64[4] = {H, KL_unclamped, sum_term, sum_klterm}, W [n], g [n]).  With `vals`
    (f64[2]) and `out4` given, out4 is updated in place and vals = {out4[0] on entry, new KL}.
    """
    _require_device(w, idxT, D)
    n = D.shape[0]
    kp1 = D.shape[1]
    dev = w.device
    if n_w is None:
        n_w = w.numel()
    nparts = _lib.load().mepol_entropy_partials_size(n)
    partials = torch.empty(max(2 * nparts, 2), dtype=torch.float64, device=dev)
    W = torch.empty(n, dtype=torch.float64, device=dev)
    g = g_out if g_out is not None else torch.empty(n, dtype=torch.float64, device=dev)
    if vals is not None:
        assert out4 is not None
        call("mepol_entropy_forward_emit", ptr(w.contiguous()), ptr(idxT), ptr(D.contiguous()), n,
             n_w, k, kp1, float(ns), float(G), float(B), float(eps), ptr(W), ptr(g),
             ptr(partials), ptr(out4), ptr(vals), _stream())
        return out4, W, g
    out4 = out4 if out4 is not None else torch.empty(4, dtype=torch.float64, device=dev)
    call("mepol_entropy_forward", ptr(w.contiguous()), ptr(idxT), ptr(D.contiguous()), n, n_w, k,
         kp1, float(ns), float(G), float(B), float(eps), ptr(W), ptr(g), ptr(partials), ptr(out4),
         _stream())
    return out4, W, g


def iw_normalize_gathered(xu_all, world, n, nt, w_out):
    """w_out [world n] <- the all-gathered [u | per-trajectory sums] blocks (world x (n + nt))
    normalised by the fixed-order sum of all ranks' trajectory sums."""
    call("mepol_iw_normalize_gathered", ptr(xu_all), world, n, nt, ptr(w_out), _stream())
    return w_out


def sharded_emit(x_all, world, stride, off, B, n_global, sums_cur, vals):
    """vals <- (B - sums_cur[0], rank-order sum of x_all[r, off + 1] / n_global);
    sums_cur <- the rank-order sums of x_all[r, off], x_all[r, off + 1]."""
    call("mepol_sharded_emit", ptr(x_all), world, stride, off, float(B), n_global, ptr(sums_cur),
         ptr(vals), _stream())


def csr_build(idxT, k, n_own, col_offset=0, row_offset=0, nq=None):
    """CSR transpose of the first k rows of idxT ([>=k, nq]) for ids [col_offset, +n_own)."""
    import ctypes

    _require_device(idxT)
    if nq is None:
        nq = idxT.shape[1]
    dev = idxT.device
    nbytes = ctypes.c_size_t()
    call("mepol_csr_workspace_size", nq, k, n_own, ctypes.byref(nbytes))
    ws = _workspace(dev, nbytes.value, tag="csr")
    off = torch.empty(n_own + 1, dtype=torch.int32, device=dev)
    rows = torch.empty(max(nq * k, 1), dtype=torch.int32, device=dev)
    call("mepol_csr_build", ptr(idxT), nq, k, col_offset, n_own, row_offset, ptr(off), ptr(rows),
         ptr(ws), ws.numel(), _stream())
    return off, rows


def entropy_gamma_nparts(n_own):
    """Block partials entropy_gamma returns (csrc/entropy.hip: one per 256-thread block of
    kGammaLanes lanes per particle, at most kGammaMaxBlocks)."""
    return int(_lib.load().mepol_entropy_gamma_partials_size(n_own))


def entropy_gamma(g, w_own, csr_off, csr_rows):
    n_own = w_own.numel()
    dev = w_own.device
    gamma = torch.empty(n_own, dtype=torch.float64, device=dev)
    nparts = entropy_gamma_nparts(n_own)
    partials = torch.empty(max(nparts, 1), dtype=torch.float64, device=dev)
    call("mepol_entropy_gamma", ptr(g), ptr(w_own), ptr(csr_off), ptr(csr_rows), n_own,
         ptr(gamma), ptr(partials), _stream())
    return gamma, partials, nparts


def entropy_reverse_scan(gamma, w, partials, nparts, offsets, nt, T_stride, grad_H, S_ext=None):
    grad = torch.empty((nt, T_stride), dtype=torch.float64, device=w.device)
    call("mepol_entropy_reverse_scan", ptr(gamma), ptr(w), ptr(partials), nparts, ptr(S_ext),
         ptr(offsets), nt, T_stride, ptr(grad_H), ptr(grad), _stream())
    return grad


def head_forward(z, Wm, bm, log_std, act, bz=None, mu_out=None, logp_out=None):
    """Fused Gaussian head: (mu [n, a], logp [n]) from the last pre-activation z (+ bias bz)."""
    n, h = z.shape
    a = Wm.shape[0]
    mu = mu_out if mu_out is not None else torch.empty((n, a), dtype=torch.float64, device=z.device)
    logp = logp_out if logp_out is not None else torch.empty(n, dtype=torch.float64,
                                                             device=z.device)
    call("mepol_head_forward", ptr(z), n, h, ptr(bz), ptr(Wm), ptr(bm), ptr(log_std), ptr(act), a,
         ptr(mu), ptr(logp), _stream())
    return mu, logp


def head_backward(grad_logp, z, Wm, log_std, act, mu, bz=None, need_dz=True, ws=None,
                  outs=None, reduce_stream=None, defer_reduce=False):
    """Returns (dz or None, dWm, dbm, dlog_std, dbz or None).  `ws`: caller-owned scratch
    (head_workspace); default: the per-stream eager cache.  `outs`: optional (dWm, dbm,
    dlog_std, dbz) tensors to write instead of fresh ones.  `reduce_stream`: the parameter
    gradients' two reduce kernels run there (ordered after the row kernel on the current
    stream, mepol_head_backward_phase), dz is ready on the current stream; the caller joins
    reduce_stream before reading dWm / dbm / dlog_std / dbz (same bits either way).
    `defer_reduce`: only the row kernel runs now; a sixth return value finish() launches the
    reduces on the then-current stream, which must be ordered after this one and before the
    workspace is reused."""
    import ctypes

    n, h = z.shape
    a = Wm.shape[0]
    dev = z.device
    if ws is None:
        nbytes = ctypes.c_size_t()
        call("mepol_head_workspace_size", n, h, a, ctypes.byref(nbytes))
        ws = _workspace(dev, nbytes.value, tag="head")
    dz = torch.empty_like(z) if need_dz else None
    if outs is not None:
        dWm, dbm, dls, dbz = outs
        assert all(t is None or t.is_contiguous() for t in outs)
    else:
        dWm = torch.empty_like(Wm)
        dbm = torch.empty(a, dtype=torch.float64, device=dev)
        dls = torch.empty(a, dtype=torch.float64, device=dev)
        dbz = torch.empty(h, dtype=torch.float64, device=dev) if bz is not None else None
    args = (ptr(grad_logp), ptr(z), n, h, ptr(bz), ptr(Wm), ptr(log_std), ptr(act), ptr(mu), a,
            ptr(dz), ptr(dWm), ptr(dbm), ptr(dls), ptr(dbz), ptr(ws), ws.numel())
    if defer_reduce:
        call("mepol_head_backward_phase", *args, 1, _stream())
        return dz, dWm, dbm, dls, dbz, lambda: call("mepol_head_backward_phase", *args, 2,
                                                    _stream())
    if reduce_stream is None:
        call("mepol_head_backward", *args, _stream())
        return dz, dWm, dbm, dls, dbz
    call("mepol_head_backward_phase", *args, 1, _stream())
    done = torch.cuda.Event()
    done.record(torch.cuda.current_stream())
    reduce_stream.wait_event(done)
    with torch.cuda.stream(reduce_stream):
        call("mepol_head_backward_phase", *args, 2, _stream())
    if not torch.cuda.is_current_stream_capturing():  # a graph keeps its buffers alive
        for t in (dWm, dbm, dls, dbz, ws):
            if t is not None:
                t.record_stream(reduce_stream)
    return dz, dWm, dbm, dls, dbz


POLICY_FWD_MAX_IN = 64
POLICY_FWD_MAX_H1 = 320


def policy_forward_ok(in_features, hidden1):
    return in_features <= POLICY_FWD_MAX_IN and hidden1 <= POLICY_FWD_MAX_H1


def h1_mask_buffer(n, hidden0, device):
    """relu'(h1) bit mask of policy_forward(mask_out=...): [n, ceil(hidden0 / 16)] int16."""
    return torch.empty((n, (hidden0 + 15) // 16), dtype=torch.int16, device=device)


def policy_forward(x, W1, b1, W2, b2, Wm, bm, log_std, act, h1_out=None, z2_out=None,
                   mu_out=None, logp_out=None, mask_out=None):
    """One-kernel forward of the two-hidden-layer Gaussian policy: returns (h1, z2, mu, logp)
    with h1 = relu(x W1^T + b1), z2 = h1 W2^T (pre-bias), mu = relu(z2 + b2) Wm^T + bm and
    logp = sum_a log N(act | mu, exp(log_std) + 1e-7).  With mask_out (h1_mask_buffer) the
    kernel also writes relu'(h1) as bits for dh1_layer1_backward(mask=...)."""
    n, f = x.shape
    h0, h1w, a = W1.shape[0], W2.shape[0], Wm.shape[0]
    dev = x.device

    def buf(t, shape):
        return t if t is not None else torch.empty(shape, dtype=torch.float64, device=dev)

    h1 = buf(h1_out, (n, h0))
    z2 = buf(z2_out, (n, h1w))
    mu = buf(mu_out, (n, a))
    logp = buf(logp_out, (n,))
    if mask_out is None:
        call("mepol_policy_forward", ptr(x), n, f, ptr(W1), ptr(b1), h0, ptr(W2), ptr(b2), h1w,
             ptr(Wm), ptr(bm), ptr(log_std), ptr(act), a, ptr(h1), ptr(z2), ptr(mu), ptr(logp),
             _stream())
    else:
        assert mask_out.shape == (n, (h0 + 15) // 16) and mask_out.dtype == torch.int16
        assert mask_out.is_contiguous()
        call("mepol_policy_forward_masked", ptr(x), n, f, ptr(W1), ptr(b1), h0, ptr(W2), ptr(b2),
             h1w, ptr(Wm), ptr(bm), ptr(log_std), ptr(act), a, ptr(h1), ptr(z2), ptr(mu),
             ptr(logp), ptr(mask_out), _stream())
    return h1, z2, mu, logp


DH1_L1_MAX_IN = 63


def dh1_layer1_ok(in_features, hidden1):
    return in_features <= DH1_L1_MAX_IN and hidden1 % 2 == 0


def dh1_layer1_backward(dz2, W2t, h1, x, ws=None, dW_out=None, db_out=None, mask=None,
                        w2=None):
    """(dW1, db1) of h1 = relu(x W1^T + b1) from dz2 = dL/dz2 [n, h1w] and W2t = W2^T
    [h0, h1w]: dh1 = dz2 W2 is reduced on chip (csrc/gemm.hip), never written.  With `w2`
    (W2 as stored, [h1w, h0]; needs `mask`) W2t is not read and may be None: the kernel
    transposes W2's tiles itself (mepol_dh1_layer1_backward_w2)."""
    n, k = dz2.shape
    f = x.shape[1]
    if w2 is not None:
        h0 = w2.shape[1]
        assert mask is not None and w2.shape[0] == k and w2.is_contiguous() and dz2.is_contiguous()
    else:
        h0 = W2t.shape[0]
        assert W2t.shape[1] == k and h1.shape == (n, h0) and dz2.is_contiguous() and W2t.is_contiguous()
    if ws is None:
        import ctypes

        nbytes = ctypes.c_size_t()
        call("mepol_dh1_layer1_workspace_size", n, h0, f, ctypes.byref(nbytes))
        ws = _workspace(x.device, nbytes.value, tag="dh1l1")
    dW = dW_out if dW_out is not None else torch.empty((h0, f), dtype=torch.float64,
                                                      device=x.device)
    db = db_out if db_out is not None else torch.empty(h0, dtype=torch.float64, device=x.device)
    assert dW.is_contiguous() and db.is_contiguous()
    if w2 is not None:
        assert mask.shape == (n, (h0 + 15) // 16) and mask.dtype == torch.int16
        call("mepol_dh1_layer1_backward_w2", ptr(dz2), n, k, ptr(w2), h0, ptr(mask), ptr(x), f,
             ptr(dW), ptr(db), ptr(ws), ws.numel(), _stream())
    elif mask is None:
        call("mepol_dh1_layer1_backward", ptr(dz2), n, k, ptr(W2t), h0, ptr(h1), ptr(x), f,
             ptr(dW), ptr(db), ptr(ws), ws.numel(), _stream())
    else:  # relu'(h1) from the forward's bit mask (policy_forward(mask_out=...))
        assert mask.shape == (n, (h0 + 15) // 16) and mask.dtype == torch.int16
        call("mepol_dh1_layer1_backward_masked", ptr(dz2), n, k, ptr(W2t), h0, ptr(mask),
             ptr(x), f, ptr(dW), ptr(db), ptr(ws), ws.numel(), _stream())
    return dW, db


def weight_grad_workspace(n, out_features, in_features, device):
    """Scratch of weight_grad (its K-slices' partial blocks), owned by the caller."""
    import ctypes

    nbytes = ctypes.c_size_t()
    call("mepol_weight_grad_workspace_size", n, out_features, in_features, ctypes.byref(nbytes))
    return torch.empty(max(nbytes.value, 1), dtype=torch.uint8, device=device)


def weight_grad(dy, x, out=None, ws=None):
    """dW = dy^T x for dy [n, out] and x [n, in] (f64, row-major): the weight gradient of a
    Linear layer over a tall batch (csrc/wgrad.hip: split-K on the f64 matrix cores, fixed-order
    sum over the K-slices)."""
    n, o = dy.shape
    i = x.shape[1]
    assert x.shape[0] == n and dy.is_contiguous() and x.is_contiguous()
    assert dy.dtype == torch.float64 and x.dtype == torch.float64
    if ws is None:
        ws = weight_grad_workspace(n, o, i, dy.device)
    dW = out if out is not None else torch.empty((o, i), dtype=torch.float64, device=dy.device)
    assert dW.is_contiguous() and dW.shape == (o, i)
    call("mepol_weight_grad", ptr(dy), n, o, ptr(x), i, ptr(dW), ptr(ws), ws.numel(), _stream())
    return dW


def gemm_nt(A, B, bias=None, relu=False, out=None, variant=0):
    """act(A B^T + bias) on the f64 matrix cores: A [n, k], B [m, k] (row-major, k even)."""
    n, k = A.shape
    m = B.shape[0]
    assert B.shape[1] == k and A.stride(1) == 1 and B.stride(1) == 1
    C = out if out is not None else torch.empty((n, m), dtype=torch.float64, device=A.device)
    call("mepol_gemm_nt", ptr(A), n, k, A.stride(0), ptr(B), m, B.stride(0), ptr(bias),
         int(relu), ptr(C), C.stride(0), variant, _stream())
    return C


def layer_forward(x, W, b, out=None):
    """h = relu(x W^T + b) for the policy's input layer (in_features <= 64)."""
    n, f = x.shape
    h = out if out is not None else torch.empty((n, W.shape[0]), dtype=torch.float64,
                                                device=x.device)
    call("mepol_layer_forward", ptr(x), n, f, ptr(W), ptr(b), W.shape[0], ptr(h), _stream())
    return h


def layer_backward(dh, h, x, ws=None):
    """(dW, db) of h = relu(x W^T + b) from dL/dh and the forward output h.  `ws`: caller-owned
    scratch (layer_workspace); default: the per-stream eager cache."""
    import ctypes

    n, f = x.shape
    out = h.shape[1]
    if ws is None:
        nbytes = ctypes.c_size_t()
        call("mepol_layer_workspace_size", n, f, out, ctypes.byref(nbytes))
        ws = _workspace(x.device, nbytes.value, tag="layer")
    dW = torch.empty((out, f), dtype=torch.float64, device=x.device)
    db = torch.empty(out, dtype=torch.float64, device=x.device)
    call("mepol_layer_backward", ptr(dh), ptr(h), ptr(x), n, f, out, ptr(dW), ptr(db), ptr(ws),
         ws.numel(), _stream())
    return dW, db


def optim_step(kind, params, grads, exp_avg, exp_avg_sq, scalars, snapshot=None):
    """In-place Adam (kind 0) / RMSprop (kind 1) update of f64 tensors; scalars is a device f64
    tensor (see include/mepol_amd.h, mepol_optim_step).  snapshot = (params_snap, exp_avg_snap,
    exp_avg_sq_snap) lists (entries may be None) receive the values from before the update."""
    import ctypes

    n = len(params)
    arr = ctypes.c_void_p * n
    snaps = list(snapshot) if snapshot is not None else [None, None, None]
    for t in (list(params) + list(grads) + list(exp_avg_sq) + list(exp_avg or [])
              + [x for lst in snaps if lst is not None for x in lst]):
        if t.dtype != torch.float64 or not t.is_contiguous() or not t.is_cuda:
            raise ValueError("optim_step needs contiguous f64 device tensors")
    for lst in snaps:
        if lst is not None and (len(lst) != n or any(
                a.numel() != b.numel() for a, b in zip(lst, params))):
            raise ValueError("optim_step: snapshot tensors must match the parameters")
    sizes = (ctypes.c_int64 * n)(*[t.numel() for t in params])
    m = arr(*[t.data_ptr() for t in exp_avg]) if exp_avg is not None else None
    sp = [arr(*[t.data_ptr() for t in lst]) if lst is not None else None for lst in snaps]
    call("mepol_optim_step_snapshot", kind, n, arr(*[t.data_ptr() for t in params]),
         arr(*[t.data_ptr() for t in grads]), m, arr(*[t.data_ptr() for t in exp_avg_sq]),
         sizes, ptr(scalars), sp[0], sp[1], sp[2], _stream())


def step_mountaincar(state, action):
    """In-place batched MountainCar step: state f64 [n,2], action f64 [n, a>=1]."""
    _require_device(state, action)
    call("mepol_step_mountaincar", ptr(state), ptr(action), state.shape[0], action.stride(0),
         _stream())
    return state


def step_gridworld(state, action):
    """In-place batched GridWorld step: state f32 [n,2], action f64 [n,2]."""
    _require_device(state, action)
    call("mepol_step_gridworld", ptr(state), ptr(action.contiguous()), state.shape[0], _stream())
    return state


def rollout_step(env_id, env_f64, env_f32, mean, noise, log_std, t, T, states_rec, actions_rec,
                 policy_in):
    n, a_dim = mean.shape
    call("mepol_rollout_step", env_id, ptr(env_f64), ptr(env_f32), ptr(mean), ptr(noise),
         ptr(log_std), n, a_dim, t, T, ptr(states_rec), ptr(actions_rec), ptr(policy_in),
         _stream())


def rollout_mlp(env_id, W1, b1, W2, b2, Wm, bm, log_std, init, noise, states_rec, actions_rec,
                visited=None):
    """All T steps of a batched MountainCar (env_id 0, init f64 [n,2]) / GridWorld (1, init f32)
    rollout with the 2-hidden-layer ReLU policy in one launch; noise [T, n, a] f64."""
    T, n, a_dim = noise.shape
    h0, h1 = W1.shape[0], W2.shape[0]
    W2t = W2.t().contiguous()
    init64 = init.contiguous() if env_id == 0 else None
    init32 = init.contiguous() if env_id == 1 else None
    import ctypes

    nbytes = ctypes.c_size_t()
    call("mepol_rollout_mlp_workspace_size", n, T, h0, h1, a_dim, ctypes.byref(nbytes))
    ws = _workspace(init.device, nbytes.value, tag="rollout")
    args = (env_id, ptr(W1.contiguous()), ptr(b1), h0, ptr(W2t), ptr(b2), h1,
            ptr(Wm.contiguous()), ptr(bm), ptr(log_std.contiguous()), a_dim, ptr(init64),
            ptr(init32), ptr(noise.contiguous()), n, T, ptr(states_rec), ptr(actions_rec),
            ptr(visited), None)
    call("mepol_rollout_mlp", *args, ptr(ws), ws.numel(), _stream())
    # word 0 (zeroed by the call): the multi-workgroup form gave up waiting for a part of a
    # trajectory.  The one-workgroup form (no workspace) sums in the same order and rewrites
    # every output, so the result is the same bits either way.
    if int(ws[:4].view(torch.int32)[0].item()) != 0:
        import warnings

        warnings.warn("mepol_rollout_mlp: workgroups of a trajectory were not co-resident; "
                      "re-ran the one-workgroup form")
        call("mepol_rollout_mlp", *args, None, 0, _stream())


def rollout_mlp_plan(n, h0, h1, a_dim):
    """{"workgroups_per_traj", "k_chunks"}: the form mepol_rollout_mlp takes for this shape and
    the layer-2 summation order it commits to (oracle.rollout_kordered's k_chunks)."""
    import ctypes

    wg, kc = ctypes.c_int(), ctypes.c_int()
    call("mepol_rollout_mlp_plan_info", n, h0, h1, a_dim, ctypes.byref(wg), ctypes.byref(kc))
    return {"workgroups_per_traj": wg.value, "k_chunks": kc.value}


def memcpy_async(dst, src):
    """dst <- src (same byte size; device or pinned host tensors), ordered on the current
    stream; inside a graph capture this is a memcpy node."""
    nbytes = src.numel() * src.element_size()
    assert dst.numel() * dst.element_size() == nbytes and dst.is_contiguous() and src.is_contiguous()
    call("mepol_memcpy_async", ptr(dst), ptr(src), nbytes, _stream())


def volume_constant(ns, G):
    return math.pi ** (ns / 2) / G
