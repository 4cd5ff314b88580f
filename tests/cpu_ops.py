"""CPU stand-ins for mepol_amd.ops (TEST INFRASTRUCTURE ONLY).

Same function signatures as the HIP-backed ops, implemented with the numpy oracle, so the
multi-rank collective algebra of mepol_amd/parallel.py can be exercised with the gloo backend
on CPU-only machines.  Never used by the product.
"""
import numpy as np
import torch

from oracle import mepol_oracle as O


class _NoCheck:
    def raise_if_invalid(self):
        pass


def knn(cand, kp1, query=None, defer_check=False):
    q = cand if query is None else query
    D, I = O.knn_exact(cand.float().numpy(), kp1, Q=q.float().numpy())
    out = (torch.as_tensor(D), torch.as_tensor(I),
           torch.as_tensor(I.T.astype(np.int32)).contiguous())
    return out + ((_NoCheck(),) if defer_check else ())


def iw_forward(logp_t, logp_b, offsets, n_particles, normalize=True):
    lt, lb = logp_t.numpy(), logp_b.numpy()
    off = offsets.numpy()
    u = np.zeros(n_particles)
    ts = np.zeros(lt.shape[0])
    for n in range(lt.shape[0]):
        L = off[n + 1] - off[n]
        x = np.exp(np.cumsum(lt[n, :L] - lb[n, :L]))
        u[off[n]:off[n + 1]] = x
        ts[n] = x.sum()
    u, ts = torch.as_tensor(u), torch.as_tensor(ts)
    if not normalize:
        return u, ts, None, None
    U = ts.sum()
    return u, ts, u / U, U


def iw_normalize(u, U):
    return u / U


def entropy_forward(w, idxT, D, k, ns, G, B, eps, n_w=None):
    w = w.numpy()
    I = idxT.numpy().T
    Dn = D.numpy()
    n_w = w.shape[0] if n_w is None else n_w
    W = w[I[:, :k]].sum(1)
    V = (Dn[:, k] ** ns * np.pi ** (ns / 2)) / G
    r = W / (V + eps)
    with np.errstate(divide="ignore", invalid="ignore"):
        term = (W / k) * np.log(r + eps)
        klt = np.log(k / (n_w * W) + eps)
        g = -(1.0 / k) * (np.log(r + eps) + r / (r + eps))
    out4 = np.array([-term.sum() + B, klt.sum() / n_w, term.sum(), klt.sum()])
    return torch.as_tensor(out4), torch.as_tensor(W), torch.as_tensor(g)


def csr_build(idxT, k, n_own, col_offset=0, row_offset=0, nq=None):
    I = idxT.numpy()[:k]
    nq = I.shape[1] if nq is None else nq
    lists = [[] for _ in range(n_own)]
    for c in range(k):
        for i in range(nq):
            j = int(I[c, i]) - col_offset
            if 0 <= j < n_own:
                lists[j].append(row_offset + i)
    off = np.zeros(n_own + 1, np.int32)
    off[1:] = np.cumsum([len(x) for x in lists])
    rows = np.array([r for x in lists for r in x] or [0], np.int32)
    return torch.as_tensor(off), torch.as_tensor(rows)


def entropy_gamma(g, w_own, csr_off, csr_rows):
    g, w = g.numpy(), w_own.numpy()
    off, rows = csr_off.numpy(), csr_rows.numpy()
    gamma = np.array([g[rows[off[j]:off[j + 1]]].sum() for j in range(w.shape[0])])
    partials = np.array([(gamma * w).sum()])
    return torch.as_tensor(gamma), torch.as_tensor(partials), 1


def entropy_reverse_scan(gamma, w, partials, nparts, offsets, nt, T_stride, grad_H, S_ext=None):
    S = float(S_ext) if S_ext is not None else float(partials[:nparts].sum())
    c = (gamma.numpy() - S) * w.numpy()
    off = offsets.numpy()
    out = np.zeros((nt, T_stride))
    for n in range(nt):
        seg = c[off[n]:off[n + 1]]
        out[n, :len(seg)] = np.cumsum(seg[::-1])[::-1]
    return torch.as_tensor(out * float(grad_H))
