"""State-space discretizer for the visitation heatmap (src/envs/discretizer.py:4-26).

Same constructor and methods as the reference (``discretize`` maps one state to a tuple of bin
indices with ``np.digitize`` semantics, ``get_empty_mat`` returns the zero count matrix), plus
``bin_index_torch`` for batches of states on the GPU: the flat (row-major) index of each state's
bin, with the comparisons done in f64 against the same f64 edges, so every state lands in the
bin ``np.digitize`` gives it.
"""
import numpy as np


class Discretizer:
    def __init__(self, features_ranges, bins_sizes, lambda_transform=None):
        assert len(features_ranges) == len(bins_sizes)
        self.num_features = len(features_ranges)
        self.feature_ranges = features_ranges
        self.bins_sizes = bins_sizes
        # interior edges only: np.digitize then returns 0 .. bins_sizes[i] - 1
        self.bins = [np.linspace(features_ranges[i][0], features_ranges[i][1],
                                 bins_sizes[i] + 1)[1:-1] for i in range(self.num_features)]
        self.lambda_transform = lambda_transform

    def discretize(self, features):
        if self.lambda_transform is not None:
            features = self.lambda_transform(features)
        return tuple(np.digitize(x=features[i], bins=self.bins[i]) for i in range(len(features)))

    def get_empty_mat(self):
        return np.zeros(self.bins_sizes)

    def bin_index_torch(self, states):
        """Flat bin index (row-major over bins_sizes) of each row of `states` [B, >= nf].

        np.digitize(x, bins) (right=False) is the i with bins[i-1] <= x < bins[i], which is
        torch.bucketize(x, bins, right=True).  The features are the leading columns (the
        reference's specs use no transform, or lambda s: [s[0], s[1]]).
        """
        import torch

        x = states.to(torch.float64)
        flat = torch.zeros(x.shape[0], dtype=torch.int64, device=x.device)
        for i in range(self.num_features):
            edges = torch.as_tensor(self.bins[i], dtype=torch.float64, device=x.device)
            idx = torch.bucketize(x[:, i].contiguous(), edges, right=True)
            flat = flat * int(self.bins_sizes[i]) + idx
        return flat

    def feature_columns(self, nf):
        """The state columns the discretized features are (lambda_transform must select
        columns, as every reference spec does: none, or lambda s: [s[0], s[1]])."""
        if self.lambda_transform is None:
            if nf != self.num_features:
                raise ValueError(f"state has {nf} features, discretizer {self.num_features}")
            return list(range(nf))
        probe = 1000.5 + 7.0 * np.arange(nf, dtype=np.float64)
        out = np.asarray(self.lambda_transform(probe), dtype=np.float64).reshape(-1)
        cols = (out - 1000.5) / 7.0
        ok = (out.size == self.num_features and np.all(cols == np.round(cols))
              and np.all((cols >= 0) & (cols < nf)))
        if not ok:
            raise NotImplementedError("device heatmap supports column-selecting transforms only")
        return [int(c) for c in cols]

    def visitation_stats(self, visited):
        """Average visitation distribution and average discrete entropy (mepol.py:26-47).

        visited: [E, T, nf] states s_{e,1..T} of E episodes (any device, f64 or f32).  Every
        episode runs all T steps (ErgodicEnv never reports done), so an episode's distribution is
        its bin counts / T, and its entropy is scipy.stats.entropy of that (natural log).
        Returns (average_state_dist [*bins_sizes] f64, average_entropy 0-d f64) tensors on
        visited's device: one bucketize per feature and one bincount over all E*T visits.
        """
        import torch

        E, T, nf = visited.shape
        cols = self.feature_columns(nf)
        nb = int(np.prod(self.bins_sizes))
        flat = self.bin_index_torch(visited.reshape(E * T, nf)[:, cols])
        ep = torch.arange(E, device=visited.device, dtype=torch.int64).repeat_interleave(T)
        counts = torch.bincount(ep * nb + flat, minlength=E * nb).reshape(E, nb)
        state_dist = counts.to(torch.float64) / T
        average_state_dist = state_dist.sum(0) / E
        p = state_dist / state_dist.sum(1, keepdim=True)
        average_entropy = torch.special.entr(p).sum(1).sum() / E
        return average_state_dist.reshape(tuple(self.bins_sizes)), average_entropy
