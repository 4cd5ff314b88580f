"""MI355X-native MEPOL hot path: batched rollout, exact k-NN entropy estimate and
importance-weighted policy gradient (drop-in for RiccZamboni/mepol's src/ modules)."""
__version__ = "0.1.0"
