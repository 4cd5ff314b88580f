from .gridworld import GridWorldContinuous
from .mountain_car import MountainCarContinuous
from .spaces import Box
from .wrappers import ErgodicEnv, unwrap

__all__ = ["GridWorldContinuous", "MountainCarContinuous", "Box", "ErgodicEnv", "unwrap"]
