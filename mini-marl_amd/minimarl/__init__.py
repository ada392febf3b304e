"""minimarl — MI355X-native QMIX / VDN rollout-and-learn hot path (HIP kernels behind a C ABI).

Product path only: everything here runs through libminimarl.so (built from
``mini-marl_amd/csrc`` for gfx950). Importing this package does not touch the
GPU; the first op loads the library and raises if it was not built.
"""
from ._lib import lib, symbols  # noqa: F401

__all__ = ["lib", "symbols"]
