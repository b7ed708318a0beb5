"""trajectory_generation_amd -- MI355X-native batched MPC step for the 6-state dynamic bicycle model.

Drop-in for DorianaG01/trajectory_generation's MPC/mpc_6stati.py (see mpc_6stati.py here), backed by
hand-written HIP kernels for gfx950 in libtrajmpc.so (C ABI: include/trajmpc.h).
"""
from . import _lib  # noqa: F401

__all__ = ["mpc_6stati", "batch", "dataset"]
