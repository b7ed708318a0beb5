"""CPU oracle package (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() (as the checker) and bench.py's
cpu_baseline leg may import this package.  The product path
(trajectory_generation_amd/) never imports it.
"""
from .pyoracle import *  # noqa: F401,F403
