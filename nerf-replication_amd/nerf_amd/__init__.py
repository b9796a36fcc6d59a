"""nerf_amd -- MI355X (gfx950) kernels of the NeRF render-and-train hot path.

``ops`` exposes torch-facing wrappers over ``libnerf_amd.so`` (C ABI in include/nerf_amd.h).
The drop-in modules under ``src/`` (same paths as the reference's module hooks) call them.
"""
from . import ops  # noqa: F401
from ._lib import LIB_PATH, lib  # noqa: F401
