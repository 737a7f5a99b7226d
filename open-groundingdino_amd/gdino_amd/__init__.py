"""gdino_amd — MI355X-native kernels for the Grounding DINO training hot path.

Python host glue over the C-ABI in include/gdino_amd.h (libgdino_amd.so,
hand-written HIP for gfx950).  The reference-compatible model API lives in the
sibling ``models`` package (models.GroundingDINO.build_groundingdino).
"""
from . import _lib  # noqa: F401
from ._lib import GdError, LIB_PATH, runtime_info  # noqa: F401

__all__ = ["GdError", "LIB_PATH", "runtime_info"]
