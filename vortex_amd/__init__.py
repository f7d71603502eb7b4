"""vortex_amd — MI355X-native (gfx950) decode engine for the Vortex canonicalize hot path.

The product is libvortex_gpu.so (HIP kernels + the C ABI in include/vortex_gpu.h).  This
package is the host-side mirror of the reference's array/encoding API for that path:
`arrays` (Array trees with the reference's encoding ids, metadata and validation),
`encode` (the reference encoders, used to build inputs) and `canonicalize` (the C-ABI call).
"""
from ._lib import ENC, PTYPE, PTYPES, VortexGpuError, gpu_lib, enc_lib  # noqa: F401
from .arrays import Array, Canonical, Context, Plan, canonicalize, take  # noqa: F401
from . import arrays, encode  # noqa: F401

__all__ = ["Array", "Canonical", "Context", "Plan", "canonicalize", "take", "arrays", "encode", "ENC", "PTYPE",
           "PTYPES", "VortexGpuError", "gpu_lib", "enc_lib"]
