"""optiland_pr_amd -- MI355X-native sequential real-ray trace core for Optiland.

The hot path of Optiland (PriUVBio/optiland_Pr) -- SurfaceGroup.trace and the ray
construction feeding it -- re-built as fused fp64 HIP kernels for gfx950, behind the
C ABI in include/optiland_rt.h, with a host-side mirror of the reference's Optic /
SurfaceGroup / RealRays / SpotDiagram / Wavefront interface.
"""

from . import _abi
from . import ops  # noqa: F401  (registers torch.ops.ort.trace_sequential / trace_pupil)
from .distribution import create_distribution
from .materials import IdealMaterial, Material
from .optic import Optic

__all__ = ["Optic", "IdealMaterial", "Material", "create_distribution", "_abi"]
__version__ = "0.1.0"
