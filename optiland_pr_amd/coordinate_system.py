"""Surface coordinate systems, lowered to ordered localize/globalize op lists.

Mirrors optiland/coordinate_system.py:27-107 (CoordinateSystem(x, y, z, rx, ry, rz,
reference_cs)). localize = reference_cs.localize, translate(-x,-y,-z), rotate_z(-rz)
if rz, rotate_y(-ry) if ry, rotate_x(-rx) if rx; globalize is the reverse. The cos/sin
of each angle are evaluated here in NumPy exactly as the reference evaluates
`be.cos(rx)` (real_rays.py:90-130), so the kernel only multiplies and adds.
"""

from __future__ import annotations

import numpy as np

from . import _abi


class CoordinateSystem:
    def __init__(self, x=0, y=0, z=0, rx=0, ry=0, rz=0, reference_cs=None):
        self.x = float(x)
        self.y = float(y)
        self.z = float(z)
        self.rx = float(rx)
        self.ry = float(ry)
        self.rz = float(rz)
        self.reference_cs = reference_cs

    @staticmethod
    def _rot(kind, angle):
        a = np.array(angle)
        return (kind, (float(np.cos(a)), float(np.sin(a)), 0.0))

    def localize_ops(self):
        ops = [] if self.reference_cs is None else self.reference_cs.localize_ops()
        ops.append((_abi.CS_TRANSLATE, (-self.x, -self.y, -self.z)))
        if self.rz:
            ops.append(self._rot(_abi.CS_ROT_Z, -self.rz))
        if self.ry:
            ops.append(self._rot(_abi.CS_ROT_Y, -self.ry))
        if self.rx:
            ops.append(self._rot(_abi.CS_ROT_X, -self.rx))
        return ops

    def globalize_ops(self):
        ops = []
        if self.rx:
            ops.append(self._rot(_abi.CS_ROT_X, self.rx))
        if self.ry:
            ops.append(self._rot(_abi.CS_ROT_Y, self.ry))
        if self.rz:
            ops.append(self._rot(_abi.CS_ROT_Z, self.rz))
        ops.append((_abi.CS_TRANSLATE, (self.x, self.y, self.z)))
        if self.reference_cs is not None:
            ops.extend(self.reference_cs.globalize_ops())
        return ops

    @property
    def position_in_gcs(self):
        """coordinate_system.py:109-119: globalize the origin."""
        x = y = z = 0.0
        L, M, N = 0.0, 0.0, 1.0
        for kind, p in self.globalize_ops():
            if kind == _abi.CS_TRANSLATE:
                x, y, z = x + p[0], y + p[1], z + p[2]
            elif kind == _abi.CS_ROT_X:
                c, s = p[0], p[1]
                y, z = y * c - z * s, y * s + z * c
            elif kind == _abi.CS_ROT_Y:
                c, s = p[0], p[1]
                x, z = x * c + z * s, -x * s + z * c
            elif kind == _abi.CS_ROT_Z:
                c, s = p[0], p[1]
                x, y = x * c - y * s, x * s + y * c
        return x, y, z
