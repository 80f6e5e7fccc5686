"""The lowering's material caches (lowering._MAT_LOWER / _MAT_N_ALPHA) serve only keys that
name a material's parameters: a custom reference material keyed by its object id
(adapter._RefMaterial: ("ref", id(m))) is re-evaluated on every lowering, so a mutated
material is never traced with stale n / alpha."""

import numpy as np

from optiland_pr_amd import lowering
from optiland_pr_amd.materials import BaseMaterial


class _Custom(BaseMaterial):
    """A material whose n changes in place, keyed by identity as the adapter keys an
    unknown reference material."""

    def __init__(self, n):
        self.value = n

    def _calculate_n(self, w):
        return np.full_like(w, self.value)

    def _calculate_k(self, w):
        return np.zeros_like(w)

    def key(self):
        return ("ref", id(self))

    def lower(self):
        return 0, [], [], [], float(self.value), 0.0


def test_identity_keyed_material_is_not_cached():
    m = _Custom(1.5)
    assert lowering._material_n_alpha(m, 0.55) == (1.5, 0.0)
    assert lowering._material_lower(m)[4] == 1.5
    m.value = 1.7  # mutated in place: same id, same key
    assert lowering._material_n_alpha(m, 0.55) == (1.7, 0.0)
    assert lowering._material_lower(m)[4] == 1.7
    assert not any(k[0][:1] == ("ref",) for k in lowering._MAT_N_ALPHA)
    assert not any(k[:1] == ("ref",) for k in lowering._MAT_LOWER)


def test_parameter_keyed_material_is_cached():
    from optiland_pr_amd.materials import IdealMaterial

    m = IdealMaterial(1.61)
    a = lowering._material_n_alpha(m, 0.55)
    assert (m.key(), 0.55) in lowering._MAT_N_ALPHA
    assert lowering._material_n_alpha(m, 0.55) is a
