"""Drop-in adapter for the reference package (Optiland, `import optiland`).

`install()` replaces optiland.surfaces.surface_group.SurfaceGroup.trace
(surface_group.py:232-244) -- the seam SURVEY 8b names -- with the trace core, reached
through the PyTorch custom op torch.ops.ort.trace_sequential (ops.py), when:
  * the rays are RealRays (not Paraxial/Polarized) held as float64 arrays -- torch tensors
    on the HIP device (be.set_backend("torch"); be.set_device("cuda"):
    the op's CUDA kernel, the MI355X trace), torch tensors on the CPU (the torch backend's
    default device, and the reference's own test setting, tests/conftest.py:5-19: the op's
    CPU kernel, the host build of the same core) or NumPy arrays (the numpy backend: the
    CPU kernel on zero-copy tensor views) -- with one wavelength or one per ray (per-ray
    wavelengths run the in-kernel dispersion formulas, ort_batch.w),
  * every traced surface is lowerable (plane / standard / even / odd asphere / Zernike /
    XY-polynomial / Chebyshev / biconic / toroidal / Forbes Q-bfs / Q-2D / grid sag
    geometry, refractive-reflective / thin-lens / phase / grating interaction without
    coating or BSDF, any physical aperture or none, homogeneous propagation),
  * under autograd, every lens value that requires grad is one the trace core
    differentiates -- radius, conic, Zernike coefficients, vertex z (the surface
    coordinate system's z, which the reference's set_thickness writes) -- or does not
    depend on a trainable tensor (see _grad_params). Gradients flow to the input rays and
    to every surface record too (ort_trace_sequential_vjp).
Otherwise the original Python loop runs unchanged (it differentiates everything
itself). The rays are updated in place as the reference does (its attributes are
reassigned, surface.py's be ops); every surface's record (_record,
standard_surface.py:266-286) is filled from the kernel's record buffer.

The lowered lens is cached on the group per wavelength key and re-uploaded only when
the lowered bytes change (the Newton schedules stay with it), so a repeated trace is the
host lowering plus one launch.

`lower_reference_group()` turns reference objects into the same LensTable bytes the
native host API produces (tested equal in tests/test_adapter.py).
"""

from __future__ import annotations

import numpy as np

from . import _abi
from .geometries import (
    BiconicGeometry,
    ChebyshevPolynomialGeometry,
    EvenAsphere,
    ForbesQ2dGeometry,
    ForbesQbfsGeometry,
    ForbesSolverConfig,
    ForbesSurfaceConfig,
    OddAsphere,
    GridSagGeometry,
    NurbsGeometry,
    Plane,
    PlaneGrating,
    PolynomialGeometry,
    StandardGeometry,
    StandardGratingGeometry,
    ToroidalGeometry,
    ZernikePolynomialGeometry,
)
from .coordinate_system import CoordinateSystem
from .interactions import BaseInteractionModel
from .materials import BaseMaterial, lower_dispersion

_ORIGINAL = {}

# calls served by the op per dispatch key, and calls handed to the reference's own loop
# (Unsupported), since install() -- so a caller can see which path ran; REASONS counts the
# fallbacks by their Unsupported message
STATS = {"cuda": 0, "cpu": 0, "fallback": 0, "w_hint": 0}
REASONS: dict = {}


class Unsupported(Exception):
    pass


class _RefMaterial(BaseMaterial):
    """Wraps a reference material: n/k come from the reference's own material code."""

    def __init__(self, m):
        self.m = m

    def _calculate_n(self, w):
        return np.asarray(_np(self.m.n(_be_array(w))), dtype=np.float64) * np.ones_like(w)

    def _calculate_k(self, w):
        return np.asarray(_np(self.m.k(_be_array(w))), dtype=np.float64) * np.ones_like(w)

    def lower(self):
        m = self.m
        if type(m).__name__ == "IdealMaterial":
            return 0, [], [], [], _f(m.index), _f(m.absorp)
        if type(m).__name__ == "AbbeMaterial":  # abbe.py: polyval(p, w)
            return _abi.MAT_ABBE, [float(v) for v in np.ravel(_np(m._p))], [], [], 0.0, 0.0
        opt = [getattr(m, a, None) for a in ("_n_wavelength", "_n")]
        return lower_dispersion(m._n_formula, _np(m.coefficients), _np(m._k_wavelength),
                                _np(m._k), *(None if v is None else _np(v) for v in opt))

    def key(self):
        # same dedup keys as the native materials (materials.py), so tables match
        m = self.m
        if isinstance(m, BaseMaterial):  # a native material passed through the seam
            return m.key()
        if type(m).__name__ == "IdealMaterial":
            return ("ideal", _f(m.index), _f(m.absorp))
        if type(m).__name__ == "AbbeMaterial":
            return ("abbe", _f(m.index), _f(m.abbe))
        fn = getattr(m, "filename", None)
        if fn:
            import os

            return ("glass", fn.split("database" + os.sep)[-1])
        return ("ref", id(m))


def _be_array(w):
    """A NumPy wavelength array as the reference's active backend holds arrays (the
    material code calls be.* on it: a torch tensor under the torch backend)."""
    try:
        import optiland.backend as be

        if be.get_backend() != "numpy":
            import torch

            return torch.as_tensor(w, dtype=torch.float64)
    except ImportError:  # pragma: no cover - not running inside the reference
        pass
    return w


def _np(v):
    try:
        import torch

        if torch.is_tensor(v):
            return v.detach().cpu().numpy()
    except ImportError:  # pragma: no cover
        pass
    return np.asarray(v)


def _f(v):
    return float(np.ravel(_np(v))[0])


def _cs(ref_cs):
    parent = None if ref_cs.reference_cs is None else _cs(ref_cs.reference_cs)
    return CoordinateSystem(_f(ref_cs.x), _f(ref_cs.y), _f(ref_cs.z), _f(ref_cs.rx),
                            _f(ref_cs.ry), _f(ref_cs.rz), reference_cs=parent)


def _geometry(g):
    name = type(g).__name__
    cs = _cs(g.cs)
    if name == "Plane":
        return Plane(cs)
    if name == "GridSagGeometry":
        return GridSagGeometry(cs, _np(g.x_grid), _np(g.y_grid), _np(g.sag_grid), g.tol,
                               g.max_iter)
    if name == "NurbsGeometry":  # nurbs_geometry.py:86-269: the net as the reference holds it
        if g.P is None:
            raise ValueError("NURBS surface without a control net (call fit_surface())")
        out = NurbsGeometry(cs, _f(g.radius), _f(g.k), g.nurbs_norm_x, g.nurbs_norm_y,
                            _f(g.x_center), _f(g.y_center), _np(g.P), _np(g.W), int(g.p),
                            int(g.q), _np(g.U), _np(g.V), tol=_f(g.tol),
                            max_iter=int(g.max_iter))
        out.is_fitted = bool(getattr(g, "is_fitted", False))
        return out
    if name == "PlaneGrating":
        return PlaneGrating(cs, _f(g.grating_order), _f(g.grating_period),
                            _f(g.groove_orientation_angle))
    if name == "StandardGratingGeometry":
        return StandardGratingGeometry(cs, _f(g.radius), _f(g.grating_order),
                                       _f(g.grating_period), _f(g.groove_orientation_angle),
                                       _f(g.k))
    if name == "StandardGeometry":
        return StandardGeometry(cs, _f(g.radius), _f(g.k))
    if name == "EvenAsphere":
        return EvenAsphere(cs, _f(g.radius), _f(g.k), g.tol, g.max_iter,
                           [float(_f(c)) for c in g.coefficients])
    if name == "OddAsphere":
        return OddAsphere(cs, _f(g.radius), _f(g.k), g.tol, g.max_iter,
                          [float(_f(c)) for c in g.coefficients])
    if name == "ZernikePolynomialGeometry":
        return ZernikePolynomialGeometry(cs, _f(g.radius), _f(g.k), g.tol, g.max_iter,
                                         np.ravel(_np(g.coefficients)), g.zernike_type,
                                         _f(g.norm_radius))
    if name == "PolynomialGeometry":
        return PolynomialGeometry(cs, _f(g.radius), _f(g.k), g.tol, g.max_iter,
                                  np.asarray(_np(g.coefficients), dtype=np.float64))
    if name == "ChebyshevPolynomialGeometry":
        return ChebyshevPolynomialGeometry(cs, _f(g.radius), _f(g.k), g.tol, g.max_iter,
                                           np.asarray(_np(g.coefficients), dtype=np.float64),
                                           _f(g.norm_x), _f(g.norm_y))
    if name == "BiconicGeometry":
        return BiconicGeometry(cs, _f(g.Rx), _f(g.Ry), _f(g.kx), _f(g.ky), g.tol, g.max_iter)
    if name == "ToroidalGeometry":
        return ToroidalGeometry(cs, _f(g.R_rot), _f(g.R_yz), _f(g.k_yz),
                                [float(v) for v in np.ravel(_np(g.coeffs_poly_y))],
                                g.tol, g.max_iter)
    if name in ("ForbesQbfsGeometry", "ForbesQ2dGeometry"):
        terms = g.radial_terms if name == "ForbesQbfsGeometry" else g.freeform_coeffs
        cfg = ForbesSurfaceConfig(radius=_f(g.radius), conic=_f(g.k),
                                  norm_radius=_f(g.norm_radius),
                                  terms={k: _f(v) for k, v in terms.items()})
        cls = ForbesQbfsGeometry if name == "ForbesQbfsGeometry" else ForbesQ2dGeometry
        return cls(cs, cfg, ForbesSolverConfig(tol=g.tol, max_iter=g.max_iter))
    raise Unsupported(name)


class _Surf:
    """Duck-typed stand-in for optiland_pr_amd.surfaces.Surface during lowering."""

    def __init__(self, geometry, pre, post, is_reflective, aperture, thickness,
                 interaction_model=None):
        self.geometry = geometry
        self.interaction_model = interaction_model
        self.material_pre = pre
        self.material_post = post
        self.is_reflective = is_reflective
        self.aperture = aperture
        self.thickness = thickness


class _Group:
    def __init__(self, surfaces):
        self.surfaces = surfaces


def _plain(d):
    """reference to_dict() output with backend arrays / tensors as lists and floats"""
    if isinstance(d, dict):
        return {k: _plain(v) for k, v in d.items()}
    if hasattr(d, "detach"):
        d = d.detach().cpu().numpy()
    if isinstance(d, np.ndarray):
        return d.tolist()
    return d


def lower_reference_group(ref_group, wavelengths, record=False):
    """Reference SurfaceGroup -> LensTable (raises Unsupported when not lowerable)."""
    from .apertures import BaseAperture
    from .lowering import lower_surface_group

    mats = {}

    def mat(m):
        if id(m) not in mats:
            mats[id(m)] = _RefMaterial(m)
        return mats[id(m)]

    surfs = []
    for s in ref_group.surfaces[1:]:
        im = s.interaction_model
        if getattr(im, "coating", None) is not None or getattr(im, "bsdf", None) is not None:
            raise Unsupported("coating/bsdf")
        if type(im).__name__ not in ("RefractiveReflectiveModel", "ThinLensInteractionModel",
                                     "PhaseInteractionModel", "DiffractiveInteractionModel"):
            raise Unsupported(type(im).__name__)
        try:  # the reference's to_dict schema (interactions/*.py, phase/*.py)
            native_im = BaseInteractionModel.from_dict(_plain(im.to_dict()))
        except (ValueError, KeyError, TypeError) as e:
            raise Unsupported(type(im).__name__) from e
        for m in (s.material_pre, s.material_post):
            if type(m.propagation_model).__name__ != "HomogeneousPropagation":
                raise Unsupported("propagation model")
        ap = None
        if s.aperture is not None:  # the reference's to_dict schema (physical_apertures)
            try:
                ap = BaseAperture.from_dict(_plain(s.aperture.to_dict()))
            except (ValueError, KeyError, AttributeError) as e:
                raise Unsupported(type(s.aperture).__name__) from e
        surfs.append(_Surf(_geometry(s.geometry), mat(s.material_pre), mat(s.material_post),
                           bool(im.is_reflective), ap, _f(s.thickness), native_im))
    # lower_surface_group skips ObjectSurface instances; pass the traced surfaces only
    return lower_surface_group(_Group(surfs), wavelengths, record=record)


def install():
    """Patch optiland's SurfaceGroup.trace (idempotent). Returns the patched class."""
    from optiland.surfaces import surface_group as sg_mod

    cls = sg_mod.SurfaceGroup
    if "trace" in _ORIGINAL:
        return cls
    _ORIGINAL["trace"] = cls.trace

    def trace(self, rays, skip=0):
        try:
            return _trace_on_mi355x(self, rays, skip)
        except Unsupported as e:
            STATS["fallback"] += 1
            REASONS[str(e)] = REASONS.get(str(e), 0) + 1
            return _ORIGINAL["trace"](self, rays, skip)

    cls.trace = trace
    _hook_ray_wavelength()
    return cls


def _hook_ray_wavelength():
    """Rays generated for a host scalar wavelength (RayGenerator.generate_rays,
    rays/ray_generator.py:28-106: w = ones_like(x) * wavelength, every element exactly the
    scalar) remember it, so the trace picks the lens's table row without reading rays.w
    back from the device (a synchronising copy per call). The hint holds only while rays.w
    is that same, unmodified tensor (identity and torch's in-place version counter)."""
    try:
        from optiland.rays import ray_generator as rg_mod
    except Exception:  # pragma: no cover - reference layout without this module
        return
    cls = rg_mod.RayGenerator
    if "generate_rays" in _ORIGINAL:
        return
    gen = cls.generate_rays
    _ORIGINAL["generate_rays"] = gen

    def generate_rays(self, *args, **kwargs):
        rays = gen(self, *args, **kwargs)
        wl = args[4] if len(args) > 4 else kwargs.get("wavelength")
        if isinstance(wl, (int, float, np.floating)) and not isinstance(wl, bool):
            w = getattr(rays, "w", None)
            rays._ort_w = (w, getattr(w, "_version", None), float(wl))
        return rays

    cls.generate_rays = generate_rays


def _host_wavelength(rays):
    """The scalar wavelength rays were built with, when rays.w is still that tensor."""
    hint = getattr(rays, "_ort_w", None)
    if hint is None:
        return None
    w, version, wl = hint
    if rays.w is not w or getattr(w, "_version", None) != version:
        return None
    return wl


def uninstall():
    from optiland.surfaces import surface_group as sg_mod

    if "trace" in _ORIGINAL:
        sg_mod.SurfaceGroup.trace = _ORIGINAL.pop("trace")
    if "generate_rays" in _ORIGINAL:
        from optiland.rays import ray_generator as rg_mod

        rg_mod.RayGenerator.generate_rays = _ORIGINAL.pop("generate_rays")


# geometries whose radius / conic the derivative kernels seed (the conic base of
# standard.py and of the Newton geometries built on it)
_RK_GEOMETRIES = ("StandardGeometry", "EvenAsphere", "OddAsphere", "ZernikePolynomialGeometry",
                  "PolynomialGeometry", "ChebyshevPolynomialGeometry", "ForbesQbfsGeometry",
                  "ForbesQ2dGeometry")


def _grad_mode_on():
    try:
        import optiland.backend as be

        return bool(be.grad_mode.requires_grad)
    except Exception:  # pragma: no cover - numpy backend / older reference
        return False


def _reaches_parameter(t, memo):
    """Does the autograd graph of t reach a torch.nn.Parameter (a trainable tensor)?
    memo: id(grad_fn) -> (grad_fn, answer), shared by the queries of one trace call (the
    ray fields and lens values share most of their graphs); it holds every node it names,
    so no id is reused while it lives."""
    import torch

    if isinstance(t, torch.nn.Parameter):
        return True
    root = t.grad_fn
    if root is None:
        return False
    stack = [(root, False)]
    while stack:
        node, expanded = stack.pop()
        if not expanded:
            if id(node) in memo:
                continue
            var = getattr(node, "variable", None)  # AccumulateGrad: a leaf
            if var is not None:
                memo[id(node)] = (node, isinstance(var, torch.nn.Parameter))
                continue
            memo[id(node)] = (node, None)  # in progress (the graph is acyclic)
            stack.append((node, True))
            stack.extend((c, False) for c, _ in node.next_functions
                         if c is not None and id(c) not in memo)
        else:
            memo[id(node)] = (node, any(memo[id(c)][1] for c, _ in node.next_functions
                                        if c is not None))
    return bool(memo[id(root)][1])


def _live(v, grad_mode, memo):
    """v is a tensor whose gradient someone wants. Under the reference's be.grad_mode
    (TorchOptimizer) every be.array is a requires-grad leaf, so there only values that
    depend on a torch.nn.Parameter count; outside it any requires-grad tensor does."""
    import torch

    if not (torch.is_tensor(v) and v.requires_grad):
        return False
    return _reaches_parameter(v, memo) if grad_mode else True


def _tensor_attrs(obj, skip=()):
    import torch

    try:
        items = vars(obj).items()
    except TypeError:
        return []
    return [(k, v) for k, v in items if k not in skip and torch.is_tensor(v)]


def _grad_params(group):
    """-> [(kind, traced-surface index, tensor)] for the differentiable lens values that
    require grad (ops.SPEC_KINDS). Raises Unsupported when a lens value the trace core does
    not differentiate (decenters, tilts, reference_cs chains, normalisation radii, asphere
    coefficients, material data, apertures ...) depends on a trainable tensor: the
    reference loop then runs and differentiates it."""
    import torch

    if not torch.is_grad_enabled():
        return []
    grad_mode = _grad_mode_on()
    memo: dict = {}
    out = []

    def refuse(where, name, v):
        if _live(v, grad_mode, memo):
            raise Unsupported(f"gradient through {where}.{name}")

    def cs_chain(cs, where, allow_z):
        for k, v in _tensor_attrs(cs, skip=("z",) if allow_z else ()):
            refuse(where, k, v)
        if cs.reference_cs is not None:
            cs_chain(cs.reference_cs, where + ".reference_cs", False)

    for ti, s in enumerate(group.surfaces[1:]):
        g = s.geometry
        name = type(g).__name__
        diff = {}
        if name in _RK_GEOMETRIES:
            diff["radius"] = getattr(g, "radius", None)
            diff["k"] = getattr(g, "k", None)
        if name == "ZernikePolynomialGeometry":
            diff["coefficients"] = g.coefficients
        for k, v in _tensor_attrs(g, skip=tuple(diff)):
            refuse(f"surface {ti + 1} geometry", k, v)
        cs = g.cs
        z_ok = cs.reference_cs is None
        cs_chain(cs, f"surface {ti + 1} cs", z_ok)
        for m in (s.material_pre, s.material_post):
            for k, v in _tensor_attrs(m):
                refuse(f"surface {ti + 1} material", k, v)
        if s.aperture is not None:
            for k, v in _tensor_attrs(s.aperture):
                refuse(f"surface {ti + 1} aperture", k, v)
        kinds = (("radius", "radius"), ("k", "conic"), ("coefficients", "zernike"))
        for attr, kind in kinds:
            v = diff.get(attr)
            if torch.is_tensor(v) and v.requires_grad:
                if kind != "zernike" and v.numel() != 1:
                    raise Unsupported(f"surface {ti + 1}: non-scalar {attr}")
                out.append((kind, ti, v))
        if z_ok and torch.is_tensor(cs.z) and cs.z.requires_grad:
            out.append(("vertex", ti, cs.z))
    return out


def _device_lens(group, wavelengths, per_ray, device):
    """Lowered lens of a reference group -- uploaded to HBM (DeviceLens) for device rays, in
    host memory (host.HostLens) for CPU rays -- cached on the group per wavelength key and
    device, and rebuilt only when the lowered bytes change (Newton schedules kept across
    edits)."""
    from .host import HostLens
    from .raytrace import DeviceLens

    table = lower_reference_group(group, wavelengths, record=True)
    table.final_mat = -1  # SurfaceGroup.trace has no image-space propagate
    fp = table.fingerprint()
    cache = group.__dict__.setdefault("_ort_lenses", {})
    key = (tuple(float(w) for w in wavelengths), bool(per_ray), str(device))
    hit = cache.get(key)
    if hit is None or hit.fingerprint != fp:
        old = hit
        if device.type == "cpu":
            hit = HostLens(table)
        else:
            hit = DeviceLens(table, device=device)
            if old is not None and old.table.surfaces.shape == table.surfaces.shape:
                hit.sched_cache = old.sched_cache
        hit.fingerprint = fp
        cache[key] = hit
    return hit


def _ray_arrays(rays):
    """The 8 ray fields as float64 torch tensors of one size on one device, and whether they
    came as NumPy arrays (the numpy backend: zero-copy CPU tensor views). Raises Unsupported
    for anything else (float32, mixed devices, scalars)."""
    import torch

    fields = [getattr(rays, a) for a in _abi.RAY_FIELDS]
    if all(isinstance(t, np.ndarray) for t in fields):
        if any(t.dtype != np.float64 or t.ndim != 1 for t in fields):
            raise Unsupported("numpy rays must be 1-d float64 arrays")
        return [torch.from_numpy(np.ascontiguousarray(t)) for t in fields], True
    if not all(torch.is_tensor(t) for t in fields):
        raise Unsupported("ray fields are neither all tensors nor all numpy arrays")
    x = fields[0]
    if x.dtype != torch.float64:
        raise Unsupported("rays must be float64")
    if any(t.dtype != torch.float64 or t.device != x.device or t.numel() != x.numel()
           for t in fields):
        raise Unsupported("ray fields of mixed sizes / devices / dtypes")
    if x.device.type not in ("cuda", "cpu"):
        raise Unsupported(f"rays on {x.device}")
    return fields, False


def _trace_on_mi355x(group, rays, skip):
    import torch

    from . import ops

    if type(rays).__name__ != "RealRays":
        raise Unsupported(type(rays).__name__)
    fields, as_numpy = _ray_arrays(rays)
    x = fields[0]
    n = x.numel()
    params = _grad_params(group) if not as_numpy else []
    w = rays.w
    if not torch.is_tensor(w):
        w = torch.as_tensor(np.asarray(w, dtype=np.float64), device=x.device)
    w = w.detach().to(device=x.device, dtype=torch.float64).reshape(-1)
    if n == 0:
        raise Unsupported("empty ray batch")
    wh = _host_wavelength(rays)
    if wh is not None:  # built from a host scalar: no device read
        lo = hi = wh
        STATS["w_hint"] += 1
    else:
        lo_hi = torch.aminmax(w)  # one read decides table rows vs per-ray dispersion
        lo, hi = (float(v) for v in torch.stack(lo_hi).cpu())
    per_ray = lo != hi
    dl = _device_lens(group, [lo], per_ray, x.device)
    if torch.is_grad_enabled():
        # ray fields count as differentiable inputs under the same rule as lens values
        grad_mode, memo = _grad_mode_on(), {}
        fields = [t if _live(t, grad_mode, memo) else t.detach() for t in fields]
        if params or any(t.requires_grad for t in fields):
            try:
                ops._check_differentiable(dl.table,
                                          adjoint=any(t.requires_grad for t in fields))
            except NotImplementedError as e:  # no derivative kernels: the reference loop
                raise Unsupported(str(e)) from e
    start = max(int(skip) - 1, 0)
    lens, meta, ft, key = ops.lens_args(dl)
    outs = torch.ops.ort.trace_sequential(
        lens, meta, ft, key, fields, w if per_ray else None, [t for _, _, t in params],
        ops.encode_spec([(k, si) for k, si, _ in params]), start, per_ray)
    STATS[x.device.type] += 1
    conv = (lambda t: t.numpy()) if as_numpy else (lambda t: t)
    group.reset()
    names = ("x", "y", "z", "L", "M", "N", "intensity", "opd")
    if skip == 0:  # the object surface records the incoming rays (object_surface.py:56-72)
        obj = group.surfaces[0]
        for nm, t in zip(names, fields, strict=True):
            setattr(obj, nm, conv(t.clone()) if as_numpy else t)
    for a, t in zip(_abi.RAY_FIELDS, outs[:8], strict=True):
        setattr(rays, a, conv(t))
    view = outs[8].view(dl.table.n_rec, 8, n)
    for slot, si in enumerate(dl.table.rec_surfaces):
        if si < start:  # surfaces[:skip] are not traced: their records stay reset
            continue
        s = group.surfaces[si + 1]
        for f, nm in enumerate(names):
            setattr(s, nm, conv(view[slot, f]))
    return rays
