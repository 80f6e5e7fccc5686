"""Lens I/O: Optiland's JSON lens format.

`Optic.to_dict` / `Optic.from_dict` (optic/optic.py:649-713) serialise a lens as nested
dictionaries -- aperture, fields, wavelengths and the surface list with each surface's
geometry (type, coordinate system with reference_cs chain, radius, conic, coefficients,
...), materials (IdealMaterial index/absorp or catalog Material name/reference),
stop flag, radial aperture and mirror flag. This module reads and writes that schema
with the native host classes, so a lens saved by the reference (e.g. its
docs/samples/*.json) traces on the MI355X without the reference installed. Catalog
glasses resolve through the baked table (data/glasses.json); unknown glasses and
unsupported surface / interaction types raise ValueError. Physical apertures of every
kind (radial, offset radial, elliptical, rectangular, polygon, boolean combinations)
round-trip in the reference's aperture schema.
"""

from __future__ import annotations

import json

import numpy as np

from .coordinate_system import CoordinateSystem
from .geometries import (
    BiconicGeometry,
    ChebyshevPolynomialGeometry,
    EvenAsphere,
    ForbesQ2dGeometry,
    ForbesQbfsGeometry,
    ForbesSolverConfig,
    ForbesSurfaceConfig,
    GridSagGeometry,
    NurbsGeometry,
    OddAsphere,
    Plane,
    PlaneGrating,
    PolynomialGeometry,
    StandardGratingGeometry,
    StandardGeometry,
    ToroidalGeometry,
    ZernikePolynomialGeometry,
    scalar,
)
from .interactions import BaseInteractionModel, RefractiveReflectiveModel
from .materials import AbbeMaterial, IdealMaterial, Material
from .apertures import BaseAperture
from .surfaces import ObjectSurface, Surface

_FIELD_TYPES = {"AngleField": "angle", "ObjectHeightField": "object_height",
                "ParaxialImageHeightField": "paraxial_image_height",
                "angle": "angle", "object_height": "object_height",
                "paraxial_image_height": "paraxial_image_height"}


def _f(v, default=0.0):
    return default if v is None else float(v)


def _cs_from(d):
    """coordinate_system.py:201-225 (from_dict)."""
    if d is None:
        return CoordinateSystem()
    return CoordinateSystem(_f(d.get("x")), _f(d.get("y")), _f(d.get("z")), _f(d.get("rx")),
                            _f(d.get("ry")), _f(d.get("rz")),
                            reference_cs=_cs_from(d["reference_cs"])
                            if d.get("reference_cs") else None)


def _cs_to(cs):
    return {"x": cs.x, "y": cs.y, "z": cs.z, "rx": cs.rx, "ry": cs.ry, "rz": cs.rz,
            "reference_cs": _cs_to(cs.reference_cs) if cs.reference_cs is not None else None}


def geometry_from_dict(d):
    """geometries/*.py from_dict (keys as written by their to_dict)."""
    t = d.get("type")
    cs = _cs_from(d.get("cs"))
    tol, max_iter = _f(d.get("tol"), 1e-10), int(d.get("max_iter", 100))
    if t == "Plane":
        return Plane(cs)
    if t == "NurbsGeometry":  # the control net as this module writes it (geometry_to_dict)
        g = NurbsGeometry(cs, _f(d.get("radius"), np.inf), _f(d.get("conic")),
                          d.get("nurbs_norm_x"), d.get("nurbs_norm_y"),
                          _f(d.get("x_center")), _f(d.get("y_center")),
                          d.get("control_points"), d.get("weights"), d.get("u_degree"),
                          d.get("v_degree"), d.get("u_knots"), d.get("v_knots"),
                          tol=_f(d.get("tol"), 1e-10), max_iter=int(d.get("max_iter", 100)))
        g.is_fitted = bool(d.get("is_fitted", False))
        if "P_size_u" in d:  # the fit grid (fit_surface refits on it)
            g.P_size_u, g.P_size_v = int(d["P_size_u"]), int(d["P_size_v"])
        return g
    if t == "GridSagGeometry":  # grid_sag.py:155-180
        return GridSagGeometry(cs, d["x_coordinates"], d["y_coordinates"], d["sag_values"],
                               _f(d.get("tol"), 1e-6), int(d.get("max_iter", 100)))
    if t in ("PlaneGrating", "StandardGratingGeometry"):
        # plane_grating.py / standard_grating.py to_dict write "order" / "period" /
        # "angle" (the reference's own from_dict cannot read them back)
        order = d.get("grating_order", d.get("order", 0))
        period = _f(d.get("grating_period", d.get("period")), np.inf)
        angle = _f(d.get("groove_orientation_angle", d.get("angle")))
        if t == "PlaneGrating":
            return PlaneGrating(cs, order, period, angle)
        return StandardGratingGeometry(cs, _f(d.get("radius"), np.inf), order, period, angle,
                                       _f(d.get("conic")))
    if t == "StandardGeometry":
        return StandardGeometry(cs, _f(d.get("radius"), np.inf), _f(d.get("conic")))
    if t == "EvenAsphere":
        return EvenAsphere(cs, _f(d.get("radius"), np.inf), _f(d.get("conic")), tol, max_iter,
                           d.get("coefficients", []))
    if t == "OddAsphere":
        return OddAsphere(cs, _f(d.get("radius"), np.inf), _f(d.get("conic")), tol, max_iter,
                          d.get("coefficients", []))
    if t == "ZernikePolynomialGeometry":
        return ZernikePolynomialGeometry(cs, _f(d.get("radius"), np.inf), _f(d.get("conic")),
                                         tol, max_iter, d.get("coefficients", []),
                                         d.get("zernike_type", "standard"),
                                         _f(d.get("norm_radius"), 1.0))
    if t == "PolynomialGeometry":
        return PolynomialGeometry(cs, _f(d.get("radius"), np.inf), _f(d.get("conic")), tol,
                                  max_iter, d.get("coefficients", []))
    if t == "ChebyshevPolynomialGeometry":
        return ChebyshevPolynomialGeometry(cs, _f(d.get("radius"), np.inf),
                                           _f(d.get("conic")), tol, max_iter,
                                           d.get("coefficients", []),
                                           _f(d.get("norm_x"), 1.0), _f(d.get("norm_y"), 1.0))
    if t == "BiconicGeometry":
        return BiconicGeometry(cs, _f(d.get("radius_x"), np.inf), _f(d.get("radius_y"), np.inf),
                               _f(d.get("conic_x")), _f(d.get("conic_y")), tol, max_iter)
    if t == "ToroidalGeometry":
        return ToroidalGeometry(cs, _f(d.get("radius_x"), np.inf), _f(d.get("radius_y"), np.inf),
                                _f(d.get("conic_yz", d.get("conic"))),
                                list(d.get("coeffs_poly_y") or []), tol, max_iter)
    if t in ("ForbesQbfsGeometry", "ForbesQ2dGeometry"):  # forbes/geometry.py:329-370, 612-640
        sc, so = d.get("surface_config", {}), d.get("solver_config", {})
        terms = _forbes_terms(sc.get("terms"), t == "ForbesQbfsGeometry")
        cfg = ForbesSurfaceConfig(radius=_f(sc.get("radius"), np.inf), conic=_f(sc.get("conic")),
                                  norm_radius=_f(sc.get("norm_radius"), 1.0), terms=terms)
        sol = ForbesSolverConfig(tol=_f(so.get("tol"), 1e-10), max_iter=int(so.get("max_iter", 100)))
        cls = ForbesQbfsGeometry if t == "ForbesQbfsGeometry" else ForbesQ2dGeometry
        return cls(cs, cfg, sol)
    raise ValueError(f"Unknown or unsupported geometry type: {t}")


def _forbes_terms(terms, radial):
    """Forbes terms from a dict: Q-bfs {n: c} (JSON turns n into a string); Q-2D
    {(kind, m, n): c} in memory, or as JSON a list of [kind, m, n, c] (tuple keys do not
    survive JSON) or string keys "a,m,n"."""
    if not terms:
        return {}
    if radial:
        return {int(k): float(v) for k, v in dict(terms).items()}
    if isinstance(terms, list):
        return {(str(a), int(m), int(n)): float(c) for a, m, n, c in terms}
    out = {}
    for k, v in terms.items():
        if isinstance(k, str):
            a, m, n = (p.strip(" '\"()") for p in k.split(","))
            k = (a, int(m), int(n))
        out[(str(k[0]), int(k[1]), int(k[2]))] = float(v)
    return out


def geometry_to_dict(g):
    d = {"type": type(g).__name__, "cs": _cs_to(g.cs)}
    if isinstance(g, (ForbesQbfsGeometry, ForbesQ2dGeometry)):
        if isinstance(g, ForbesQbfsGeometry):
            terms = {str(k): scalar(v) for k, v in g.radial_terms.items()}
        else:
            terms = [[k[0], int(k[1]), int(k[2]), scalar(v)]
                     for k, v in g.freeform_coeffs.items()]
        d["surface_config"] = {"radius": scalar(g.radius), "conic": scalar(g.k),
                               "norm_radius": g.norm_radius, "terms": terms}
        d["solver_config"] = {"tol": g.tol, "max_iter": g.max_iter}
        return d
    if isinstance(g, NurbsGeometry):  # the reference's NurbsGeometry has no to_dict of its
        # own (geometries/base.py's writes no net): the control net, knots and fit window
        net = g.P is not None
        d.update(radius=scalar(g.radius), conic=scalar(g.k), tol=float(g.tol),
                 max_iter=int(g.max_iter), nurbs_norm_x=g.nurbs_norm_x,
                 nurbs_norm_y=g.nurbs_norm_y, x_center=float(g.x_center),
                 y_center=float(g.y_center), is_fitted=bool(g.is_fitted),
                 control_points=np.asarray(g.P).tolist() if net else None,
                 weights=np.asarray(g.W).tolist() if net else None,
                 u_degree=int(g.p) if net else None, v_degree=int(g.q) if net else None,
                 u_knots=np.asarray(g.U).tolist() if net else None,
                 v_knots=np.asarray(g.V).tolist() if net else None,
                 P_size_u=int(g.P_size_u), P_size_v=int(g.P_size_v))
        return d
    if isinstance(g, GridSagGeometry):
        d.update(x_coordinates=g.x_grid.tolist(), y_coordinates=g.y_grid.tolist(),
                 sag_values=g.sag_grid.tolist(), tol=g.tol, max_iter=g.max_iter)
        return d
    if isinstance(g, (PlaneGrating, StandardGratingGeometry)):
        d.update(order=g.grating_order, period=g.grating_period,
                 angle=g.groove_orientation_angle)
    if isinstance(g, Plane):
        d["radius"] = float("inf")
        return d
    d["radius"] = g.radius
    d["conic"] = g.k
    if hasattr(g, "tol"):
        d["tol"] = g.tol
        d["max_iter"] = g.max_iter
    if isinstance(g, (EvenAsphere, PolynomialGeometry, ChebyshevPolynomialGeometry)):
        d["coefficients"] = np.asarray(g.coefficients, dtype=float).tolist()
    if isinstance(g, ZernikePolynomialGeometry):
        c = g.coefficients
        d["coefficients"] = (c.detach().cpu().numpy() if hasattr(c, "detach")
                             else np.asarray(c, dtype=float)).tolist()
        d["zernike_type"] = g.zernike_type
        d["norm_radius"] = g.norm_radius
    if isinstance(g, ChebyshevPolynomialGeometry):
        d["norm_x"], d["norm_y"] = g.norm_x, g.norm_y
    if isinstance(g, BiconicGeometry):
        d.update(radius_x=g.Rx, radius_y=g.Ry, conic_x=g.kx, conic_y=g.ky)
    if isinstance(g, ToroidalGeometry):
        d.update(radius_x=g.R_rot, radius_y=g.R_yz, conic_yz=g.k_yz,
                 coeffs_poly_y=list(g.coeffs_poly_y))
    return d


def material_from_dict(d):
    """materials: IdealMaterial (ideal.py from_dict) or a catalog Material (material.py:269-289)."""
    t = d.get("type")
    if t == "IdealMaterial":
        return IdealMaterial(_f(d.get("index"), 1.0), _f(d.get("absorp")))
    if t in ("Material", "MaterialFile"):
        return Material(d["name"], d.get("reference"))
    if t == "AbbeMaterial":  # abbe.py:100-126
        for key in ("index", "abbe"):
            if key not in d:
                raise ValueError(f"Missing required key: {key}")
        return AbbeMaterial(d["index"], d["abbe"])
    raise ValueError(f"Unsupported material type: {t}")


def material_to_dict(m):
    if isinstance(m, AbbeMaterial):
        return {"type": "AbbeMaterial", "propagation_model": {"class": "HomogeneousPropagation"},
                "index": float(m.index[0]), "abbe": float(m.abbe[0])}
    if isinstance(m, IdealMaterial):
        return {"type": "IdealMaterial", "index": float(np.ravel(m.index)[0]),
                "absorp": float(np.ravel(m.absorp)[0])}
    return {"type": "Material", "name": m.name, "reference": m.reference,
            "robust_search": True, "min_wavelength": None, "max_wavelength": None}


def optic_from_dict(data):
    """optic.py:674-713 (Optic.from_dict) into a native Optic."""
    from .fields import Aperture, Field
    from .optic import Optic

    optic = Optic()
    ap = data.get("aperture")
    if ap:
        optic.aperture = Aperture(ap["type"], ap["value"])
    sg = optic.surface_group
    prev = None
    for k, sd in enumerate(data["surface_group"]["surfaces"]):
        for key in ("coating", "bsdf"):
            if sd.get(key):
                raise ValueError(f"surface {k}: {key} is out of scope for the trace core")
        geometry = geometry_from_dict(sd["geometry"])
        post = material_from_dict(sd["material_post"])
        if sd.get("type") == "ObjectSurface" or k == 0:
            s = ObjectSurface(geometry, post)
        else:
            apd = sd.get("aperture")
            aperture = None
            if apd:  # physical_apertures/*.py from_dict
                if "type" not in apd:
                    apd = dict(apd, type="RadialAperture")
                aperture = BaseAperture.from_dict(apd)
            imd = sd.get("interaction_model")  # standard_surface.py:352-365
            model = (BaseInteractionModel.from_dict(imd) if imd else
                     RefractiveReflectiveModel(is_reflective=bool(sd.get("is_reflective", False))))
            s = Surface(prev, post, geometry, is_stop=bool(sd.get("is_stop", False)),
                        aperture=aperture, surface_type=sd.get("surface_type"),
                        interaction_model=model)
            if isinstance(geometry, ZernikePolynomialGeometry):
                s.surface_type = "zernike"
            elif isinstance(geometry, ChebyshevPolynomialGeometry):
                s.surface_type = "chebyshev"
        s.thickness = _f(sd.get("thickness"))
        sg.surfaces.append(s)
        prev = s
    sg._relink()
    sg.use_absolute_cs = True
    fields = data.get("fields", {})
    fdef = fields.get("field_definition")
    ftype = (fdef or {}).get("field_type") if isinstance(fdef, dict) else None
    ftype = ftype or fields.get("field_type")
    if ftype is not None:
        if ftype not in _FIELD_TYPES:
            raise ValueError(f"field type {ftype!r} is not supported by the trace core")
        optic.set_field_type(_FIELD_TYPES[ftype])
    for fd in fields.get("fields", []):
        optic.fields.add_field(Field(_f(fd.get("x")), _f(fd.get("y")), _f(fd.get("vx")),
                                     _f(fd.get("vy"))))
    optic.obj_space_telecentric = bool(fields.get("object_space_telecentric", False))
    for wd in data.get("wavelengths", {}).get("wavelengths", []):
        optic.add_wavelength(wd["value"], bool(wd.get("is_primary", False)),
                             wd.get("unit", "um"))
    optic.polarization = data.get("wavelengths", {}).get("polarization", "ignore")
    apod = data.get("apodization")  # optic.py:691-693
    if apod:
        from .apodization import BaseApodization

        optic.apodization = BaseApodization.from_dict(apod)
    return optic


def optic_to_dict(optic):
    """optic.py:649-672 (Optic.to_dict) for the native Optic."""
    surfaces = []
    for s in optic.surface_group.surfaces:
        d = {"type": "ObjectSurface" if isinstance(s, ObjectSurface) else "Surface",
             "geometry": geometry_to_dict(s.geometry),
             "material_post": material_to_dict(s.material_post),
             "thickness": float(s.thickness)}
        if not isinstance(s, ObjectSurface):
            d.update(material_pre=material_to_dict(s.material_pre), is_stop=bool(s.is_stop),
                     aperture=None if s.aperture is None else s.aperture.to_dict(),
                     coating=None, bsdf=None, is_reflective=bool(s.is_reflective),
                     surface_type=s.surface_type,
                     interaction_model=s.interaction_model.to_dict())
        surfaces.append(d)
    fields = [{"field_type": optic.field_type, "x": f.x, "y": f.y, "vx": f.vx, "vy": f.vy}
              for f in optic.fields.fields]
    return {
        "version": 1.0,
        "aperture": None if optic.aperture is None else
        {"type": optic.aperture.ap_type, "value": optic.aperture.value,
         "object_space_telecentric": optic.obj_space_telecentric},
        "fields": {"fields": fields, "telecentric": False, "field_type": optic.field_type,
                   "object_space_telecentric": optic.obj_space_telecentric},
        "wavelengths": {"wavelengths": [{"value": w.value, "is_primary": w.is_primary,
                                         "unit": "um"}
                                        for w in optic.wavelengths.wavelengths],
                        "polarization": optic.polarization},
        "apodization": optic.apodization.to_dict() if optic.apodization else None,
        "pickups": [],
        "solves": {"solves": []},
        "surface_group": {"surfaces": surfaces},
    }


def load_optiland_json(path):
    """Read an Optiland JSON lens file (e.g. docs/samples/Cooke_triplet.json)."""
    with open(path) as f:
        return optic_from_dict(json.load(f))


def save_optiland_json(optic, path):
    with open(path, "w") as f:
        json.dump(optic_to_dict(optic), f, indent=1)
