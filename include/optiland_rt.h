/*
 * optiland_rt.h -- C ABI of the MI355X sequential real-ray-trace core.
 *
 * This library replaces the per-surface Python loop of the reference
 *   optiland/surfaces/surface_group.py:232-244      SurfaceGroup.trace(rays, skip)
 *   optiland/surfaces/standard_surface.py:186-233   Surface.trace (real-ray branch)
 * together with the ray construction it is fed by
 *   optiland/rays/ray_generator.py:28-106            RayGenerator.generate_rays
 *   optiland/fields/field_types.py:139-180           AngleField.get_ray_origins
 * and the image-space propagate in optiland/raytrace/real_ray_tracer.py:84-89.
 *
 * Everything here is plain C: device pointers, sizes and a hipStream_t (passed as
 * void* so the header does not need HIP headers). Every pointer named "device" must
 * point to device (HBM) memory owned by the caller. Calls are asynchronous on the
 * given stream; nothing in this library allocates, frees or synchronises, so any call
 * can be captured in a hipGraph.
 *
 * Floating-point: fp64 throughout, compiled with -ffp-contract=off so that every
 * +,-,*,/,sqrt is evaluated in the same order and rounding as the reference NumPy
 * backend (see DESIGN.md "Parity").
 */
#ifndef OPTILAND_RT_H
#define OPTILAND_RT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORT_ABI_VERSION 20
#define ORT_MAX_SURFACES 64

/* ---- geometry kinds ----------------------------------- */
enum ort_geometry { /* see optiland/geometries */
  ORT_GEOM_PLANE = 0,        /* plane.py:61-98                                     */
  ORT_GEOM_STANDARD = 1,     /* standard.py:73-167 (sphere / conic)                */
  ORT_GEOM_EVEN_ASPHERE = 2, /* even_asphere.py:82-129 + newton_raphson.py:119-168 */
  ORT_GEOM_ODD_ASPHERE = 3,  /* odd_asphere.py:73-130 + newton_raphson.py:119-168  */
  ORT_GEOM_ZERNIKE = 4,      /* zernike.py:133-246 + zernike/base.py:42-299        */
  ORT_GEOM_POLYNOMIAL = 5,   /* polynomial.py:93-140 (XY polynomial)               */
  ORT_GEOM_CHEBYSHEV = 6,    /* chebyshev.py:104-215                               */
  ORT_GEOM_BICONIC = 7,      /* biconic.py:69-158                                  */
  ORT_GEOM_TOROIDAL = 8,     /* toroidal.py:75-233                                 */
  ORT_GEOM_FORBES_QBFS = 9,  /* forbes/geometry.py:183-330 + forbes/qpoly.py       */
  ORT_GEOM_FORBES_Q2D = 10,  /* forbes/geometry.py:333-640 + forbes/qpoly.py       */
  ORT_GEOM_GRID_SAG = 11,    /* grid_sag.py:61-149: bilinear sag grid, own Newton   */
  ORT_GEOM_NURBS = 12        /* nurbs/nurbs_geometry.py:606-822 (v20): (u, v) solve */
};
/* Coefficient blocks in lens.coef at ort_surface.coef_off (n_coef doubles):
 *   GRID_SAG            nx, ny, x_0 .. x_(nx-1), y_0 .. y_(ny-1), sag[ny][nx] (row = y);
 *                       the intersection starts at t = 0 and stops when max |dt| < tol
 *                       over the call (grid_sag.py:108-140): schedule / newton_stat bit j
 *                       then means "the stop test passed after j updates"
 *   EVEN / ODD_ASPHERE  C_0 .. C_{n-1}
 *   POLYNOMIAL          ni, nj, C[0][0], C[0][1], ..., C[ni-1][nj-1]  (x^i y^j, row-major)
 *   CHEBYSHEV           ni, nj, norm_x, norm_y, C[0][0], ..., C[ni-1][nj-1]
 *   BICONIC             cx, cy, kx, ky  (c = 1/R, 0 for an infinite or zero radius);
 *                       ort_surface.radius / conic = R_x / k_x (the Newton start guess)
 *   TOROIDAL            R_rot, c_yz, k_yz, has_yz (0/1), n_poly, alpha_1 .. alpha_n;
 *                       ort_surface.radius = R_yz, conic = 0 (the Newton start guess)
 *   FORBES_QBFS         norm_radius, L, dep_normal (0 when every coefficient is 0),
 *                       b_0 .. b_{L-1} (orthonormal P_n coefficients)
 *   FORBES_Q2D          norm_radius, vertex dz/dx, vertex dz/dy, L0, b_0 .. b_{L0-1}
 *                       (m = 0 part, as FORBES_QBFS), M, then for m = 1 .. M two
 *                       Clenshaw records (cosine, then sine): L, d_0 .. d_{L-1},
 *                       A_0 .. A_{L-1}, B_0 .. B_{L-1}, C_0 .. C_{L-1} (L = 0: no terms)
 *   NURBS               p, q, nu, nv, U[nu + p + 1], V[nv + q + 1], Pw[4][nu][nv]
 *                       (x w, y w, z w, w); clamped knots, degrees 1 .. 5. Not a Newton
 *                       surface of the schedule: each ray solves its own (u, v) 2 x 2
 *                       iteration (ort_nurbs.h) to its own |r| < tol (tol / max_iter from
 *                       the surface record); no derivative kernels (the VJP entry points
 *                       refuse it, as they refuse GRID_SAG)
 * ZERNIKE uses lens.zern[coef_off .. coef_off + n_coef) instead. */

/* ---- surface flags ------------------------------------------------------------ */
enum ort_surface_flags {
  ORT_SURF_REFLECTIVE = 1u << 0, /* interaction_model.is_reflective (material "mirror") */
  ORT_SURF_RADIUS_INF = 1u << 1, /* standard.py:100-103 plane branch of a conic guess   */
  ORT_SURF_APERTURE = 1u << 2,   /* radial physical aperture: physical_apertures/radial.py */
  ORT_SURF_RECORD = 1u << 3,     /* snapshot the ray state after this surface (_record)  */
  ORT_SURF_TRANSLATE = 1u << 4,  /* informational: the frame is the translation cs_t only  */
  ORT_SURF_APERTURE_PROG = 1u << 5, /* general aperture: a program in lens.coef (ap_off) */
  ORT_SURF_INV_R2 = 1u << 6,       /* inv_r2 holds RN(1 / (R * R)) (finite, normal range)  */
  ORT_SURF_ALPHA_ALL = 1u << 7,    /* optics.alpha_pre > 0 at every wavelength row: the     */
                                   /* absorption step runs unconditionally (homogeneous.py) */
  ORT_SURF_ALPHA_NONE = 1u << 8,   /* optics.alpha_pre == 0 at every row: no absorption     */
                                   /* (neither bit: decided per ray / row)                  */
  /* (v19) the Newton slope is not the sag's derivative: a Zernike surface with a term whose
   * normalisation is not 1 (standard / noll: zernike.py:163-231 omits it from the normal).
   * The adjoint VJP then replays every Newton update, not only the last kHist (4). */
  ORT_SURF_SLOPE_INEXACT = 1u << 9
};

/* ---- lens-wide frame facts (ort_lens.frame_flags) --------------------------------- */
enum ort_lens_flags {
  /* every surface's frame is a translation along z only: both op lists empty and
   * cs_t[0], cs_t[1] == +0 (a centred axial lens such as every sample objective). The
   * kernels then skip localize's x + -0, y + -0 (identities) and the op-list loops. */
  ORT_LENS_AXIAL = 1u << 0
};

/* ---- interaction models (optiland/interactions) ----------------------------------
 * What happens at the surface after the ray reaches it (standard_surface.py:225). The
 * parameters live in lens.coef at ort_surface.ia_off:
 *   REFRACT_REFLECT  (none)    refractive_reflective_model.py:32-55 + real_rays.py:141-181
 *   THIN_LENS        f         thin_lens_interaction_model.py:55-113: paraxial phase
 *                              transformation; leaves the direction unnormalised (N = 1),
 *                              the next propagation normalises it (homogeneous.py:55-57)
 *   PHASE            kind, efficiency, then the profile's parameters (ort_phase_kind):
 *                              phase_interaction_model.py:45-132 (generalised Snell's law)
 *                    CONSTANT  phase                          phase/constant.py
 *                    LINEAR    K_x, K_y (order 2 pi / period times cos / sin of the angle,
 *                              phase/linear_grating.py:51-54)
 *                    RADIAL    n, a_1 .. a_n (phi = sum a_i r^(2i), phase/radial.py)
 *   DIFFRACTIVE      order m, period, then
 *                    0, -sin(angle), cos(angle)   PlaneGrating: constant grating vector
 *                                                 (plane_grating.py:105-124)
 *                    1, tan(angle), R**2, R**3, k + 1   StandardGratingGeometry: grating
 *                                                 vector from the groove tangent
 *                                                 (standard_grating.py:93-146, 224-247)
 *                              diffractive_model.py:28-61 + real_rays.py:183-498 */
enum ort_interaction {
  ORT_IA_REFRACT_REFLECT = 0,
  ORT_IA_THIN_LENS = 1,
  ORT_IA_PHASE = 2,
  ORT_IA_DIFFRACTIVE = 3
};
enum ort_phase_kind { ORT_PHASE_CONSTANT = 0, ORT_PHASE_LINEAR = 1, ORT_PHASE_RADIAL = 2 };

/* ---- coordinate-system op (coordinate_system.py:73-107, real_rays.py:90-130) ---- */
enum ort_cs_kind {
  ORT_CS_TRANSLATE = 0, /* p = (dx, dy, dz)                         rays/base.py:28-42 */
  ORT_CS_ROT_X = 1,     /* p = (cos a, sin a)                       real_rays.py:90-102 */
  ORT_CS_ROT_Y = 2,     /*                                          real_rays.py:104-116 */
  ORT_CS_ROT_Z = 3      /*                                          real_rays.py:118-130 */
};

typedef struct ort_cs_op {
  int32_t kind;
  int32_t reserved;
  double p[3];
} ort_cs_op; /* 32 bytes */

/* One traced surface (the object surface is not in the table: it only records,
 * object_surface.py:56-72). Localize = translate by -cs_t, then cs ops
 * [cs_loc_off, +n_cs_loc) in order; globalize = cs ops [cs_glob_off, +n_cs_glob) in
 * order, then translate by +cs_t. */
typedef struct ort_surface {
  double radius;      /* R (may be +-inf)                                            */
  double conic;       /* k                                                           */
  double tol;         /* Newton tolerance            newton_raphson.py:58-61         */
  double norm_radius; /* Zernike normalisation radius zernike.py:91-116             */
  double ap_rmax2;    /* r_max**2 of a radial aperture  radial.py:50-63              */
  double ap_rmin2;    /* r_min**2                                                    */
  int32_t geometry;   /* enum ort_geometry                                           */
  int32_t flags;      /* enum ort_surface_flags                                      */
  int32_t max_iter;   /* Newton max_iter                                             */
  int32_t n_coef;     /* asphere coefficients / Zernike terms                        */
  int32_t coef_off;   /* offset into lens.coef (asphere) or lens.zern (Zernike)      */
  int32_t mat_pre;    /* column of n_tab/alpha_tab for material_pre                  */
  int32_t mat_post;   /* column for material_post                                    */
  int32_t cs_loc_off;
  int32_t n_cs_loc;
  int32_t cs_glob_off;
  int32_t n_cs_glob;
  int32_t rec_slot;   /* slot in the record buffer when ORT_SURF_RECORD              */
  double cs_t[3];     /* root-frame translation: localize = x + -cs_t, then the loc    */
                      /* ops; globalize = the glob ops, then x + cs_t                  */
  int32_t ap_off;     /* ORT_SURF_APERTURE_PROG: aperture program at lens.coef[ap_off] */
  int32_t ap_len;     /* its length in doubles                                       */
  int32_t interaction; /* enum ort_interaction                                        */
  int32_t ia_off;      /* its parameter block at lens.coef[ia_off]                    */
  double inv_r2;       /* ORT_SURF_INV_R2: the correctly rounded 1 / (R * R); the conic */
                       /* normal's (1 + k) r^2 / (R * R) is then q = a y refined once by  */
                       /* its residual (Markstein), the same IEEE quotient without a      */
                       /* per-ray reciprocal                                              */
  /* lens-constant subexpressions of the conic formulas, formed on the host with the same
   * IEEE operations (standard.py:104-118, 154-167): 2 R, RN(1 + k), RN(R * R) */
  double two_r;
  double one_plus_k;
  double r_sq;
  /* Zernike surfaces up to radial order 6 (v16): the term sum also in Cartesian form,
   * a block at lens.coef[zm_off]: As[K] (the sag's monomial coefficients, normalisation
   * included), An[K] (the normal's: zernike.py:163-231 omits the normalisation
   * constant), then the per-term monomials Ms[nt][K] (= norm_j * Mn[j]) and Mn[nt][K],
   * K = (zm_deg + 1)(zm_deg + 2) / 2 in p-major order of xn^p yn^q (q fastest), xn = x /
   * norm_radius. zm_deg < 0: polar evaluation only. As / An are sum_j c_j M[j] in term
   * order (acc = acc + c_j M[j][k]): formed by the host, or on the device by
   * ort_patch_zernike after device-resident coefficients change. */
  int32_t zm_off;
  int32_t zm_deg;
} ort_surface; /* 176 bytes */

/* Aperture programs (the physical_apertures package): postfix, each op a double opcode followed
 * by its operands; primitives push contains(x, y) of the ray's local (x, y), the boolean
 * ops pop two and push one; a ray is clipped (i = 0, real_rays.py:132-139) when the
 * final value is false.
 *   ORT_AP_RADIAL    r_min^2 r_max^2 ox oy  r_min^2 <= (x-ox)^2 + (y-oy)^2 <= r_max^2
 *                                           (radial.py:54-63, offset_radial.py:46-58)
 *   ORT_AP_ELLIPSE   ox oy a^2 b^2          (x-ox)^2 / a^2 + (y-oy)^2 / b^2 <= 1
 *                                           (elliptical.py:40-55)
 *   ORT_AP_RECT      x_min x_max y_min y_max (rectangular.py:40-60)
 *   ORT_AP_POLYGON   n x0 y0 ... x(n-1) y(n-1): even-odd crossing test of the implicitly
 *                    closed polygon, matplotlib Path.contains_points semantics
 *                    (polygon.py:50-66 via backend path_contains_points)
 *   ORT_AP_UNION / ORT_AP_INTERSECT / ORT_AP_DIFFERENCE: a | b, a & b, a & ~b
 *                    (base.py:255-340) */
enum ort_aperture_op {
  ORT_AP_RADIAL = 1,
  ORT_AP_ELLIPSE = 2,
  ORT_AP_RECT = 3,
  ORT_AP_POLYGON = 4,
  ORT_AP_UNION = 5,
  ORT_AP_INTERSECT = 6,
  ORT_AP_DIFFERENCE = 7
};

/* Per (wavelength, surface) optical constants, read in the same scalar-load batch as
 * the surface record (one round trip per surface instead of three dependent ones). */
typedef struct ort_surface_optics {
  double n_pre;     /* n of material_pre (standard_surface.py:218 OPD)                */
  double u;         /* n_pre / n_post (real_rays.py:152); the same IEEE quotient the  */
                    /* reference forms per ray                                        */
  double alpha_pre; /* 4 pi k / lambda of material_pre, 0 when k == 0 (homogeneous.py) */
  double n_post;    /* n of material_post (thin-lens / phase / grating interactions)  */
  double u_sq;      /* RN(u * u), the u ** 2 of real_rays.py:156                       */
} ort_surface_optics; /* 40 bytes */

/* One Zernike term: c * norm * R_n^|m|(rho) * {cos m phi | sin |m| phi}
 * (zernike/base.py:42-68, 228-299). Radial coefficients a_k (for rho^(n-2k)) and
 * derivative coefficients d_k (for rho^(n-2k-1)) live in lens.coef at rad_off and
 * rad_off + n_rad. */
typedef struct ort_zernike_term {
  double c;
  double norm;
  int32_t n;
  int32_t m;
  int32_t rad_off;
  int32_t n_rad;
} ort_zernike_term; /* 32 bytes */

/* Dispersion of one material for per-ray wavelengths (ort_batch.w): n(lambda) by the
 * material's formula (materials/material_file.py:250-428) or tabulated n, k(lambda) by
 * linear interpolation of tabulated data (material_file.py:219-249, numpy.interp
 * semantics), or constants (materials/ideal.py). Lambda-independent subexpressions of
 * the formulas are formed on the host, so coef[coef_off ..] holds
 *   FORMULA_1   1 + C0, then pairs (B_i, C_i ** 2)     n = sqrt(n0 + sum B w^2 / (w^2 - C))
 *   FORMULA_2   1 + C0, then pairs (B_i, C_i)
 *   FORMULA_3   C0, then pairs (A_i, e_i)              n = sqrt(C0 + sum A w^e)
 *   FORMULA_4   C0, C1, C2, C3 ** C4, C5, C6, C7 ** C8, then pairs (A_i, e_i)
 *   FORMULA_5   C0, then pairs (A_i, e_i)              n = C0 + sum A w^e
 *   FORMULA_6   1 + C0, then pairs (B_i, C_i)          n = n0 + sum B / (C - w^-2)
 *   FORMULA_7   C0 .. C(n-1)  (Herzberger)
 *   FORMULA_8   C0 .. C3      (retro)
 *   FORMULA_9   C0 .. C5      (exotic)
 *   TABULATED   lambda_0 .. lambda_(n-1), n_0 .. n_(n-1)  (n_coef = points)
 * and, when k_len > 0, k wavelengths at coef[k_off], k values at coef[k_off + k_len]. */
enum ort_material_kind {
  ORT_MAT_IDEAL = 0,
  ORT_MAT_FORMULA_1 = 1, /* ... ORT_MAT_FORMULA_9 = 9: refractiveindex.info formulas */
  ORT_MAT_TABULATED = 10,
  /* AbbeMaterial (materials/abbe.py:37-51): n = polyval(p, lambda), p_0 .. p_3 in coef
   * (highest power first, numpy.polyval's Horner order), defined on 0.380 .. 0.750 um
   * (outside: NaN here; the host raises the reference's ValueError first), k = 0 */
  ORT_MAT_ABBE = 11
};
typedef struct ort_material {
  int32_t kind;     /* enum ort_material_kind                                          */
  int32_t n_coef;   /* doubles at coef[coef_off] (TABULATED: points)                   */
  int32_t coef_off;
  int32_t k_len;    /* tabulated k points; 0: k = k_const                              */
  int32_t k_off;
  int32_t reserved;
  double n_const;   /* IDEAL: n                                                        */
  double k_const;   /* IDEAL: k (glasses without k data: 0)                            */
} ort_material; /* 40 bytes */

/* The lowered lens (all pointers are device pointers). */
typedef struct ort_lens {
  const ort_surface* surfaces;
  const ort_cs_op* cs_ops;
  const double* coef;
  const ort_zernike_term* zern;
  const double* n_tab;     /* [n_lambda][n_mat] refractive index n(lambda)          */
  const double* alpha_tab; /* [n_lambda][n_mat] 4*pi*k/lambda (0 when k == 0)       */
  const ort_surface_optics* optics; /* [n_lambda][n_surfaces]                       */
  int32_t n_surfaces;      /* traced surfaces S (<= ORT_MAX_SURFACES)               */
  int32_t n_lambda;
  int32_t n_mat;
  int32_t final_mat;       /* material_post of the last surface (image space); < 0:  *
                            * no image-space propagate (bare SurfaceGroup.trace)     */
  uint32_t geometry_mask;  /* OR of (1u << geometry) over the surfaces; selects the  */
                           /* kernel specialisation (no Newton code for sphere lenses) */
  uint32_t interaction_mask; /* OR of (1u << interaction) over the surfaces: anything   */
                             /* beyond REFRACT_REFLECT selects the interaction kernels  */
  double final_thickness;  /* real_ray_tracer.py:84-89 image-space propagate distance */
  const ort_material* materials; /* [n_mat]: per-ray dispersion (ort_batch.w); may be  *
                                  * NULL when no batch carries per-ray wavelengths    */
  const double* wavelengths; /* [n_lambda] um, the wavelength of each table row (phase  *
                              * and grating interactions use it); may be NULL when      *
                              * interaction_mask has no PHASE / DIFFRACTIVE bit         */
  uint32_t frame_flags;      /* enum ort_lens_flags (0: make no assumption)              */
  uint32_t reserved;
} ort_lens;

/* Ray state, structure of arrays, one double per ray per attribute (device). */
typedef struct ort_rays {
  double* x;
  double* y;
  double* z;
  double* L;
  double* M;
  double* N;
  double* i;
  double* opd;
} ort_rays;

/* Per (field, wavelength) segment parameters for in-kernel ray generation
 * (ray_generator.py:71-89 + field_types.py:160-172, infinite object, AngleField,
 * or field_types.py:173-181 finite object). Host scalars are computed in NumPy. */
enum ort_gen_mode {
  ORT_GEN_INFINITE = 0,
  ORT_GEN_FINITE = 1,
  /* object-space telecentric (ray_generator.py:56-73): the pupil target is
   * (Px vx + x0, Py vy + y0, epl) with epl = sqrt(1 - NA^2) / NA + z0 formed on the
   * host; epd is unused */
  ORT_GEN_TELECENTRIC = 2
};
typedef struct ort_segment {
  double epd;      /* EPD (paraxial.py:232-297)                                     */
  double epl;      /* EPL (paraxial.py:207-230); TELECENTRIC: the target plane z    */
  double vx, vy;   /* 1 - vignetting factor                                         */
  double x_off;    /* infinite: -tan(radians(field_x)) * (offset + EPL); finite: x0 */
  double y_off;
  double z0;       /* starting plane z                                              */
  int32_t lambda_idx;
  int32_t mode;    /* enum ort_gen_mode                                             */
} ort_segment; /* 64 bytes */

/* Pupil apodization (the optiland/apodization package): the generated ray's intensity as a
 * function of its normalised pupil coordinates, apodization.get_intensity(Px, Py)
 * (ray_generator.py:91-95; no apodization: 1). r = sqrt(Px^2 + Py^2). Lens-constant
 * subexpressions are formed on the host with the reference's own operations:
 *   GAUSSIAN        p0 = 2 sigma^2        exp(-(Px^2 + Py^2) / p0)          gaussian.py
 *   COSINE_SQUARED  p0 = R, p1 = 2 R      r < R ? cos(pi r / p1)^2 : 0      cosine_squared.py
 *   HANN            p0 = D / 2, p1 = D    r < p0 ? 0.5 (1 - cos(2 pi r / D)) : 0   hann.py
 *   POLYNOMIAL      p0 = R, p1 = p        r < R ? (1 - (r / R)^2)^p : 0     polynomial.py
 *   SUPER_GAUSSIAN  p0 = w, p1 = n        exp(-((r / w)^n))                 super_gaussian.py
 *   TUKEY           p0 = R, p1 = R (1 - alpha / 2), p2 = R alpha / 2:
 *                   r <= p1 ? 1 : r < R ? 0.5 (1 + cos(pi (r - p1) / p2)) : 0   tukey.py */
enum ort_apod_kind {
  ORT_APOD_UNIFORM = 0,
  ORT_APOD_GAUSSIAN = 1,
  ORT_APOD_COSINE_SQUARED = 2,
  ORT_APOD_HANN = 3,
  ORT_APOD_POLYNOMIAL = 4,
  ORT_APOD_SUPER_GAUSSIAN = 5,
  ORT_APOD_TUKEY = 6
};
typedef struct ort_apodization {
  int32_t kind;  /* enum ort_apod_kind */
  int32_t reserved;
  double p[4];
} ort_apodization; /* 40 bytes */

/* A batch of rays: n_rays rays split into consecutive segments of seg_len rays (the
 * reference's field-major layout real_ray_tracer.py:74-77, generalised to (field,
 * wavelength) pairs). Rays also fall into "Newton groups" of group_len consecutive rays:
 * one group is one reference trace call, over which the reference's global Newton stop
 * rule (newton_raphson.py:148) applies. Usually group_len == seg_len (one Optic.trace per
 * (field, wavelength)); trace_generic uses seg_len 1 and group_len n_rays.
 * seg may be NULL: then every ray uses lambda index 0 and no ray generation is possible. */
typedef struct ort_batch {
  int64_t n_rays;
  int64_t seg_len;        /* >= 1                                                    */
  int64_t group_len;      /* >= 1                                                    */
  int32_t n_seg;          /* entries in seg (>= ceil(n_rays / seg_len) when seg set) */
  int32_t pupil_per_ray;  /* px/py hold n_rays points (1) or seg_len points tiled (0) */
  const ort_segment* seg; /* device                                                   */
  /* Per-ray wavelengths in um (device, [n_rays]; NULL: the wavelength of each ray is
   * its segment's lambda_idx into the n_tab / alpha_tab / optics tables). When set,
   * n and k are evaluated per ray and surface from lens.materials, as the reference
   * does for a RealRays with any wavelength array (material.n(rays.w),
   * standard_surface.py:218, refractive_reflective_model.py:32-55, homogeneous.py:30-57).
   * ort_trace_sequential only. */
  const double* w;
  /* Pupil apodization of the generated rays (device, one record; NULL: intensity 1).
   * Read by the entry points that generate rays (ort_trace_pupil, its VJP,
   * ort_generate_rays). */
  const ort_apodization* apod;
} ort_batch;

/* Newton semantics (newton_raphson.py:137-166). */
enum ort_newton_mode {
  /* Every ray performs exactly sched[s] updates at Newton surface s, and the kernel
   * reports per surface the AND over rays of the "converged at update j" bitmask and
   * the max over rays of the last non-converged update index, so the host can verify
   * that sched[s] equals the reference's global stopping index
   * (max|f| < tol over ALL rays). See ort_newton_stat. */
  ORT_NEWTON_SCHEDULE = 0,
  /* Per-wavefront early exit: a wave stops when all of its 64 lanes have
   * |f| < tol (or max_iter). Faster, not bit-identical to the global criterion. */
  ORT_NEWTON_WAVE = 1
};

/* Newton statistics of one (group, surface). The "stop index" k of an update sequence is
 * the number of updates after which the reference's global test would pass: for the
 * Newton-Raphson kinds the test |f(t_k)| < tol evaluated before update k (k = 0 .. U,
 * newton_raphson.py:140-149), for GRID_SAG the test |dt| < tol after update k - 1
 * (k = 1 .. U, grid_sag.py:125-129; bit 0 is never set). */
typedef struct ort_newton_stat {
  uint64_t conv_mask[2]; /* AND over rays: bit b of word w set when the test passed at
                            stop index k = opt.conv_base + 64 w + b (a 128-index window) */
  int32_t last_bad;      /* max over rays of the largest k <= sched that failed the test
                            (or was NaN); -1 when every ray passed at every k            */
  int32_t max_updates;   /* ORT_NEWTON_WAVE: max updates any wave performed              */
} ort_newton_stat; /* 24 bytes */

typedef struct ort_options {
  int32_t newton_mode;   /* enum ort_newton_mode                                     */
  int32_t start_surface; /* SurfaceGroup.trace skip, counted in traced surfaces (>= 0) */
  /* ORT_NEWTON_SCHEDULE: device int32 [n_groups][n_surfaces], updates per Newton group
   * and surface (entries of non-Newton surfaces are ignored). NULL means "max_iter"
   * everywhere. */
  const int32_t* sched;
  /* first stop index of the ort_newton_stat.conv_mask window (>= 0; 0 covers every
   * schedule up to 127 updates -- the default max_iter is 100) */
  int32_t conv_base;
  int32_t flags;          /* ORT_OPT_NO_INIT: newton_stat / status are already initialised */
                          /* (by ort_newton_fixup): the call issues no memset;            */
                          /* ORT_OPT_EXACT: every ray on the per-operation exact sequences  */
                          /* (no deferred-check pass; the results are the same bits --    */
                          /* this is for checking exactly that)                            */
  /* nullable device int32: the launch does nothing unless *run_if == 1 (read on the
   * device; lenses with Newton surfaces only). With ort_newton_fixup this re-traces on a
   * corrected schedule without a host round trip. */
  const int32_t* run_if;
  /* nullable device double [rows][n_rays] (v19: rows = the sum over the surfaces of 7 for
   * a plane / conic, 11 for a Newton surface, surface by surface; ort_vjp_tape_size bytes
   * hold any lens's tape): a Newton-lens launch with this set writes
   * the adjoint tape of its own rays as it traces (each surface's incoming global ray,
   * its distance t and the Newton iterates before the last four updates, the initial
   * guess in the iterate rows no update fills -- every row written), so the
   * backward (ort_vjp_params.tape) runs the reverse sweep only */
  double* tape;
  /* Verify-and-re-trace (ABI v14; nullable): with verify_stats set, the launch first
   * applies ort_newton_fixup's rule to verify_stats (the ort_newton_stat of the launch that
   * ran *sched) -- every workgroup derives the same decision -- writes the decision to
   * *verify_flag and the schedule to sched_out (device int32 [n_groups][n_surfaces], not
   * sched), and traces on the corrected schedule only when the decision is 1; a
   * verify_prev_flag (nullable) other than 1 is passed on to *verify_flag and nothing is
   * traced. One launch in place of ort_newton_fixup + a run_if re-launch. Needs a lens
   * with Newton surfaces, ORT_NEWTON_SCHEDULE, ORT_OPT_NO_INIT (newton_stat / status
   * initialised by the caller) and n_groups * n_surfaces <= ORT_VERIFY_MAX_SCHED. */
  const ort_newton_stat* verify_stats;
  const int32_t* verify_prev_flag;
  int32_t* verify_flag;
  int32_t* sched_out;
  /* ort_trace_pupil with a tape (v18; nullable): every workgroup of 256 rays also writes
   * rms_part[workgroup][4] = { rays, sum x, sum y, sum of (x - mx)^2 + (y - my)^2 about the
   * workgroup's own mean } of its final (image) points -- RayOperand.rms_spot_size's
   * reduction (optimization/operand/ray.py:300-340) on the rays still in registers; then
   * ort_rms_finish combines the rows. ceil(n_rays / 256) rows. */
  double* rms_part;
} ort_options;
#define ORT_VERIFY_MAX_SCHED 1024
enum ort_option_flags { ORT_OPT_NO_INIT = 1, ORT_OPT_EXACT = 2 };

/* status bits written with atomicOr into *status (device int32) */
enum ort_status {
  ORT_STATUS_ZERNIKE_RANGE = 1u << 0,   /* zernike.py:234-246 ValueError            */
  ORT_STATUS_CHEBYSHEV_RANGE = 1u << 1, /* chebyshev.py:203-215 ValueError          */
  ORT_STATUS_BAD_GEOMETRY = 1u << 2,    /* a surface with an unknown geometry id: its
                                           rays are NaN (never a silent substitute)  */
  ORT_STATUS_BAD_APODIZATION = 1u << 3  /* ort_batch.apod holds an unknown kind: the
                                           generated intensities are NaN             */
};

/* Pupil distribution generated on the device (distribution.py:72-408), see
 * ort_generate_pupil. Tables are device memory prepared by the host (a few KB). */
enum ort_pupil_kind {
  ORT_PUPIL_UNIFORM = 0,   /* linspace grid masked to the unit disk        */
  ORT_PUPIL_HEXAPOLAR = 1, /* 1 + 3 n (n + 1) points on n rings            */
  ORT_PUPIL_RANDOM = 2,    /* numpy default_rng (PCG64) uniform r, theta   */
  ORT_PUPIL_RING = 3,
  ORT_PUPIL_LINE_X = 4,
  ORT_PUPIL_LINE_Y = 5,
  ORT_PUPIL_CROSS = 6
};
typedef struct ort_pupil {
  int32_t kind;              /* ort_pupil_kind                                        */
  int32_t positive_only;     /* LINE_X / LINE_Y: linspace(0, 1, n) instead of (-1, 1)  */
  int64_t n;                 /* the distribution's num_points / num_rings argument    */
  int64_t n_points;          /* points generated                                      */
  int32_t n_rows;            /* UNIFORM: grid rows holding points                     */
  int32_t reserved;
  const int64_t* row_start;  /* UNIFORM [n_rows]: index of the row's first point      */
  const int64_t* row_col;    /* UNIFORM [n_rows][2]: grid row, its first column       */
  const uint64_t* rng_chunk; /* RANDOM [ceil(n_points / 256)][4]: PCG64 state (lo, hi) *
                              * before draw 256 c (radii) and before draw n_points +   *
                              * 256 c (angles)                                        */
  const uint64_t* rng_lane;  /* RANDOM [256][4]: the LCG map advanced l + 1 steps:     *
                              * multiplier (lo, hi), increment (lo, hi)               */
} ort_pupil;

/* ---- entry points ------------------------------------------------------------- */

int ort_abi_version(void);

/* Trace rays_in through the lens, writing rays_out (may alias rays_in for an in-place
 * trace, as the reference mutates RealRays in place). rec (nullable) receives
 * [n_rec][8][n_rays] doubles (x,y,z,L,M,N,i,opd) after every surface flagged
 * ORT_SURF_RECORD, at its rec_slot (standard_surface.py:266-286). newton_stat
 * (nullable; device, [n_groups][n_surfaces] entries, n_groups =
 * ceil(n_rays / group_len)) and status (nullable;
 * device int32) are initialised by this call. Returns 0, or a negative ort_error. */
int ort_trace_sequential(const ort_lens* lens, const ort_rays* rays_in, ort_rays* rays_out,
                         const ort_batch* batch, const ort_options* opt, double* rec,
                         ort_newton_stat* newton_stat, int32_t* status, void* stream);

/* Generate rays from pupil samples and trace them in one launch (the pupil
 * coordinates are the only per-ray input: 16 bytes per ray). With pupil_per_ray == 0,
 * px, py hold seg_len pupil points shared by every segment (real_ray_tracer.py:74-77:
 * Px tiled over fields). */
int ort_trace_pupil(const ort_lens* lens, const double* px, const double* py,
                    ort_rays* rays_out, const ort_batch* batch, const ort_options* opt,
                    double* rec, ort_newton_stat* newton_stat, int32_t* status,
                    void* stream);

/* Parameters of the backward pass. Parameter p (0 <= p < n_param) enters the trace
 * through any of: the coefficient of Zernike term j of lens->zern (zern_param[j] == p),
 * the radius / conic / vertex z of traced surface s (surf_tangent[(p*S + s)*3 + 0/1/2]
 * = d value / d p; a thickness variable moves the vertices after it), the image-space
 * propagation distance (final_tangent[p]). NULL tables contribute nothing.
 *
 * mode ORT_VJP_UNROLLED: forward-mode tangents through the primal's exact Newton
 *   update counts (the derivative of the unrolled iteration, as torch autograd computes
 *   it); one re-trace per 4 parameters. Needs a device workspace of
 *   ort_vjp_workspace_size() bytes (v15: the per-block partial sums, reduced in a fixed
 *   order -- the gradient is the same bits run to run).
 * mode ORT_VJP_ADJOINT: one reverse-mode pass whatever n_param: closed-form
 *   intersections through their implicit equations, Newton intersections through the
 *   last kHist = 4 updates of the unrolled iteration (taped iterates) and the initial
 *   guess -- the unrolled derivative exactly when a surface ran U <= 4 updates; with
 *   U > 4 the older updates are dropped (their share is a product of converged
 *   residuals) except on ORT_SURF_SLOPE_INEXACT surfaces (standard / noll Zernike, whose
 *   Newton slope omits the normalisation constant and converges linearly), where U > 4
 *   writes NaN into the gradient: take ORT_VJP_UNROLLED for such a schedule (v19).
 *   Needs n_zern and a device workspace of ort_vjp_workspace_size() bytes, and at most
 *   ORT_VJP_ADJOINT_MAX_SLOTS parameter slots, 3 n_surfaces + n_zern + 1 (v17: the
 *   slots' per-block partial sums live in LDS); beyond that use ORT_VJP_UNROLLED.
 * Lenses with thin-lens / phase / grating surfaces (interaction_mask beyond
 * REFRACT_REFLECT): ORT_VJP_UNROLLED only (v20: the forward-mode sweep carries the
 * interaction models in duals; the adjoint refuses them with ORT_ERR_ARG, as both modes
 * refuse GRID_SAG / NURBS surfaces). A grating surface's radius / conic take no tangent
 * (its grating-vector constants are host-formed). */
#define ORT_VJP_ADJOINT_MAX_SLOTS 512
enum ort_vjp_mode { ORT_VJP_UNROLLED = 0, ORT_VJP_ADJOINT = 1 };
typedef struct ort_vjp_params {
  int32_t n_param;
  int32_t mode;                /* ort_vjp_mode                                          */
  const int32_t* zern_param;   /* [n_zern] parameter index per term, < 0: constant      */
  const double* surf_tangent;  /* [n_param][n_surfaces][3]                              */
  const double* final_tangent; /* [n_param]                                             */
  int32_t n_zern;              /* entries of zern_param (terms of lens->zern)           */
  int32_t grad_init;           /* 1: grad is overwritten with the VJP (no zeroing first; */
                               /* v14, formerly reserved = 0: accumulate)               */
  void* workspace;             /* device scratch (ADJOINT: tape + wave partials;         */
                               /* UNROLLED: block partials)                             */
  int64_t workspace_size;      /* bytes available at workspace                          */
  /* ADJOINT, nullable: device int32 [n_slot] (n_slot = 3 n_surfaces + n_zern + 1, slot
   * order: radius, conic, vertex z of each surface, the Zernike terms, the final
   * thickness), nonzero where some tangent is nonzero -- the slots the kernel must sum.
   * It depends only on the tangent tables, so a caller that keeps them resident can keep
   * this too; NULL: derived on the device by one extra launch per call. */
  const int32_t* slot_need;
  /* ADJOINT, nullable: the tape the primal ort_trace_pupil wrote (ort_options.tape, with
   * the schedule of opt): the kernel skips its own forward re-trace and reads the final
   * ray state from `primal` (that launch's outputs: L, M, N and i are read). */
  const double* tape;
  ort_rays primal;
  /* ADJOINT (v18): Zernike coefficient adjoints in the Cartesian monomial basis. 0: one
   * slot per Zernike term (as before v18). Otherwise the number of monomial slots of the
   * lens, sum over its Zernike surfaces with a Cartesian block (zm_deg >= 0) of
   * (zm_deg + 1)(zm_deg + 2) -- two per monomial: the sag's and the normal slopes' --
   * appended after the final-thickness slot in surface order (n_slot = 3 n_surfaces +
   * n_zern + 1 + n_mono); the kernel sums per-ray monomial values over the rays and the
   * parameter reduction applies the surfaces' term matrices (Ms / Mn of the block) once
   * per launch. A value that is not the lens's count disables the basis (per-term slots
   * serve; the workspace is still sized with it). Requires zern_param. slot_need, when
   * given, covers all n_slot slots. */
  int32_t n_mono;
  int32_t reserved;
  /* ADJOINT with params->tape (v18; nullable): the cotangents of the x and y outputs gain
   * those of an rms spot size rms = sqrt(mean((x - mx)^2 + (y - my)^2)) over all rays:
   * g (x - mx) / (n rms), g (y - my) / (n rms) -- ort_rms_spot_vjp folded into the sweep's
   * cotangent load (the primal's x, y read from params->primal). rms_stats: the 5 doubles
   * of ort_rms_spot / ort_rms_finish (n, mx, my, rms, ...); rms_grad: g (one double). */
  const double* rms_stats;
  const double* rms_grad;
} ort_vjp_params;

/* Workspace bytes params->mode needs for this lens, batch and parameter set (ADJOINT:
 * without the tape when params->tape is set). */
int64_t ort_vjp_workspace_size(const ort_lens* lens, const ort_batch* batch,
                               const ort_vjp_params* params);
/* Bytes that hold the adjoint tape of one trace of this lens (ort_options.tape,
 * ort_vjp_params.tape): n_surfaces x 11 rows of n_rays doubles, the most any lens of
 * n_surfaces surfaces writes (v19: the tape itself has 7 rows per plane / conic). */
int64_t ort_vjp_tape_size(const ort_lens* lens, const ort_batch* batch);

/* Backward of ort_trace_pupil: the vector-Jacobian product
 *   grad[p] += sum_rays sum_f cotangent.f[ray] * d out.f[ray] / d param_p
 * for the output fields f of rays_out (x, y, z, L, M, N, i, opd; a NULL cotangent field
 * counts as zero). opt must be ORT_NEWTON_SCHEDULE with the schedule the verified primal
 * trace ran (see ort_vjp_mode for how Newton surfaces are differentiated). grad is
 * accumulated (one addition per parameter of sums formed in a fixed order, both modes:
 * deterministic): zero it first, or set params->grad_init = 1 to have it overwritten. Ray generation is not differentiated (the reference builds
 * its paraxial quantities from detached copies, surface_group.py:143-153). Replaces
 * reverse-mode torch autograd through the trace (SurfaceGroup.trace under the torch
 * backend, driven by optimization/optimizer/torch/base.py:95-154; variables written by
 * variable/{zernike_coeff,radius,conic,thickness}.py). */
int ort_trace_pupil_vjp(const ort_lens* lens, const double* px, const double* py,
                        const ort_batch* batch, const ort_options* opt,
                        const ort_vjp_params* params, const ort_rays* cotangent,
                        double* grad, void* stream);

/* Backward of ort_trace_sequential (resident rays in, SurfaceGroup.trace under autograd:
 * optimization/optimizer/torch/base.py:116-131 traces under be.grad_mode, and the
 * reference's torch backend differentiates every be.* op of surface_group.py:232-244):
 *   grad[p]      += sum_rays  cotangent . d rays_out / d param_p
 *                           + rec_cotangent . d rec / d param_p
 *   grad_in.f[r]  = d (cotangent . rays_out + rec_cotangent . rec) / d rays_in.f[r]
 * with parameters as for ort_trace_pupil_vjp (params: tangent tables, mode, workspace of
 * ort_vjp_workspace_size bytes for ORT_VJP_ADJOINT). rays_in is the trace's input (the
 * primal must not have traced in place over it); per-ray wavelengths (batch->w) allowed.
 * rec_cotangent (nullable): [n_rec][8][n_rays] cotangents of the record buffer the primal
 * wrote (ORT_SURF_RECORD slots); then rec, that primal record buffer, is required (its
 * intensity rows weight the absorption adjoint). grad_in (nullable; NULL fields are not
 * written): cotangents of the input rays x, y, z, L, M, N, i, opd -- ORT_VJP_ADJOINT only
 * (forward mode carries parameter tangents only: ORT_ERR_ARG). grad is accumulated (zero
 * it first); grad may be NULL when n_param == 0. opt: ORT_NEWTON_SCHEDULE with the
 * schedule the verified primal ran. */
int ort_trace_sequential_vjp(const ort_lens* lens, const ort_rays* rays_in,
                             const ort_batch* batch, const ort_options* opt,
                             const ort_vjp_params* params, const ort_rays* cotangent,
                             const double* rec_cotangent, const double* rec, double* grad,
                             const ort_rays* grad_in, void* stream);

/* Per-geometry primitives of traced surface `surface` of `lens`, in the surface's local
 * frame (no localize / globalize), for n points or rays:
 *   ort_surface_sag_normal: sag(x, y) and the unit normal at (x, y)
 *     (BaseGeometry.sag / surface_normal, e.g. standard.py:73-87, :154-167,
 *     even_asphere.py:82-129, zernike.py:133-231); any output may be NULL.
 *   ort_surface_distance: distance t along each ray to the surface (geometry.distance,
 *     plane.py:61-77, standard.py:89-140, newton_raphson.py:119-168); Newton surfaces
 *     follow the global stop rule over the n rays with opt / newton_stat exactly as
 *     ort_trace_sequential with group_len = n (opt NULL: max_iter updates).
 * status: ORT_STATUS_ZERNIKE_RANGE as for the trace (zernike.py:234-246). */
/* Device-resident Zernike coefficients (v16): zern[rows[i]].c = c[i] for i < n, then every
 * Cartesian block (ort_surface.zm_off) of the lens re-formed from the term table:
 * As = sum_j c_j Ms[j], An = sum_j c_j Mn[j] in term order. Writes the lens's term table
 * and coefficient array (caller-owned device memory the lens points to); one single-
 * workgroup launch, no synchronisation. Replaces the host-side coefficient upload of
 * ZernikeCoeffVariable.update_value (optimization/variable/zernike_coeff.py:71-95) for
 * coefficients held in HBM. */
int ort_patch_zernike(const ort_lens* lens, const double* c, const int64_t* rows, int64_t n,
                      void* stream);
/* The same patch with the coefficients read through a device array of n pointers
 * (c_ptrs[i] -> the value for term row rows[i]): the optimiser's separate parameter
 * tensors are read where they live, without a concatenation launch first (ABI v17). */
int ort_patch_zernike_ptrs(const ort_lens* lens, const double* const* c_ptrs,
                           const int64_t* rows, int64_t n, void* stream);

/* One Adam step of device-resident Zernike coefficients fused with the patch of the lens's
 * term table and Cartesian blocks (v18): torch.optim.Adam's update (amsgrad and maximize
 * off; weight_decay the L2 form: grad + weight_decay * param) of up to ORT_ADAM_MAX_TENSORS
 * parameter tensors, each the coefficients of term rows [row0, row0 + count) of
 * lens->zern, then every touched surface re-formed as ort_patch_zernike does -- one launch
 * for the optimiser's two and the patch. step[k] (v19): a device double, tensor k's Adam
 * step count (torch.optim.Adam's state["step"], incremented here before the update, as torch
 * does); each tensor's rows lie within one Zernike surface, so one workgroup updates it and
 * its count, once per call.
 * Pointers by value (no device pointer table): a HIP graph captures the launch as is.
 * Replaces the optimiser step of optimization/optimizer/torch/base.py:116-132 for
 * ZernikeCoefficientVariables followed by the lens update of the next trace. */
#define ORT_ADAM_MAX_TENSORS 16
typedef struct ort_adam_params {
  int32_t n_tensors;
  int32_t reserved;
  double* param[ORT_ADAM_MAX_TENSORS];
  const double* grad[ORT_ADAM_MAX_TENSORS];
  double* exp_avg[ORT_ADAM_MAX_TENSORS];
  double* exp_avg_sq[ORT_ADAM_MAX_TENSORS];
  int64_t row0[ORT_ADAM_MAX_TENSORS];
  int64_t count[ORT_ADAM_MAX_TENSORS];
  double* step[ORT_ADAM_MAX_TENSORS]; /* v19: per tensor (v18: one per surface) */
  double lr, beta1, beta2, eps, weight_decay;
} ort_adam_params;
int ort_adam_patch_zernike(const ort_lens* lens, const ort_adam_params* p, void* stream);

int ort_surface_sag_normal(const ort_lens* lens, int32_t surface, const double* x,
                           const double* y, int64_t n, double* sag, double* nx, double* ny,
                           double* nz, int32_t* status, void* stream);
int ort_surface_distance(const ort_lens* lens, int32_t surface, const ort_rays* rays,
                         int64_t n, const ort_options* opt, double* t,
                         ort_newton_stat* newton_stat, int32_t* status, void* stream);

/* Device-side check of a Newton schedule (the host's speculate / verify step, see
 * ORT_NEWTON_SCHEDULE), so a warm schedule is verified without a host round trip:
 * reads the statistics `stats` [n_groups][n_surfaces] of a launch that ran `sched` and
 * applies the reference's stopping rule (newton_raphson.py:140-149) per (group, Newton
 * surface): the first stop index k < sched that every ray passed -> sched = k; sched below
 * max_iter with a ray failing at sched -> sched grown (2 sched + 2, at least 8, then
 * max_iter); sched is updated in place. *flag (device int32) = 0 when every schedule was
 * right, 1 when one changed (re-launch with run_if = flag), 2 when a decision needs a
 * conv_mask window beyond the one stats holds (the host must finish). prev_flag
 * (nullable): when *prev_flag != 1 the stats belong to a launch that did not run, so
 * nothing is checked and *flag = *prev_flag. One single-block launch. */
int ort_newton_fixup(const ort_lens* lens, int64_t n_groups, const ort_newton_stat* stats,
                     int32_t conv_base, int32_t* sched, const int32_t* prev_flag,
                     int32_t* flag, ort_newton_stat* next_stats, int32_t* next_status,
                     void* stream);
/* next_stats / next_status (nullable): when *flag becomes 1 they are initialised for the
 * re-launch (launch it with ORT_OPT_NO_INIT), so a round costs two launches. */

/* The last launch of `rounds` verify-and-re-trace rounds (ABI v17) on per-call buffers
 * stats [rounds + 1][n_groups][n_surfaces], flags [rounds + 1], statuses [rounds + 1]:
 * ort_newton_fixup's check of the last round (stats[rounds], sched; prev_flag =
 * flags[rounds - 1], flag = flags[rounds]), then the state the next call on the same
 * buffers starts from -- *status_out = statuses[r] of the last round r that ran (round 0,
 * or the largest r with flags[r - 1] == 1), every statuses[r] = 0, every stats entry 0xFF
 * bytes (conv_mask all ones, last_bad = max_updates = -1) -- and, when sched_copy is not
 * NULL, the settled schedule copied to it (device int32 [n_groups][n_surfaces]). One
 * single-block launch in place of the final fixup, the two initialisations and the copy
 * of every call; the first call's buffers are initialised by the caller. */
int ort_newton_finish(const ort_lens* lens, int64_t n_groups, ort_newton_stat* stats,
                      int32_t rounds, int32_t conv_base, int32_t* sched, int32_t* flags,
                      int32_t* statuses, int32_t* status_out, int32_t* sched_copy,
                      void* stream);

/* ort_newton_finish and ort_rms_finish in ONE launch (v18): a second workgroup combines
 * the taped forward's rms rows (ort_options.rms_part, rms_rows of them) into rms_stats[5]
 * and *rms (nullable) beside the check -- the rows are final once the rounds are. The
 * device-verified rounds of RayOperand.rms_spot_size's trace end with it. */
int ort_newton_finish_rms(const ort_lens* lens, int64_t n_groups, ort_newton_stat* stats,
                          int32_t rounds, int32_t conv_base, int32_t* sched, int32_t* flags,
                          int32_t* statuses, int32_t* status_out, int32_t* sched_copy,
                          const double* rms_part, int64_t rms_rows, double* rms_stats,
                          double* rms, void* stream);

/* Pupil coordinates of a distribution on the device: px[k], py[k] for k < n_points
 * (distribution.py:72-408; the grid kinds bit-identical to NumPy, cos / sin correctly
 * rounded). Feeds ort_trace_pupil without host-side sampling or a host-to-device copy. */
int ort_generate_pupil(const ort_pupil* pupil, double* px, double* py, void* stream);

/* n(lambda) and k(lambda) of material `mat` of the lens (lens.materials) at n device
 * wavelengths: BaseMaterial.n / .k (materials/base.py:73-119) on the device, the same
 * evaluation the trace kernels run per ray when ort_batch.w is set. n_out / k_out are
 * device [n] (either may be NULL). */
int ort_material_nk(const ort_lens* lens, int32_t mat, const double* w, int64_t n,
                    double* n_out, double* k_out, void* stream);

/* ---- spot-diagram statistics (analysis/spot_diagram.py:317-357, 425-437) ----------
 * Traced rays laid out as n_fields x n_wl pairs of n_pupil consecutive rays
 * (pair = field * n_wl + wavelength, the order SpotDiagram traces them in one launch).
 * Points with i > 0 count (spot_diagram.py:425-427); their (x, y, z) are taken into the
 * image-surface frame by local_ops (the surface's localize ops applied to points,
 * visualization/system/utils.py:16-46; n_local_ops = 0: global coordinates). Per pair
 * out[pair][5] = { count, centroid x, centroid y (mean of the pair's points),
 * rms radius, max radius } with both radii about the centroid of the field's ref_wl
 * pair (spot_diagram.py:_center_spots). NaN points propagate as in NumPy; a pair without
 * points gives NaN statistics. Deterministic: every reduction runs in a fixed order,
 * no atomics. */
typedef struct ort_spot_layout {
  int64_t n_pupil;            /* rays per pair                                        */
  int32_t n_fields;
  int32_t n_wl;               /* >= 1                                                 */
  int32_t ref_wl;             /* the reference wavelength's index, 0 <= ref_wl < n_wl */
  int32_t n_local_ops;
  const ort_cs_op* local_ops; /* device [n_local_ops], or NULL when n_local_ops == 0   */
} ort_spot_layout;

/* Bytes of device workspace ort_spot_stats needs for this layout (< 0: ORT_ERR_ARG). */
int64_t ort_spot_workspace_size(const ort_spot_layout* layout);

/* rays: device x, y, z, i of n_fields * n_wl * n_pupil rays (other fields unused; z
 * only with local_ops); out: device [n_fields * n_wl][5]. Three launches on `stream`,
 * no synchronisation, no allocation (graph-capturable). */
int ort_spot_stats(const ort_rays* rays, const ort_spot_layout* layout, void* workspace,
                   int64_t workspace_size, double* out, void* stream);

/* SpotDiagram's trace + statistics (spot_diagram.py:381-438 then :317-357) for a lens
 * without Newton geometries: ort_trace_pupil of the n_fields * n_wl pairs (segments in
 * pair order, batch->seg_len == layout->n_pupil, shared pupil) into rays_out, then
 * out[pair][5] as ort_spot_stats computes it. When each pair's chunks hold one ray per
 * thread (n_pupil <= 65,536) the closed-form kernel writes the statistics' first pass from
 * its epilogue (3 launches: the trace, the second pass, the totals); otherwise 4. The numbers are
 * bit-identical to ort_trace_pupil followed by ort_spot_stats either way. Replaces
 * SpotDiagram._generate_field_data's trace loop + the statistics over its data
 * (analysis/spot_diagram.py:317-357, 381-438). Newton lenses: ORT_ERR_ARG. */
int ort_trace_spot(const ort_lens* lens, const double* px, const double* py,
                   ort_rays* rays_out, const ort_batch* batch, const ort_options* opt,
                   int32_t* status, const ort_spot_layout* layout, void* workspace,
                   int64_t workspace_size, double* out, void* stream);

/* RayOperand.rms_spot_size's reduction (optimization/operand/ray.py:300-340):
 * rms = sqrt(mean((x - mean x)^2 + (y - mean y)^2)) over all n points (no intensity mask),
 * two passes in a fixed order (the spot-statistics kernels with one pair). stats (device
 * double[5]) = { n, mean x, mean y, rms, max radius }; rms (device double, nullable) gets
 * the rms again as its own scalar (the autograd op's output). Three launches.
 * ort_rms_spot_vjp: gx[i] = g (x_i - mean x) / (n rms), gy likewise, g = *grad_out (a
 * device scalar, read on the device: no host synchronisation). One launch. */
int64_t ort_rms_spot_workspace_size(int64_t n);
int ort_rms_spot(const double* x, const double* y, int64_t n, void* workspace,
                 int64_t workspace_size, double* stats, double* rms, void* stream);
int ort_rms_spot_vjp(const double* x, const double* y, int64_t n, const double* stats,
                     const double* grad_out, double* gx, double* gy, void* stream);
/* The rms spot size from the workgroup rows a taped ort_trace_pupil wrote (ort_options.
 * rms_part, n_rows = ceil(n_rays / 256)), one launch (v18): the mean mx, my and
 * sum (x - mx)^2 + (y - my)^2 by Chan's pairwise combination of the rows in index order
 * (deterministic; the same quantity as ort_rms_spot's two passes up to rounding).
 * stats[5] = n, mx, my, rms, NaN (no max radius); *rms = stats[3]. */
int ort_rms_finish(const double* part, int64_t n_rows, double* stats, double* rms,
                   void* stream);

/* Sharded spot statistics: rays holds THIS rank's slice of every pair (layout->n_pupil
 * rays per pair, the same pair order on every rank). Two phases, each two launches:
 *   phase 1: out[pair][3] = { count, sum x, sum y } of this rank's i > 0 points (image
 *            frame); the caller sums them over the ranks (all_reduce) -> sums1;
 *   phase 2: the centroid of each field's ref_wl pair from the reduced sums1, then
 *            out[pair][3] = { sum of (x - cx)^2 + (y - cy)^2, max radius, NaN flag } of
 *            this rank's points; the caller reduces SUM, MAX, MAX over the ranks.
 * Then, as spot_diagram.py:317-357 forms them: centroid = sum / count, rms radius =
 * sqrt(sum r^2 / count), geometric radius = max radius (NaN when the flag is set or the
 * spot is empty). workspace: ort_spot_workspace_size(layout) bytes. */
int ort_spot_partials(const ort_rays* rays, const ort_spot_layout* layout, int32_t phase,
                      const double* sums1, void* workspace, int64_t workspace_size,
                      double* out, void* stream);

/* ---- chief-ray wavefront (wavefront/strategy.py:68-239, opd.py:143-157) ------------
 * Host-formed constants of one (field, wavelength): the reference sphere centred on the
 * chief ray's image point (xc, yc, zc) with r2 = R**2 (R from the chief ray and the exit
 * pupil, strategy.py:236-241), the image-space index, the chief ray's own reference OPD
 * opd_ref (after its tilt correction), and for angle fields (tilt = 1) the launch-plane
 * tilt direction (ux, uy) and EPD (:118-166). xc2 / yc2 / zc2 = xc**2 ... as NumPy forms
 * them; wl_mm = wavelength * 1e-3. */
typedef struct ort_wavefront_ref {
  double xc, yc, zc;
  double xc2, yc2, zc2;
  double r2;
  double n_image;
  double opd_ref;
  double ux, uy;
  double epd;
  double wl_mm;
  int32_t tilt;
  int32_t reserved;
} ort_wavefront_ref; /* 112 bytes */

/* Bytes of device workspace ort_wavefront_opd needs for n rays (< 0: ORT_ERR_ARG). */
int64_t ort_wavefront_workspace_size(int64_t n);

/* rays: the n traced rays at the image (device x, y, z, L, M, N, i, opd); px, py: their
 * pupil coordinates (device, read only when ref->tilt). Writes opd_wv[n] (OPD in waves,
 * strategy.py:226) and, when non-NULL, the exit-pupil points pupil_x / y / z[n]
 * (:227-230), and sums[11] (device): count and sum of opd_wv^2 over i > 0 (opd.py rms)
 * and the intensity-weighted sums w, wx, wy, wxx, wxy, wyy, w opd, wx opd, wy opd of the
 * pupil points for the piston / tilt fit (wavefront.py:97-143). Two launches on
 * `stream`, fixed-order reductions, no synchronisation. */
int ort_wavefront_opd(const ort_rays* rays, const double* px, const double* py, int64_t n,
                      const ort_wavefront_ref* ref, double* opd_wv, double* pupil_x,
                      double* pupil_y, double* pupil_z, void* workspace,
                      int64_t workspace_size, double* sums, void* stream);

/* Ray generation only (ray_generator.py:28-106): fills rays_out from pupil points. */
int ort_generate_rays(const double* px, const double* py, ort_rays* rays_out,
                      const ort_batch* batch, void* stream);

/* Error codes */
enum ort_error {
  ORT_OK = 0,
  ORT_ERR_ARG = -1,      /* null pointer / bad size / unknown geometry_mask bits       */
  ORT_ERR_SURFACES = -2, /* n_surfaces outside [0, ORT_MAX_SURFACES]                  */
  ORT_ERR_LAUNCH = -3    /* hipGetLastError() after launch                            */
};

#ifdef __cplusplus
}
#endif
#endif /* OPTILAND_RT_H */
