"""A second restatement of the integrator's rounds for opaque scenes,
written from the GLSL text apart from oracle/pt_oracle.cpp (test
infrastructure only; tests/test_path_restatement.py).  With
tests/trace_restatement.py for Trace() it re-derives, per pixel, what
Reset / Run(k) leave in the slot state and the accumulator:

  main (seeding, escape -> accumulate -> GenerateNewPath)  basic_scatter.glsl:312-360
  GenerateNewPath / GenerateCameraRay                      basic_scatter.glsl:7-42, scene.glsl.inc:613-655
  LoadTraceResult / LoadPath / StorePathVertexData         basic.glsl.inc:99-131,159-215
  Scatter                                                  basic_scatter.glsl:114-310
  ResolveMedium                                            basic_scatter.glsl:45-66
  SampleSurfaceIntegrand                                   basic_scatter.glsl:68-109
  BasicDiffuse_SampleBSDF / _EvaluateBSDF                  basic_diffuse.glsl.inc
  BasicMetal_GetParameters / _HasDiracBSDF / _Evaluate / _Sample  basic_metal.glsl.inc
  MaterialTexturableReflectance / Value, SampleTexture     scene.glsl.inc:180-302
  SampleSkyboxSpectrum / Radiance (lat-long sky texture)   scene.glsl.inc:206-227
  SampleParametricSpectrum, SampleStandardObserver         spectrum.glsl.inc:10-34,169-192
  RandomDirection, RandomPointOnDisk, RandomVonMisesFisher,
  VonMisesFisherPDF, ComputeCoordinateFrame                common.glsl.inc:120-125,205-254
  GGXRoughnessAlpha / SmithG1 / VisibleNormal / Distribution,
  SchlickFresnelMetal                                      common.glsl.inc:278-360,425-436

  BasicTranslucent_GetParameters / _LoadMedium / _HasDiracBSDF / _Evaluate /
  _SampleBSDF                                              basic_translucent.glsl.inc
  CauchyEmpiricalIOR, ComputeCosThetaRefracted, FresnelDielectric  common.glsl.inc:356-420
  SampleDirectionHG (medium scattering in Scatter)         common.glsl.inc:256-276

Scope: the three basic materials, OpenPBR's default fall-through (the
reference's dispatch has no OpenPBR case, so such a hit ends the path) and
the opt-in OpenPBR sampler (openpbr.glsl.inc:66-515 with DESIGN.md §6 row
4's deviations (a)-(d)), nested media with
absorption and scattering, a scattering scene medium; the sky may be
textured and light-sampled (C1-C5, a metal room, a scattering-glass scene,
the fuzz scenes, tests/test_openpbr.py's scene).
Numerics: DESIGN.md §2's convention (float32, nothing fused, reductions left
to right, normalize = v * (1 / sqrt(dot)), mix = x*(1-a) + y*a); exp, log,
sin, cos, atan2, asin are the convention's own functions (the oracle's
exported pt_exp / pt_log / pt_sin / pt_cos / pt_atan2 / pt_asin), the
octahedral packing tests/kat.py's; pow(x, 5) and pow(x, 6) are products
(x^2 x^2) x and (x^2 x^2) x^2, as GPU compilers lower a constant integer power.
Texture filtering follows the Vulkan rules (SampleTexture below).
"""
from __future__ import annotations

import collections
import ctypes as C

import numpy as np

import kat
import oracle_lib
import trace_restatement as tr

f32 = np.float32
PI = f32(3.141592653)
TAU = f32(6.283185306)
EPSILON = f32(1e-9)
HIT_TIME_LIMIT = f32(1048576.0)
LAMBDA_MIN, LAMBDA_MAX = f32(360.0), f32(830.0)
NONE = 0xFFFFFFFF
STATS = collections.Counter()   # which branches a render took (the tests check coverage)


def _fp(name, *a):
    return f32(getattr(oracle_lib.lib(), f"oracle_fp_{name}")(*[float(x) for x in a]))


class Rng:
    """Random() / Random0To1() (common.glsl.inc:189-202) from main's seed."""

    def __init__(self, x, y, frame):
        self.state = kat.seed(x, y, frame)

    def r01(self):
        v, self.state = kat.pcg(self.state)
        return f32(v) / f32(4294967296.0)


def _mix(a, b, t):
    return a * (f32(1.0) - t) + b * t


def _fract(x):
    return x - np.floor(x)


def _normalize(v):
    # GLSL normalize of a zero vector is inf * 0 = NaN in IEEE float32 (the
    # OpenPBR sampler reaches it); the arithmetic is the restated behaviour.
    with np.errstate(divide="ignore", invalid="ignore"):
        r = f32(1.0) / np.sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2])
        return [v[0] * r, v[1] * r, v[2] * r]


def _safe_normalize(v):
    lsq = (v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]
    if lsq < f32(1e-12):
        return [f32(0.0), f32(0.0), f32(1.0)]
    d = np.sqrt(lsq)
    return [v[0] / d, v[1] / d, v[2] / d]


def _dot(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def _cross(a, b):
    return [a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]]


def _mat_vec(m, v, w):
    w = f32(w)
    return [((m[r] * v[0] + m[4 + r] * v[1]) + m[8 + r] * v[2]) + m[12 + r] * w for r in range(3)]


def _max4(v):
    return np.fmax(np.fmax(v[0], v[1]), np.fmax(v[2], v[3]))


def random_point_on_disk(g):
    r = np.sqrt(g.r01())
    theta = g.r01() * TAU
    return r * _fp("cos", theta), r * _fp("sin", theta)


def random_direction(g):
    z = f32(2.0) * g.r01() - f32(1.0)
    r = np.sqrt(f32(1.0) - z * z)
    phi = TAU * g.r01()
    return [r * _fp("cos", phi), r * _fp("sin", phi), z]


def vmf_pdf(kappa, mu, d):
    """VonMisesFisherPDF (common.glsl.inc:249-254)."""
    if kappa < EPSILON:
        return f32(1.0) / (f32(4.0) * PI)
    c = kappa / ((f32(2.0) * PI) * (f32(1.0) - _fp("exp", f32(-2.0) * kappa)))
    return c * _fp("exp", kappa * (_dot(mu, d) - f32(1.0)))


def coordinate_frame(z):
    """ComputeCoordinateFrame (common.glsl.inc:120-125)."""
    v = [f32(1.0), f32(0.0), f32(0.0)] if abs(z[0]) < f32(0.9) else [f32(0.0), f32(1.0), f32(0.0)]
    x = _normalize(_cross(v, z))
    return x, _cross(x, z)


def random_vmf(g, kappa, mu):
    """RandomVonMisesFisher(Kappa, Mu) (common.glsl.inc:228-247)."""
    xi = g.r01()
    one = f32(1.0)
    z = one + (one / kappa) * _fp("log", xi + (one - xi) * _fp("exp", f32(-2.0) * kappa))
    r = np.sqrt(one - z * z)
    phi = g.r01() * TAU
    v = [r * _fp("cos", phi), r * _fp("sin", phi), z]
    mx, my = coordinate_frame(mu)
    return _safe_normalize([(v[0] * mx[i] + v[1] * my[i]) + v[2] * mu[i] for i in range(3)])


def ggx_alpha(rough, aniso):
    """GGXRoughnessAlpha (common.glsl.inc:281-288)."""
    s = f32(1.0) - aniso
    ax = (rough * rough) * np.sqrt(f32(2.0) / (f32(1.0) + s * s))
    return ax, s * ax


def ggx_g1(d, a):
    """GGXSmithG1 (common.glsl.inc:294-301)."""
    dsq = [d[0] * d[0], d[1] * d[1], d[2] * d[2]]
    if dsq[2] < EPSILON:
        return f32(0.0)
    t = (a[0] * a[0] * dsq[0] + a[1] * a[1] * dsq[1]) / dsq[2]
    return f32(2.0) / (f32(1.0) + np.sqrt(f32(1.0) + t))


def ggx_visible_normal(d, a, u1, u2):
    """GGXVisibleNormal (common.glsl.inc:306-345)."""
    one = f32(1.0)
    vz = _safe_normalize([a[0] * d[0], a[1] * d[1], d[2]])
    lsq = vz[0] * vz[0] + vz[1] * vz[1]
    if lsq > 0:
        ln = np.sqrt(lsq)
        vx = [-vz[1] / ln, vz[0] / ln, f32(0.0) / ln]
    else:
        vx = [one, f32(0.0), f32(0.0)]
    vy = _cross(vz, vx)
    r = np.sqrt(u1)
    phi = TAU * u2
    s = f32(0.5) * (one + vz[2])
    tx = r * _fp("cos", phi)
    ty = (one - s) * np.sqrt(one - tx * tx) + (s * r) * _fp("sin", phi)
    tz = np.sqrt(np.fmax(f32(0.0), (one - tx * tx) - ty * ty))
    n = [(tx * vx[i] + ty * vy[i]) + tz * vz[i] for i in range(3)]
    return _safe_normalize([a[0] * n[0], a[1] * n[1], np.fmax(f32(0.0), n[2])])


def ggx_distribution(n, a):
    """GGXDistribution (common.glsl.inc:349-354)."""
    inv = [f32(1.0) / a[0], f32(1.0) / a[1]]
    b = (n[0] * n[0] * (inv[0] * inv[0]) + n[1] * n[1] * (inv[1] * inv[1])) + n[2] * n[2] * f32(1.0)
    return f32(1.0) / ((((PI * a[0]) * a[1]) * b) * b)


def _pow5(x):
    x2 = x * x
    return (x2 * x2) * x


def _pow6(x):
    x2 = x * x
    return (x2 * x2) * x2


def schlick_fresnel_metal(base, spec, c):
    """SchlickFresnelMetal, F82-tint (common.glsl.inc:425-436)."""
    one = f32(1.0)
    cmax = one / f32(7.0)
    den = cmax * _pow6(one - cmax)
    nom = c * _pow6(one - c)
    out = []
    for k in range(4):
        fs = base[k] + (one - base[k]) * _pow5(one - c)
        fsm = base[k] + (one - base[k]) * _pow5(one - cmax)
        fm = spec[k] * fsm
        out.append(fs - (nom / den) * (fsm - fm))
    return out


def cauchy_ior(base, abbe, lam):
    """CauchyEmpiricalIOR (common.glsl.inc:360-371)."""
    lc, ld, lf = f32(656.3), f32(587.6), f32(486.1)
    one = f32(1.0)
    b = (base - one) / (abbe * (one / (lf * lf) - one / (lc * lc)))
    a = base - b / (ld * ld)
    return [a + b / (l * l) for l in lam]


def cos_refracted(eta, c):
    """ComputeCosThetaRefracted (common.glsl.inc:378-382)."""
    c2 = f32(1.0) - (eta * eta) * (f32(1.0) - c * c)
    return -np.sign(c) * np.sqrt(np.fmax(c2, f32(0.0)))


def fresnel_dielectric(eta, c1, c2):
    """FresnelDielectric(Eta, CosTheta1, CosTheta2) (common.glsl.inc:395-403)."""
    ks = eta * c1
    rs = (ks + c2) / (ks - c2)
    kp = eta * c2
    rp = (kp + c1) / (kp - c1)
    return f32(0.5) * (rs * rs + rp * rp)


def fresnel4(eta, c1, c2=None):
    """The vec4 overloads (common.glsl.inc:406-420)."""
    if c2 is None:
        c2 = [cos_refracted(eta[k], c1[k]) for k in range(4)]
    return [fresnel_dielectric(eta[k], c1[k], c2[k]) for k in range(4)]


def sample_direction_hg(g_, u1, u2):
    """SampleDirectionHG (common.glsl.inc:259-276)."""
    one, two = f32(1.0), f32(2.0)
    if abs(g_) < f32(1e-3):
        z = one - two * u1
    else:
        s = (one - g_ * g_) / ((one + g_) - (two * g_) * u1)
        z = -((one + g_ * g_) - s * s) / (two * g_)
    r = np.sqrt(one - z * z)
    phi = u2 * TAU
    return [r * _fp("cos", phi), r * _fp("sin", phi), z]


def parametric(beta, lam):
    """SampleParametricSpectrum(vec3 Beta, float Lambda)."""
    x = (beta[0] * lam + beta[1]) * lam + beta[2]
    return f32(0.5) + x / (f32(2.0) * np.sqrt(f32(1.0) + x * x))


def observer(lam):
    """SampleStandardObserver (spectrum.glsl.inc:10-34)."""
    def g(mu, lo, hi):
        t = (lam - f32(mu)) * (f32(lo) if lam < f32(mu) else f32(hi))
        return _fp("exp", (f32(-0.5) * t) * t)
    x = (f32(0.362) * g(442.0, 0.0624, 0.0374) + f32(1.056) * g(599.8, 0.0264, 0.0323)) \
        - f32(0.065) * g(501.1, 0.0490, 0.0382)
    y = f32(0.821) * g(568.8, 0.0213, 0.0247) + f32(0.286) * g(530.9, 0.0613, 0.0322)
    z = f32(1.217) * g(437.0, 0.0845, 0.0278) + f32(0.681) * g(459.0, 0.0385, 0.0725)
    return [x, y, z]


class World:
    """The packed scene: trace tables, materials, textures, atlas, camera, globals."""

    def __init__(self, scene):
        self.arrays = scene.arrays()
        packs = scene.packs()
        self.S = tr.Scene(self.arrays)
        self.mat = self.arrays["materials"].astype(np.uint32)
        self.tex = self.arrays["textures"]
        g = self.arrays["globals"][0]
        self.openpbr = False   # ptSetBasicRendererOpenPBR (the opt-in OpenPBR sampler)
        self.sky_index = int(g["SkyboxTextureIndex"])
        self.light_p = f32(g["SkyboxSamplingProbability"])
        self.sky_brightness = f32(g["SkyboxBrightness"])
        self.kappa = f32(g["SkyboxConcentration"])
        self.sky_mean = [f32(c) for c in g["SkyboxMeanDirection"]]
        self.scatter_rate = f32(g["SceneScatterRate"])
        self.aw, self.ah, layers = packs.atlas_width, packs.atlas_height, packs.atlas_layer_count
        n = self.aw * self.ah * layers * 4
        self.atlas = np.frombuffer((C.c_float * n).from_address(packs.atlas), np.float32).reshape(
            layers, self.ah, self.aw, 4) if n else None
        for m in self.S.shape_material:
            assert self.mat[32 * m] in (0, 1, 2, 3), "scope: material types 0-3"

    def mfloat(self, m, a):
        return self.mat[32 * m + a:32 * m + a + 1].view(np.float32)[0]

    def sample_texture(self, index, uv):
        """SampleTexture: textureLod(atlas, (U, V, layer), 0) with REPEAT
        addressing, by the Vulkan filtering rules in full precision: nearest
        takes the texel at floor(u * width); linear blends the four texels
        around u * width - 0.5 with weights (1 - a)(1 - b), a(1 - b),
        (1 - a)b, ab."""
        t = self.tex[index]
        mn, mx = t["AtlasPlacementMinimum"].astype(np.float32), t["AtlasPlacementMaximum"].astype(np.float32)
        u = _mix(mn[0], mx[0], _fract(uv[0]))
        v = _mix(mn[1], mx[1], _fract(uv[1]))
        layer = self.atlas[int(t["AtlasImageIndex"])]
        if int(t["Flags"]) & 1:
            i = int(np.floor(u * f32(self.aw))) % self.aw
            j = int(np.floor(v * f32(self.ah))) % self.ah
            return layer[j, i]
        x = u * f32(self.aw) - f32(0.5)
        y = v * f32(self.ah) - f32(0.5)
        fx, fy = np.floor(x), np.floor(y)
        a, b = x - fx, y - fy
        i0, j0 = int(fx) % self.aw, int(fy) % self.ah
        i1, j1 = (i0 + 1) % self.aw, (j0 + 1) % self.ah
        one = f32(1.0)
        w = [(one - a) * (one - b), a * (one - b), (one - a) * b, a * b]
        t00, t10, t01, t11 = layer[j0, i0], layer[j0, i1], layer[j1, i0], layer[j1, i1]
        return np.array([((w[0] * t00[c] + w[1] * t10[c]) + w[2] * t01[c]) + w[3] * t11[c] for c in range(4)],
                        np.float32)

    def reflectance(self, m, lam, uv, a=1):
        """MaterialTexturableReflectance(m, a) (BASE_SPECTRUM = 1, metal SPECULAR_SPECTRUM = 5)."""
        beta = [self.mfloat(m, a), self.mfloat(m, a + 1), self.mfloat(m, a + 2)]
        value = [parametric(beta, l) for l in lam]
        ti = int(self.mat[32 * m + a + 3])
        if ti != NONE:
            tb = self.sample_texture(ti, uv)
            value = [value[k] * parametric([tb[0], tb[1], tb[2]], lam[k]) for k in range(4)]
        return value

    def value(self, m, a, uv):
        """MaterialTexturableValue (scene.glsl.inc:292-302)."""
        v = self.mfloat(m, a)
        ti = int(self.mat[32 * m + a + 1])
        if ti != NONE:
            v = v * self.sample_texture(ti, uv)[0]
        return v

    def sky_spectrum(self, d):
        """SampleSkyboxSpectrum (scene.glsl.inc:206-218): (beta, intensity)."""
        if self.sky_index == NONE:
            return [f32(0.0), f32(0.0), f32(100.0), f32(1.0)]
        phi = _fp("atan2", d[1], d[0])
        theta = _fp("asin", d[2])
        u = f32(0.5) + phi / TAU
        v = f32(0.5) + theta / PI
        return list(self.sample_texture(self.sky_index, [u, v]))


def new_path(W_, cam, g, x, y, W, H, flags):
    """GenerateNewPath: the ray (origin, packed velocity) and Lambda0."""
    if flags & 2:
        jx = g.r01()
        jy = g.r01()
        sx, sy = f32(x) + jx, f32(y) + jy
    else:
        sx, sy = f32(x) + f32(0.5), f32(y) + f32(0.5)
    nx, ny = sx / f32(W), sy / f32(H)
    model = int(cam["Model"])
    size = cam["SensorSize"].astype(np.float32)
    if model in (0, 1):
        sp = [-size[0] * (nx - f32(0.5)), -size[1] * (f32(0.5) - ny), f32(cam["SensorDistance"])]
        a = f32(cam["ApertureRadius"])
        if model == 0:
            dx, dy = random_point_on_disk(g)
            o = [a * dx, a * dy, f32(0.0)]
            v = _normalize([o[0] - sp[0], o[1] - sp[1], o[2] - sp[2]])
        else:
            fl = f32(cam["FocalLength"])
            den = sp[2] - fl
            op = [(-sp[i] * fl) / den for i in range(3)]
            dx, dy = random_point_on_disk(g)
            o = [a * dx, a * dy, f32(0.0)]
            v = _normalize([op[0] - o[0], op[1] - o[1], op[2] - o[2]])
    else:
        phi = (nx - f32(0.5)) * TAU
        theta = (f32(0.5) - ny) * PI
        ct, st = _fp("cos", theta), _fp("sin", theta)
        o = [f32(0.0)] * 3
        v = [ct * _fp("sin", phi), st, -ct * _fp("cos", phi)]
    to = cam["Transform"]["To"].astype(np.float32).reshape(16)
    O = _mat_vec(to, o, 1.0)
    V = _mat_vec(to, v, 0.0)
    lam0 = g.r01()
    return O, int(kat.pack_unit_vector(np.array([V], np.float32))[0]), lam0


class Slot:
    __slots__ = ("O", "PV", "lam0", "thr", "prob", "sample", "active")

    def start(self, O, PV, lam0):
        self.O, self.PV, self.lam0 = O, PV, lam0
        self.thr = [f32(1.0)] * 4
        self.prob = [f32(1.0)] * 4
        self.sample = [f32(0.0)] * 3
        self.active = [NONE] * 4


def resolve_medium(W_, shape, lam):
    """ResolveMedium (basic_scatter.glsl:45-66): (priority, ior, absorption,
    scattering, anisotropy); BasicTranslucent_LoadMedium for glass, vacuum for
    the other materials (DESIGN.md §2 deviation 2)."""
    zero = [f32(0.0)] * 4
    if shape == NONE:
        return NONE, [f32(1.0)] * 4, zero, [W_.scatter_rate] * 4, f32(0.0)
    m = W_.S.shape_material[shape]
    typ = W_.mat[32 * m]
    if typ == 2:     # BasicTranslucent_LoadMedium
        a_ior, a_abbe, a_depth, a_tr, a_sc, a_aniso = 1, 2, 10, 7, 11, 14
    elif typ == 3 and W_.openpbr:   # OpenPBR_Medium (openpbr.glsl.inc:160-191)
        a_ior, a_abbe, a_depth, a_tr, a_sc, a_aniso = 13, 26, 25, 17, 21, 24
    else:
        return shape, [f32(1.0)] * 4, zero, zero, f32(0.0)
    ior = cauchy_ior(W_.mfloat(m, a_ior), W_.mfloat(m, a_abbe), lam)
    depth = W_.mfloat(m, a_depth)
    if depth > 0:
        tr_ = [parametric([W_.mfloat(m, a_tr + i) for i in range(3)], l) for l in lam]
        sc = [parametric([W_.mfloat(m, a_sc + i) for i in range(3)], l) / depth for l in lam]
        ext = [-_fp("log", t) / depth for t in tr_]
        return shape, ior, [np.fmax(ext[k] - sc[k], f32(0.0)) for k in range(4)], sc, W_.mfloat(m, a_aniso)
    return shape, ior, zero, zero, f32(0.0)


def metal_parameters(W_, m, lam, uv):
    """BasicMetal_GetParameters: base, specular, alpha, rough."""
    base = W_.reflectance(m, lam, uv, 1)
    spec = W_.reflectance(m, lam, uv, 5)
    a = ggx_alpha(W_.value(m, 9, uv), W_.value(m, 11, uv))
    return base, spec, a, bool(a[0] * a[1] > EPSILON)


def evaluate_bsdf(W_, m, lam, uv, exterior, In, Out):
    """MaterialEvaluateBSDF (In = the path's Out, Out = the new In):
    (ok, throughput, probability)."""
    if W_.mat[32 * m] == 2:
        return translucent_evaluate(W_, m, lam, uv, exterior, In, Out)
    if W_.mat[32 * m] == 3:   # OpenPBR: not dispatched (scene.glsl.inc:686-692,735)
        return False, None, None
    if W_.mat[32 * m] == 0:
        r = W_.reflectance(m, lam, uv)
        p = In[2] / PI
        return True, [p * r[k] for k in range(4)], [p] * 4
    base, spec, a, rough = metal_parameters(W_, m, lam, uv)
    if In[2] <= 0 or Out[2] <= 0 or not rough:
        return False, None, None
    h = _safe_normalize([In[i] + Out[i] for i in range(3)])
    gm = ggx_g1(In, a)
    d = ggx_distribution(h, a)
    p = (gm * d) / (f32(4.0) * In[2])
    gs = ggx_g1(Out, a)
    f = schlick_fresnel_metal(base, spec, _dot(In, h))
    return True, [(p * gs) * f[k] for k in range(4)], [p] * 4


def sample_bsdf(W_, g, m, lam, uv, exterior, In):
    """MaterialSampleBSDF: (ok, Out, throughput, probability)."""
    if W_.mat[32 * m] == 2:
        return translucent_sample(W_, g, m, lam, uv, exterior, In)
    if W_.mat[32 * m] == 3:
        if not W_.openpbr:
            return False, None, None, None
        q = openpbr_parameters(W_, g, m, lam, uv, exterior)
        return openpbr_sample(g, q, In)
    if W_.mat[32 * m] == 0:
        d = random_direction(g)
        Out = _safe_normalize([d[0], d[1], d[2] + f32(1.0)])
        return (True, Out) + evaluate_bsdf(W_, m, lam, uv, exterior, In, Out)[1:]
    base, spec, a, rough = metal_parameters(W_, m, lam, uv)
    if In[2] <= 0:
        return False, None, None, None
    u1 = g.r01()
    u2 = g.r01()
    n = ggx_visible_normal(In, a, u1, u2)
    c = min(_dot(n, In), f32(1.0))
    Out = [(f32(2.0) * c) * n[i] - In[i] for i in range(3)]
    if Out[2] <= 0:
        return False, None, None, None
    p = f32(1.0)
    if rough:
        gm = ggx_g1(In, a)
        d = ggx_distribution(n, a)
        p = p * ((gm * d) / (f32(4.0) * In[2]))
    gs = ggx_g1(Out, a)
    f = schlick_fresnel_metal(base, spec, c)
    return True, Out, [(p * gs) * f[k] for k in range(4)], [p] * 4


def translucent_parameters(W_, m, lam, uv, In, exterior):
    """BasicTranslucent_GetParameters: relative IOR, alpha, rough."""
    interior = cauchy_ior(W_.mfloat(m, 1), W_.mfloat(m, 2), lam)
    if In[2] < 0:
        rel = [interior[k] / exterior[k] for k in range(4)]
    else:
        rel = [exterior[k] / interior[k] for k in range(4)]
    a = ggx_alpha(W_.value(m, 3, uv), W_.value(m, 5, uv))
    return rel, a, bool(a[0] * a[1] > EPSILON)


def _refraction_terms(In, Out, rel, a, cin, cout, d0=None, n0=None):
    """The rough refraction probability D (1 - F) Gm J |cos / In.z| shared
    by evaluate and sample (basic_translucent.glsl.inc)."""
    f = fresnel4(rel, cin, cout)
    d = [f32(0.0)] * 4
    for k in range(4):
        if k == 0 and d0 is not None:
            d[0] = d0
        elif cin[k] * cout[k] < 0:
            d[k] = ggx_distribution(n0[k], a)
    gm = ggx_g1(In, a)
    one = f32(1.0)
    out = []
    for k in range(4):
        t = cin[k] * rel[k] + cout[k]
        j = abs(cout[k]) / (t * t)
        out.append((((d[k] * (one - f[k])) * gm) * j) * abs(cin[k] / In[2]))
    return out


def translucent_evaluate(W_, m, lam, uv, exterior, In, Out):
    rel, a, rough = translucent_parameters(W_, m, lam, uv, In, exterior)
    if not rough:
        return True, [f32(0.0)] * 4, [f32(0.0)] * 4
    gm = ggx_g1(In, a)
    if In[2] * Out[2] > 0:
        h = _safe_normalize([Out[i] + In[i] for i in range(3)])
        c = _dot(h, In)
        f = fresnel4(rel, [c] * 4)
        d = ggx_distribution(h, a)
        p = [((f[k] * gm) * d) / (f32(4.0) * In[2]) for k in range(4)]
    else:
        hs = [_safe_normalize([Out[i] + In[i] * rel[k] for i in range(3)]) for k in range(4)]
        cin = [_dot(In, hs[k]) for k in range(4)]
        cout = [_dot(Out, hs[k]) for k in range(4)]
        p = _refraction_terms(In, Out, rel, a, cin, cout, n0=hs)
    gs = ggx_g1(Out, a)
    return True, [p[k] * gs for k in range(4)], p


def translucent_sample(W_, g, m, lam, uv, exterior, In):
    rel, a, rough = translucent_parameters(W_, m, lam, uv, In, exterior)
    u1 = g.r01()
    u2 = g.r01()
    sg = np.sign(In[2])
    n = ggx_visible_normal([In[0] * sg, In[1] * sg, In[2] * sg], a, u1, u2)
    c = np.clip(_dot(n, In), f32(-1.0), f32(1.0))
    cr = cos_refracted(rel[0], c)
    refl = fresnel_dielectric(rel[0], c, cr)
    if g.r01() < refl:
        STATS["reflect"] += 1
        Out = [(f32(2.0) * c) * n[i] - In[i] for i in range(3)]
        if Out[2] * In[2] <= 0:
            return False, None, None, None
        p = fresnel4(rel, [c] * 4)
        if rough:
            gm = ggx_g1(In, a)
            d = ggx_distribution(n, a)
            p = [p[k] * ((gm * d) / (f32(4.0) * abs(In[2]))) for k in range(4)]
        gs = ggx_g1(Out, a)
        return True, Out, [p[k] * gs for k in range(4)], p
    STATS["refract"] += 1
    Out = [(cr + rel[0] * c) * n[i] - rel[0] * In[i] for i in range(3)]
    if Out[2] * In[2] >= 0:
        return False, None, None, None
    if rough:
        ns = [n] + [_safe_normalize([Out[i] + In[i] * rel[k] for i in range(3)]) for k in (1, 2, 3)]
        cin = [c] + [_dot(In, ns[k]) for k in (1, 2, 3)]
        cout = [cr] + [_dot(Out, ns[k]) for k in (1, 2, 3)]
        p = _refraction_terms(In, Out, rel, a, cin, cout, d0=ggx_distribution(n, a), n0=ns)
    else:
        p = [f32(1.0) - refl, f32(0.0), f32(0.0), f32(0.0)]
    gs = ggx_g1(Out, a)
    return True, Out, [p[k] * gs for k in range(4)], p


def _pow(x, y):
    """pow(x, y) = exp(y log x) on the convention's exp / log."""
    return _fp("exp", y * _fp("log", x))


class OpenPBRParameters:
    pass


def openpbr_parameters(W_, g, m, lam, uv, exterior):
    """OpenPBR_Parameters (openpbr.glsl.inc:66-158); Emission is never read
    by OpenPBR_Sample and is not evaluated."""
    f = lambda a: W_.mfloat(m, a)   # noqa: E731
    q = OpenPBRParameters()
    q.lam = lam
    q.coat = g.r01() < f(32)
    q.metal = g.r01() < f(7)
    q.translucent = (not q.metal) and g.r01() < f(20)
    q.base = [f(2) * parametric([f(3), f(4), f(5)], l) for l in lam]
    q.diffuse_roughness = f(8)
    ti = int(W_.mat[32 * m + 6])
    if ti != NONE:
        tb = W_.sample_texture(ti, uv)
        q.base = [q.base[k] * parametric([tb[0], tb[1], tb[2]], lam[k]) for k in range(4)]
    if q.coat:
        q.coat_rel = [exterior[k] / f(36) for k in range(4)]
        q.coat_tr = [parametric([f(33), f(34), f(35)], l) for l in lam]
        q.coat_alpha = ggx_alpha(f(37), f(38))
    q.spec_weight = f(9)
    q.spec = [parametric([f(10), f(11), f(12)], l) for l in lam]
    sior = cauchy_ior(f(13), f(26), lam)
    if q.coat:
        q.spec_rel = [f(36) / sior[k] for k in range(4)]
    else:
        q.spec_rel = [exterior[k] / sior[k] for k in range(4)]
    rough = f(14)
    ti = int(W_.mat[32 * m + 15])
    if ti != NONE:
        rough = rough * W_.sample_texture(ti, uv)[0]
    q.spec_alpha = ggx_alpha(rough, f(16))
    q.bounces = int(W_.mat[32 * m + 1])
    return q


def _sgn3(v):
    s_ = np.sign(v[2])
    return [v[0] * s_, v[1] * s_, v[2] * s_]


def openpbr_coat(g, q, Out, thr, dens):
    """OpenPBR_CoatSample (openpbr.glsl.inc:194-283); the Fresnel call takes
    (Eta, CosTheta, CosThetaRefracted)."""
    if not q.coat:
        return [-Out[0], -Out[1], -Out[2]], thr, dens
    u1 = g.r01()
    u2 = g.r01()
    n = ggx_visible_normal(_sgn3(Out), q.coat_alpha, u1, u2)
    c = _dot(n, Out)
    rel = q.coat_rel
    if Out[2] < 0:
        rel = [f32(1.0) / r for r in rel]
    one = f32(1.0)
    rcs = one - (rel[0] * rel[0]) * (one - c * c)
    rc = -np.sign(Out[2]) * np.sqrt(np.fmax(rcs, f32(0.0)))
    refl = fresnel_dielectric(rel[0], c, rc)
    if g.r01() < refl:
        STATS["coat_reflect"] += 1
        In = [(f32(2.0) * c) * n[i] - Out[i] for i in range(3)]
        if In[2] * Out[2] <= 0:
            return In, thr, [f32(0.0)] * 4
        g1 = ggx_g1(In, q.coat_alpha)
        thr = [t * g1 for t in thr]
        if Out[2] < 0:
            e = -(f32(0.5) / Out[2] + f32(0.5) / In[2])
            thr = [thr[k] * _pow(q.coat_tr[k], e) for k in range(4)]
    else:
        STATS["coat_refract"] += 1
        In = [(rel[0] * c + rc) * n[i] - rel[0] * Out[i] for i in range(3)]
        if In[2] * Out[2] > 0:
            return In, thr, [f32(0.0)] * 4
        g1 = ggx_g1(In, q.coat_alpha)
        thr = [t * g1 for t in thr]
        e = f32(-0.5) / Out[2] if Out[2] < 0 else f32(-0.5) / In[2]
        thr = [thr[k] * _pow(q.coat_tr[k], e) for k in range(4)]
    return In, thr, dens


def openpbr_specular(g, q, Out, thr, dens):
    """OpenPBR_BaseSpecularSample (openpbr.glsl.inc:286-435); rough
    refraction keeps the reference's zero Fresnel vector (:390-391)."""
    one = f32(1.0)
    u1 = g.r01()
    u2 = g.r01()
    n = ggx_visible_normal(_sgn3(Out), q.spec_alpha, u1, u2)
    c = _dot(n, Out)
    if q.metal:
        STATS["spec_metal"] += 1
        In = [(f32(2.0) * c) * n[i] - Out[i] for i in range(3)]
        if Out[2] * In[2] <= 0:
            return In, thr, [f32(0.0)] * 4
        sh = ggx_g1(Out, q.spec_alpha)
        fr = [q.spec_weight * x for x in schlick_fresnel_metal(q.base, q.spec, abs(c))]
        return In, [thr[k] * (fr[k] * sh) for k in range(4)], dens
    rel = q.spec_rel
    if Out[2] < 0:
        rel = [one / r for r in rel]
    if q.spec_weight < one:
        sw = np.sqrt(q.spec_weight)
        R = [(sw * (one - r)) / (one + r) for r in rel]
        rel = [(one - x) / (one + x) for x in R]
    rc = cos_refracted(rel[0], c)
    refl = fresnel_dielectric(rel[0], c, rc)
    if g.r01() < refl:
        STATS["spec_reflect"] += 1
        In = [(f32(2.0) * c) * n[i] - Out[i] for i in range(3)]
        if In[2] * Out[2] <= 0:
            return In, thr, [f32(0.0)] * 4
        if Out[2] > 0:
            thr = [thr[k] * q.spec[k] for k in range(4)]
        g1 = ggx_g1(In, q.spec_alpha)
        return In, [t * g1 for t in thr], dens
    In = [(rel[0] * c + rc) * n[i] - rel[0] * Out[i] for i in range(3)]
    if In[2] * Out[2] > 0:
        return In, thr, [f32(0.0)] * 4
    sh = ggx_g1(In, q.spec_alpha)
    a = q.spec_alpha
    STATS["spec_refract"] += 1
    if np.sqrt(a[0] * a[0] + a[1] * a[1]) > EPSILON:
        fr = [f32(0.0)] * 4
        ns = [None] + [_safe_normalize([In[i] + Out[i] * rel[k] for i in range(3)]) for k in (1, 2, 3)]
        d = [ggx_distribution(n, a), f32(0.0), f32(0.0), f32(0.0)]
        for k in (1, 2, 3):
            if _dot(In, ns[k]) * _dot(Out, ns[k]) < 0:
                d[k] = ggx_distribution(ns[k], a)
        mx = np.fmax(EPSILON, _max4(d))
        d = [x / mx for x in d]
        return In, [thr[k] * ((d[k] * fr[k]) * sh) for k in range(4)], [dens[k] * (d[k] * fr[k]) for k in range(4)]
    return (In, [thr[0] * sh, thr[1] * f32(0.0), thr[2] * f32(0.0), thr[3] * f32(0.0)],
            [dens[0] * one, dens[1] * f32(0.0), dens[2] * f32(0.0), dens[3] * f32(0.0)])


def openpbr_diffuse(g, q, Out, thr):
    """OpenPBR_BaseDiffuseSample (openpbr.glsl.inc:438-461): Oren-Nayar."""
    if q.translucent:
        return [-Out[0], -Out[1], -Out[2]], thr
    STATS["oren_nayar"] += 1
    d = random_direction(g)
    In = _safe_normalize([d[0], d[1], d[2] + f32(1.0)])
    S = _dot(In, Out) - In[2] * Out[2]
    T = np.fmax(In[2], Out[2]) if S > 0 else f32(1.0)
    s2 = q.diffuse_roughness * q.diffuse_roughness
    one = f32(1.0)
    A = [(one - (f32(0.5) * s2) / (s2 + f32(0.33))) + ((f32(0.17) * b) * s2) / (s2 + f32(0.13)) for b in q.base]
    B = (f32(0.45) * s2) / (s2 + f32(0.09))
    return In, [thr[k] * (q.base[k] * (A[k] + (B * S) / T)) for k in range(4)]


def openpbr_sample(g, q, Out):
    """OpenPBR_Sample (openpbr.glsl.inc:463-515): the layer walk.
    (ok, In, throughput, probability); In = -Out with no bounce (DESIGN.md
    §6 row 4 (c))."""
    EXTERNAL, COAT, SPEC, DIFF = -1, 0, 1, 2
    STATS["openpbr_walk"] += 1
    layer = (COAT if q.coat else SPEC) if Out[2] > 0 else SPEC
    thr = [f32(1.0)] * 4
    dens = [f32(1.0)] * 4
    In = [-Out[0], -Out[1], -Out[2]]
    for _ in range(q.bounces):
        if layer == COAT:
            In, thr, dens = openpbr_coat(g, q, Out, thr, dens)
            layer = SPEC if In[2] < 0 else EXTERNAL
        elif layer == SPEC:
            In, thr, dens = openpbr_specular(g, q, Out, thr, dens)
            layer = DIFF if In[2] < 0 else COAT
        elif layer == DIFF:
            In, thr = openpbr_diffuse(g, q, Out, thr)
            layer = EXTERNAL if In[2] < 0 else SPEC
        else:
            break
        if _max4(dens) < EPSILON:
            return False, None, None, None
        Out = [-In[0], -In[1], -In[2]]
    return True, In, thr, dens


def sample_surface_integrand(W_, g, m, lam, uv, exterior, TX, TY, N, out):
    """SampleSurfaceIntegrand (basic_scatter.glsl:68-109): (ok, In, throughput, probability)."""
    typ = int(W_.mat[32 * m])
    dirac = ((typ == 1 and W_.value(m, 9, uv) < f32(1e-3)) or (typ == 2 and W_.value(m, 3, uv) < f32(1e-3))
             or (typ == 3 and W_.openpbr))   # the OpenPBR sampler has no evaluate: never light-sampled
    light_p = f32(0.0) if dirac else W_.light_p
    mu = [_dot(W_.sky_mean, TX), _dot(W_.sky_mean, TY), _dot(W_.sky_mean, N)]
    STATS[("diffuse", "metal", "glass", "openpbr")[typ] + ("_dirac" if dirac else "")] += 1
    if g.r01() < light_p:
        STATS["light"] += 1
        inn = random_vmf(g, W_.kappa, mu)
        if inn[2] < 0:
            return False, None, None, None
        ok, thru, mpdf = evaluate_bsdf(W_, m, lam, uv, exterior, out, inn)
    else:
        ok, inn, thru, mpdf = sample_bsdf(W_, g, m, lam, uv, exterior, out)
    if not ok:
        return False, None, None, None
    sky_pdf = vmf_pdf(W_.kappa, mu, inn)
    one = f32(1.0)
    return True, inn, thru, [light_p * sky_pdf + (one - light_p) * mpdf[k] for k in range(4)]


def scatter(W_, sl, g, hit, ptp):
    """Scatter (basic_scatter.glsl:114-310); returns (continues, O', V')."""
    O = [f32(c) for c in sl.O]
    V = [f32(c) for c in kat.unpack_unit_vector(np.array([sl.PV], np.uint32))[0]]
    l0 = sl.lam0
    lam = [_mix(LAMBDA_MIN, LAMBDA_MAX, l0), _mix(LAMBDA_MIN, LAMBDA_MAX, _fract(l0 + f32(0.25))),
           _mix(LAMBDA_MIN, LAMBDA_MAX, _fract(l0 + f32(0.50))), _mix(LAMBDA_MIN, LAMBDA_MAX, _fract(l0 + f32(0.75)))]
    active = min(sl.active)
    prio, ior, absorb, scat, aniso = resolve_medium(W_, active, lam)
    htime = HIT_TIME_LIMIT if hit is None else hit[1]
    sl.thr = [sl.thr[k] * _fp("exp", -absorb[k] * htime) for k in range(4)]
    st = HIT_TIME_LIMIT
    if scat[0] > 0:
        st = -_fp("log", g.r01()) / scat[0]
    if htime >= st and st < HIT_TIME_LIMIT:
        STATS["medium" if abs(aniso) < f32(1e-3) else "medium_hg"] += 1
        o2 = [O[i] + V[i] * st for i in range(3)]
        X, Y = coordinate_frame(V)
        u1 = g.r01()
        u2 = g.r01()
        sd = sample_direction_hg(aniso, u1, u2)
        dens = [scat[k] * _fp("exp", -scat[k] * st) for k in range(4)]
        mx = np.fmax(EPSILON, _max4(dens))
        dens = [d / mx for d in dens]
        sl.thr = [sl.thr[k] * dens[k] for k in range(4)]
        sl.prob = [sl.prob[k] * dens[k] for k in range(4)]
        v2 = _normalize([(X[i] * sd[0] + Y[i] * sd[1]) + V[i] * sd[2] for i in range(3)])
        return bool(_max4(sl.prob) > EPSILON), o2, v2
    if htime >= st:
        sp = W_.sky_spectrum(V)
        em = [sp[3] * parametric(sp[:3], l) * W_.sky_brightness for l in lam]
        cluster = ((sl.prob[0] + sl.prob[1]) + sl.prob[2]) + sl.prob[3]
        e = [em[k] * sl.thr[k] for k in range(4)]
        obs = [observer(l) for l in lam]
        xyz = [((obs[0][i] * e[0] + obs[1][i] * e[1]) + obs[2][i] * e[2]) + obs[3][i] * e[3] for i in range(3)]
        sl.sample = [sl.sample[i] + xyz[i] / cluster for i in range(3)]
        sl.prob = [f32(0.0)] * 4
        return False, None, None
    shape, material, time, pn, ptg, uv = hit[0], hit[2], hit[1], hit[3], hit[4], hit[5]
    N = [f32(c) for c in kat.unpack_unit_vector(np.array([pn], np.uint32))[0]]
    TX = [f32(c) for c in kat.unpack_unit_vector(np.array([ptg], np.uint32))[0]]
    TY = _cross(N, TX)
    pos = [O[i] + time * V[i] for i in range(3)]
    out = [-_dot(V, TX), -_dot(V, TY), -_dot(V, N)]
    exterior = [f32(1.0)] * 4
    if out[2] > 0:
        real = prio > shape
        if real:
            exterior = ior
    else:
        real = prio == shape
        if real:
            ext = NONE
            for a in sl.active:
                if a != active:
                    ext = min(ext, a)
            exterior = resolve_medium(W_, ext, lam)[1]
    if real:
        ok, inn, thru, prob = sample_surface_integrand(W_, g, material, lam, uv, exterior, TX, TY, N, out)
        if not ok:
            return False, None, None
        scale = f32(1.0) / np.fmax(EPSILON, _max4(prob))
        sl.thr = [sl.thr[k] * (thru[k] * scale) for k in range(4)]
        sl.prob = [sl.prob[k] * (prob[k] * scale) for k in range(4)]
    else:
        inn = [-out[0], -out[1], -out[2]]
    if inn[2] * out[2] < 0:
        if out[2] > 0:
            for i in range(4):
                if sl.active[i] == NONE:
                    sl.active[i] = shape
                    break
        else:
            for i in range(4):
                if sl.active[i] == shape:
                    sl.active[i] = NONE
                    break
    if g.r01() < ptp:
        return False, None, None
    sl.prob = [p * (f32(1.0) - ptp) for p in sl.prob]
    v2 = [(inn[0] * TX[i] + inn[1] * TY[i]) + inn[2] * N[i] for i in range(3)]
    o2 = [pos[i] + f32(1e-3) * v2[i] for i in range(3)]
    return bool(_max4(sl.prob) > EPSILON), o2, v2


def store_active(sl):
    """StorePathVertexData / LoadPath's active-shape words (basic.glsl.inc:
    184-193, 214-215): (A[1] << 16) | A[0] in 32 bits, so an empty slot 0
    (SHAPE_INDEX_NONE = 0xFFFFFFFF) ORs slot 1 away -- kept as written."""
    a = sl.active
    words = [(((a[1] << 16) | a[0]) & 0xFFFFFFFF), (((a[3] << 16) | a[2]) & 0xFFFFFFFF)]
    out = []
    for w in words:
        for v in (w & 0xFFFF, w >> 16):
            out.append(NONE if v == 0xFFFF else v)
    sl.active = out


def render(scene, W, H, schedule, flags=3, ptp=0.0, camera=0, openpbr=False):
    """Reset + Run(r) for r in schedule (FrameIndex from 0): (slots, accum)."""
    W_ = World(scene)
    W_.openpbr = openpbr
    cam = W_.arrays["cameras"][camera]
    ptp = f32(ptp)
    accum = np.zeros((H, W, 4), np.float32)
    slots = [[Slot() for _ in range(W)] for _ in range(H)]
    frame = 0
    for y in range(H):
        for x in range(W):
            g = Rng(x, y, frame)
            slots[y][x].start(*new_path(W_, cam, g, x, y, W, H, flags))
    for rounds in schedule:
        frame += 1
        for _ in range(rounds):
            for y in range(H):
                for x in range(W):
                    sl = slots[y][x]
                    V = kat.unpack_unit_vector(np.array([sl.PV], np.uint32))[0]
                    h = tr.trace(W_.S, sl.O, V, HIT_TIME_LIMIT)
                    hit = None
                    if h.shape != tr.SHAPE_INDEX_NONE:
                        normal, tangent, uv = tr.hit_attributes(W_.S, h)
                        pn = int(kat.pack_unit_vector(np.array([normal], np.float32))[0])
                        ptg = int(kat.pack_unit_vector(np.array([tangent], np.float32))[0])
                        hit = (h.shape, h.time, W_.S.shape_material[h.shape], pn, ptg, uv)
                    g = Rng(x, y, frame)
                    cont, o2, v2 = scatter(W_, sl, g, hit, ptp)
                    if cont:
                        sl.O = o2
                        sl.PV = int(kat.pack_unit_vector(np.array([v2], np.float32))[0])
                        store_active(sl)
                    else:
                        val = [sl.sample[0], sl.sample[1], sl.sample[2], f32(1.0)]
                        if flags & 1:
                            val = [accum[y, x, k] + val[k] for k in range(4)]
                        accum[y, x] = val
                        sl.start(*new_path(W_, cam, g, x, y, W, H, flags))
    return slots, accum
