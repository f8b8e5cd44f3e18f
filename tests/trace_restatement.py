"""A second restatement of the reference's Trace(), written independently of
oracle/pt_oracle.cpp from the GLSL text, to cross-check the oracle's
traversal (test infrastructure only; tests/test_trace_restatement.py).

Follows, statement by statement:
  Trace                 src/scene/scene.glsl.inc:522-533 (closest hit only)
  Intersect (TLAS)      src/scene/scene.glsl.inc:468-520
  IntersectShape        src/scene/scene.glsl.inc:401-465
  IntersectMeshNode     src/scene/scene.glsl.inc:336-399
  IntersectMeshFace     src/scene/scene.glsl.inc:304-334
  IntersectBoundingBox  src/core/common.glsl.inc:153-185
  InverseTransformRay   src/core/common.glsl.inc:84-91 (InverseTransformPosition/Vector :70-80)
  hit attributes        src/scene/scene.glsl.inc:535-608 (SafeNormalize :93-100,
                        TransformNormal / TransformDirection, ComputeTangentVector :113-117;
                        octahedral packing from tests/kat.py)
and the record packing of StoreTraceHit (src/integrator/basic.glsl.inc:142-156):
ShapeAndMaterialIndex = Shape << 16 | Material, 0xFFFFFFFF on a miss.

Arithmetic is float32 (numpy float32 scalars: every + - * / is rounded to
float32; nothing is fused), under the numerics convention DESIGN.md §2
writes down for what GLSL leaves open: vector reductions (dot, mat4 * vec4)
left to right, cross products as the three differences of rounded products,
min/max ignoring a NaN operand (fminf / fmaxf).  Scalar Python loops: meant
for a few hundred rays per scene.
"""
from __future__ import annotations

import numpy as np

import kat
import oracle_lib

f32 = np.float32
INFINITY = f32(1e30)             # common.glsl.inc:4
EPSILON = f32(1e-9)              # common.glsl.inc:5
SHAPE_INDEX_NONE = 0xFFFFFFFF    # scene.glsl.inc:7
MESH_FACE_OF_INSTANCE = 0xFFFFFFFE
PLANE, SPHERE, CUBE, MESH = 1, 2, 3, 0


def _v(a):
    return [f32(a[0]), f32(a[1]), f32(a[2])]


def _dot(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def _cross(a, b):
    return [a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]]


def _sub(a, b):
    return [a[0] - b[0], a[1] - b[1], a[2] - b[2]]


def _mat_vec(m, v, w):
    """(M * vec4(v, w)).xyz for a column-major float[16] M."""
    w = f32(w)
    return [((m[r] * v[0] + m[4 + r] * v[1]) + m[8 + r] * v[2]) + m[12 + r] * w for r in range(3)]


def _fmin(a, b):
    return np.fmin(a, b)


def _fmax(a, b):
    return np.fmax(a, b)


def intersect_bounding_box(O, V, reach, mn, mx):
    """common.glsl.inc:153-185: the entry time, or INFINITY on a miss."""
    with np.errstate(divide="ignore", invalid="ignore"):
        tmin = [(mn[i] - O[i]) / V[i] for i in range(3)]
        tmax = [(mx[i] - O[i]) / V[i] for i in range(3)]
    early = [_fmin(tmin[i], tmax[i]) for i in range(3)]
    late = [_fmax(tmin[i], tmax[i]) for i in range(3)]
    entry = _fmax(_fmax(early[0], early[1]), early[2])
    exit_ = _fmin(_fmin(late[0], late[1]), late[2])
    if exit_ < entry:
        return INFINITY
    if exit_ <= 0:
        return INFINITY
    if entry >= reach:
        return INFINITY
    return entry


class Hit:
    __slots__ = ("time", "shape", "prim", "kind", "coords", "scene_complexity", "mesh_complexity")

    def __init__(self, duration):
        self.scene_complexity = 0   # shape nodes visited (scene.glsl.inc:117, 480)
        self.mesh_complexity = 0    # mesh nodes visited (:118, 345)
        self.time = f32(duration)
        self.shape = SHAPE_INDEX_NONE
        self.prim = 0
        self.kind = -1
        self.coords = None


class Scene:
    """The packed buffers as float32 / uint32 tables (from Scene.arrays())."""

    def __init__(self, arrays):
        sh = arrays["shapes"]
        self.shape_type = [int(t) for t in sh["Type"]]
        self.shape_material = [int(m) for m in sh["MaterialIndex"]]
        self.shape_root = [int(r) for r in sh["MeshRootNodeIndex"]]
        self.shape_from = [np.asarray(t, np.float32).reshape(16) for t in sh["Transform"]["From"]]
        self.shape_to = [np.asarray(t, np.float32).reshape(16) for t in sh["Transform"]["To"]]
        mv = arrays["mesh_vertices"]
        self.vertex_normal = mv["PackedNormal"].astype(np.uint32)
        self.vertex_uv = mv["PackedUV"].astype(np.uint32)
        sn = arrays["shape_nodes"]
        self.sn_min = [_v(x) for x in sn["Minimum"]]
        self.sn_max = [_v(x) for x in sn["Maximum"]]
        self.sn_children = [int(c) for c in sn["ChildNodeIndices"]]
        self.sn_shape = [int(s) for s in sn["ShapeIndex"]]
        mn = arrays["mesh_nodes"]
        self.mn_min = [_v(x) for x in mn["Minimum"]]
        self.mn_max = [_v(x) for x in mn["Maximum"]]
        self.mn_begin = [int(x) for x in mn["FaceBeginOrNodeIndex"]]
        self.mn_end = [int(x) for x in mn["FaceEndIndex"]]
        mf = arrays["mesh_faces"]
        self.f0 = [_v(x) for x in mf["Position0"]]
        self.f1 = [_v(x) for x in mf["Position1"]]
        self.f2 = [_v(x) for x in mf["Position2"]]
        self.fv = [(int(a), int(b), int(c)) for a, b, c in zip(mf["VertexIndex0"], mf["VertexIndex1"], mf["VertexIndex2"])]
        self.shape_count = int(arrays["globals"]["ShapeCount"][0])


def intersect_mesh_face(S, O, V, face, hit):
    """scene.glsl.inc:304-334."""
    p0 = S.f0[face]
    e1 = _sub(S.f1[face], p0)
    e2 = _sub(S.f2[face], p0)
    rce2 = _cross(V, e2)
    det = _dot(e1, rce2)
    if abs(det) < EPSILON:
        return
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = f32(1.0) / det
    s = _sub(O, p0)
    u = inv * _dot(s, rce2)
    if u < 0 or u > 1:
        return
    sce1 = _cross(s, e1)
    v = inv * _dot(V, sce1)
    if v < 0 or u + v > 1:
        return
    t = inv * _dot(e2, sce1)
    if t < 0 or t > hit.time:
        return
    hit.time = t
    hit.shape = MESH_FACE_OF_INSTANCE
    hit.prim = face
    hit.kind = MESH
    hit.coords = [(f32(1.0) - u) - v, u, v]


def intersect_mesh_node(S, O, V, root, hit):
    """scene.glsl.inc:336-399."""
    stack = []
    node = root
    while True:
        hit.mesh_complexity += 1
        if S.mn_end[node] > 0:
            for face in range(S.mn_begin[node], S.mn_end[node]):
                intersect_mesh_face(S, O, V, face, hit)
        else:
            a = S.mn_begin[node]
            b = a + 1
            ta = intersect_bounding_box(O, V, hit.time, S.mn_min[a], S.mn_max[a])
            tb = intersect_bounding_box(O, V, hit.time, S.mn_min[b], S.mn_max[b])
            if ta > tb:
                if ta < INFINITY:
                    stack.append(a)
                node = b
                continue
            if tb < INFINITY:
                stack.append(b)
                node = a
                continue
            if ta < INFINITY:
                node = a
                continue
        if not stack:
            break
        node = stack.pop()


def intersect_shape(S, O, V, idx, hit):
    """scene.glsl.inc:401-465 (InverseTransformRay first)."""
    m = S.shape_from[idx]
    O = _mat_vec(m, O, 1.0)
    V = _mat_vec(m, V, 0.0)
    kind = S.shape_type[idx]
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        if kind == MESH:
            intersect_mesh_node(S, O, V, S.shape_root[idx], hit)
            if hit.shape == MESH_FACE_OF_INSTANCE:
                hit.shape = idx
        elif kind == PLANE:
            t = -O[2] / V[2]
            if t < 0 or t > hit.time:
                return
            hit.time, hit.shape, hit.prim = t, idx, 0
            hit.kind, hit.coords = PLANE, [O[i] + V[i] * t for i in range(3)]
        elif kind == SPHERE:
            vv = _dot(V, V)
            p = _dot(O, V)
            q = _dot(O, O) - f32(1.0)
            d2 = p * p - q * vv
            if d2 < 0:
                return
            d = np.sqrt(d2)
            if d < p:
                return
            s0 = -p - d
            s1 = -p + d
            s = s1 if s0 < 0 else s0
            if s < 0 or s > vv * hit.time:
                return
            hit.time, hit.shape, hit.prim = s / vv, idx, 0
            hit.kind, hit.coords = SPHERE, [O[i] + V[i] * hit.time for i in range(3)]
        elif kind == CUBE:
            lo = [(f32(-1.0) - O[i]) / V[i] for i in range(3)]
            hi = [(f32(1.0) - O[i]) / V[i] for i in range(3)]
            early = [_fmin(lo[i], hi[i]) for i in range(3)]
            late = [_fmax(lo[i], hi[i]) for i in range(3)]
            t0 = _fmax(_fmax(early[0], early[1]), early[2])
            t1 = _fmin(_fmin(late[0], late[1]), late[2])
            if t1 < t0 or t1 <= 0:
                return
            t = t1 if t0 < 0 else t0
            if t >= hit.time:
                return
            hit.time, hit.shape, hit.prim = t, idx, 0
            hit.kind, hit.coords = CUBE, [O[i] + V[i] * t for i in range(3)]


def trace(S, O, V, duration):
    """Trace() up to the closest hit (scene.glsl.inc:468-533)."""
    hit = Hit(duration)
    if S.shape_count == 0:
        return hit
    O, V = _v(O), _v(V)
    stack = []
    node = 0
    while True:
        hit.scene_complexity += 1
        children = S.sn_children[node]
        if children == 0:
            intersect_shape(S, O, V, S.sn_shape[node], hit)
        else:
            a, b = children & 0xFFFF, children >> 16
            ta = intersect_bounding_box(O, V, hit.time, S.sn_min[a], S.sn_max[a])
            tb = intersect_bounding_box(O, V, hit.time, S.sn_min[b], S.sn_max[b])
            if ta > tb:
                if ta < INFINITY:
                    stack.append(a)
                node = b
                continue
            if tb < INFINITY:
                stack.append(b)
                node = a
                continue
            if ta < INFINITY:
                node = a
                continue
        if not stack:
            break
        node = stack.pop()
    return hit


# --- hit attributes (scene.glsl.inc:535-608) -------------------------------------

def _normalize(v):
    """GLSL normalize under the convention: v * (1 / sqrt(dot(v, v)))."""
    r = f32(1.0) / np.sqrt(_dot(v, v))
    return [v[0] * r, v[1] * r, v[2] * r]


def _safe_normalize(v):
    """common.glsl.inc:93-100: V / sqrt(LenSq), or +Z for a tiny vector."""
    lsq = _dot(v, v)
    if lsq < f32(1e-12):
        return [f32(0.0), f32(0.0), f32(1.0)]
    d = np.sqrt(lsq)
    return [v[0] / d, v[1] / d, v[2] / d]


def _transform_normal(n, frm):
    """common.glsl.inc TransformNormal: normalize((vec4(N, 0) * From).xyz)."""
    z = f32(0.0)
    return _normalize([((n[0] * frm[4 * c] + n[1] * frm[4 * c + 1]) + n[2] * frm[4 * c + 2]) + z * frm[4 * c + 3]
                       for c in range(3)])


def _transform_direction(d, to):
    """normalize(TransformVector(D)) = normalize((To * vec4(D, 0)).xyz)."""
    return _normalize(_mat_vec(to, d, 0.0))


def _tangent(n):
    """ComputeTangentVector (common.glsl.inc:113-117)."""
    v = [f32(1.0), f32(0.0), f32(0.0)] if abs(n[0]) < f32(0.9) else [f32(0.0), f32(1.0), f32(0.0)]
    return _normalize(_cross(v, n))


def _half2(u):
    lo = np.array([u & 0xFFFF], np.uint16).view(np.float16)[0]
    hi = np.array([u >> 16], np.uint16).view(np.float16)[0]
    return f32(lo), f32(hi)


def _sign(x):
    return f32(1.0) if x > 0 else (f32(-1.0) if x < 0 else f32(0.0))


def hit_attributes(S, h):
    """(Normal, TangentX, UV) of a hit (scene.glsl.inc:540-600); a sphere's
    atan2 is the numerics convention's own (the oracle's exported pt_atan2)."""
    to, frm = S.shape_to[h.shape], S.shape_from[h.shape]
    c = h.coords
    if h.kind == MESH:
        i0, i1, i2 = S.fv[h.prim]
        n0, n1, n2 = kat.unpack_unit_vector(np.array([S.vertex_normal[i0], S.vertex_normal[i1],
                                                      S.vertex_normal[i2]], np.uint32))
        n = [(n0[k] * c[0] + n1[k] * c[1]) + n2[k] * c[2] for k in range(3)]
        normal = _transform_normal(_safe_normalize(n), frm)
        tangent = _tangent(normal)
        uv0, uv1, uv2 = _half2(int(S.vertex_uv[i0])), _half2(int(S.vertex_uv[i1])), _half2(int(S.vertex_uv[i2]))
        uv = [(uv0[k] * c[0] + uv1[k] * c[1]) + uv2[k] * c[2] for k in range(2)]
    elif h.kind == PLANE:
        normal = _transform_normal([f32(0.0), f32(0.0), f32(1.0)], frm)
        tangent = _transform_direction([f32(1.0), f32(0.0), f32(0.0)], to)
        uv = [c[0] - np.floor(c[0]), c[1] - np.floor(c[1])]
    elif h.kind == SPHERE:
        normal = _transform_normal(c, frm)
        tangent = _transform_direction(_cross(c, [-c[1], c[0], f32(0.0)]), to)
        at = f32(oracle_lib.lib().oracle_fp_atan2(float(c[1]), float(c[0])))
        uv = [(at + f32(3.141592653)) / f32(6.283185306), (c[2] + f32(1.0)) / f32(2.0)]
    else:
        q = [abs(c[0]), abs(c[1]), abs(c[2])]
        half, one = f32(0.5), f32(1.0)
        if q[0] >= q[1] and q[0] >= q[2]:
            sg = _sign(c[0])
            nrm, tx, uv = [sg, f32(0), f32(0)], [f32(0), sg, f32(0)], [half * (one + c[1]), half * (one + c[2])]
        elif q[1] >= q[0] and q[1] >= q[2]:
            sg = _sign(c[1])
            nrm, tx, uv = [f32(0), sg, f32(0)], [f32(0), f32(0), sg], [half * (one + c[0]), half * (one + c[2])]
        else:
            sg = _sign(c[2])
            nrm, tx, uv = [f32(0), f32(0), sg], [sg, f32(0), f32(0)], [half * (one + c[0]), half * (one + c[1])]
        normal = _transform_normal(nrm, frm)
        tangent = _transform_direction(tx, to)
    return normal, tangent, uv


def trace_records(arrays, origins, velocities, durations):
    """Per ray, as StoreTraceHit (basic.glsl.inc:142-156) writes them: time,
    ShapeAndMaterialIndex, packed normal, packed tangent, U, V (NaN on a miss)."""
    S = Scene(arrays)
    n = len(origins)
    times = np.zeros(n, np.float32)
    sm = np.zeros(n, np.uint32)
    pn = np.zeros(n, np.uint32)
    ptg = np.zeros(n, np.uint32)
    uv = np.full((n, 2), np.nan, np.float32)
    for i in range(n):
        h = trace(S, origins[i], velocities[i], durations[i])
        if h.shape == SHAPE_INDEX_NONE:
            sm[i] = 0xFFFFFFFF
            continue
        sm[i] = (h.shape << 16) | S.shape_material[h.shape]
        times[i] = h.time
        normal, tangent, u = hit_attributes(S, h)
        pn[i] = kat.pack_unit_vector(np.array([normal], np.float32))[0]
        ptg[i] = kat.pack_unit_vector(np.array([tangent], np.float32))[0]
        uv[i] = u
    return times, sm, pn, ptg, uv
