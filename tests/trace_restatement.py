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
    __slots__ = ("time", "shape", "prim")

    def __init__(self, duration):
        self.time = f32(duration)
        self.shape = SHAPE_INDEX_NONE
        self.prim = 0


class Scene:
    """The packed buffers as float32 / uint32 tables (from Scene.arrays())."""

    def __init__(self, arrays):
        sh = arrays["shapes"]
        self.shape_type = [int(t) for t in sh["Type"]]
        self.shape_material = [int(m) for m in sh["MaterialIndex"]]
        self.shape_root = [int(r) for r in sh["MeshRootNodeIndex"]]
        self.shape_from = [np.asarray(t, np.float32).reshape(16) for t in sh["Transform"]["From"]]
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


def intersect_mesh_node(S, O, V, root, hit):
    """scene.glsl.inc:336-399."""
    stack = []
    node = root
    while True:
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


def trace(S, O, V, duration):
    """Trace() up to the closest hit (scene.glsl.inc:468-533)."""
    hit = Hit(duration)
    if S.shape_count == 0:
        return hit
    O, V = _v(O), _v(V)
    stack = []
    node = 0
    while True:
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


def trace_records(arrays, origins, velocities, durations):
    """(time, ShapeAndMaterialIndex) per ray, as StoreTraceHit writes them."""
    S = Scene(arrays)
    n = len(origins)
    times = np.zeros(n, np.float32)
    sm = np.zeros(n, np.uint32)
    for i in range(n):
        h = trace(S, origins[i], velocities[i], durations[i])
        if h.shape == SHAPE_INDEX_NONE:
            sm[i] = 0xFFFFFFFF
        else:
            sm[i] = (h.shape << 16) | S.shape_material[h.shape]
            times[i] = h.time
    return times, sm
