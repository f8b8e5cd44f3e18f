"""Second, independent restatement of the reference's host-side BVH builders
(test infrastructure): BuildMeshNode, the mesh part of PackSceneData and the
TLAS pairing, written from the reference's source text in numpy float32, to
cross-check the product's C++ restatement (csrc/scene/scene.cpp) node for
node.  The reference cannot be built here, so the builder is
otherwise pinned only by structural invariants; two restatements written
separately from the same text catch transcription slips in either.

Float semantics: every arithmetic step is one IEEE binary32 operation in the
reference's order (numpy float32, no FMA); glm::min / glm::max / std::min /
std::max on floats keep the first operand on ties ((b < a) ? b : a and
(a < b) ? b : a), so a running minimum keeps the first occurrence.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
INF = F32(np.inf)
BINS = 32


def first_min(vals: np.ndarray):
    """Running glm::min from +INF over vals in order (first occurrence of the minimum)."""
    return vals[int(np.argmin(vals))] if len(vals) else INF


def first_max(vals: np.ndarray):
    return vals[int(np.argmax(vals))] if len(vals) else -INF


def binned_first(vals: np.ndarray, labels: np.ndarray, nbins: int, largest: bool) -> np.ndarray:
    """Per label, the running glm::min (or max) of vals in stream order: the
    extreme value, its first occurrence on ties (which keeps the sign of a
    zero); +INF (-INF) for an empty label."""
    out = np.full(nbins, -INF if largest else INF, dtype=F32)
    if len(vals) == 0:
        return out
    key = -vals if largest else vals
    o = np.lexsort((np.arange(len(vals)), key, labels))
    lab = labels[o]
    starts = np.flatnonzero(np.r_[True, lab[1:] != lab[:-1]])
    out[lab[starts]] = vals[o][starts]
    return out


def gmin(a, b):
    return b if b < a else a


def gmax(a, b):
    return b if a < b else a


def half_area(mn, mx):
    """HalfArea (scene.cpp:53-63): E = Max - Min; E.x*E.y + E.y*E.z + E.z*E.x."""
    with np.errstate(all="ignore"):
        e = [F32(mx[i] - mn[i]) for i in range(3)]
        return F32(F32(F32(e[0] * e[1]) + F32(e[1] * e[2])) + F32(e[2] * e[0]))


def centroids(P: np.ndarray, faces: np.ndarray, axis: int) -> np.ndarray:
    """GetMeshFaceCentroid (scene.cpp:423-432): 0 + p0 + p1 + p2, then / 3."""
    c = np.zeros(len(faces), dtype=F32)
    for j in range(3):
        c = (c + P[faces[:, j], axis]).astype(F32)
    return (c / F32(3.0)).astype(F32)


def vertex_stream(P: np.ndarray, faces: np.ndarray, axis: int) -> np.ndarray:
    """Coordinates in Grow order: face by face, vertex 0, 1, 2."""
    return P[faces.reshape(-1), axis]


def build_mesh(P: np.ndarray, faces_in: np.ndarray):
    """BuildMeshNode (scene.cpp:435-599) from the root (scene.cpp:851-863).
    Returns (nodes, faces): nodes as [begin, end, child, min(3), max(3)]."""
    P = np.ascontiguousarray(P, dtype=F32)
    faces = np.array(faces_in, dtype=np.int64).reshape(-1, 3).copy()
    nodes = [[0, len(faces), 0, None, None]]

    def build(ni):
        begin, end = nodes[ni][0], nodes[ni][1]
        fc = end - begin
        sub = faces[begin:end]
        nodes[ni][3] = [first_min(vertex_stream(P, sub, a)) for a in range(3)]
        nodes[ni][4] = [first_max(vertex_stream(P, sub, a)) for a in range(3)]
        split_axis, split_pos, split_cost = 0, F32(0), INF
        for axis in range(3):
            c = centroids(P, sub, axis)
            cmin, cmax = first_min(c), first_max(c)
            if cmin == cmax:
                continue
            with np.errstate(all="ignore"):
                per_unit = F32(F32(BINS) / F32(cmax - cmin))
                idx = np.minimum((per_unit * (c - cmin).astype(F32)).astype(F32).astype(np.uint32), BINS - 1)
            bcount = np.bincount(idx, minlength=BINS)
            lab = np.repeat(idx.astype(np.int64), 3)            # each face's three Grow calls
            mins = [binned_first(vertex_stream(P, sub, a), lab, BINS, False) for a in range(3)]
            maxs = [binned_first(vertex_stream(P, sub, a), lab, BINS, True) for a in range(3)]
            bmin = [[mins[a][b] for a in range(3)] for b in range(BINS)]
            bmax = [[maxs[a][b] for a in range(3)] for b in range(BINS)]
            left_area = [F32(0)] * (BINS - 1)
            left_count = [0] * (BINS - 1)
            right_area = [F32(0)] * (BINS - 1)
            right_count = [0] * (BINS - 1)
            lmn, lmx, rmn, rmx = [INF] * 3, [-INF] * 3, [INF] * 3, [-INF] * 3
            ls = rs = 0
            for i in range(BINS - 1):                              # scene.cpp:511-532
                j = BINS - 2 - i
                if bcount[i] > 0:
                    ls += int(bcount[i])
                    lmn = [gmin(lmn[a], bmin[i][a]) for a in range(3)]
                    lmx = [gmax(lmx[a], bmax[i][a]) for a in range(3)]
                left_count[i] = ls
                left_area[i] = half_area(lmn, lmx)
                if bcount[j + 1] > 0:
                    rs += int(bcount[j + 1])
                    rmn = [gmin(rmn[a], bmin[j + 1][a]) for a in range(3)]
                    rmx = [gmax(rmx[a], bmax[j + 1][a]) for a in range(3)]
                right_count[j] = rs
                right_area[j] = half_area(rmn, rmx)
            interval = F32(F32(cmax - cmin) / F32(BINS))         # scene.cpp:535-549
            pos = F32(cmin + interval)
            for i in range(BINS - 1):
                with np.errstate(all="ignore"):
                    cost = F32(F32(F32(left_count[i]) * left_area[i]) + F32(F32(right_count[i]) * right_area[i]))
                if cost < split_cost:
                    split_cost, split_axis, split_pos = cost, axis, pos
                pos = F32(pos + interval)
        no_split = F32(F32(fc) * half_area(nodes[ni][3], nodes[ni][4]))
        if split_cost >= no_split:                                 # scene.cpp:553-554
            return
        si, swap = begin, end - 1                                  # scene.cpp:557-573
        while si < swap:
            f = faces[si]
            cen = F32(F32(F32(F32(0) + P[f[0], split_axis]) + P[f[1], split_axis]) + P[f[2], split_axis]) / F32(3)
            if F32(cen) < split_pos:
                si += 1
            else:
                faces[[si, swap]] = faces[[swap, si]]
                swap -= 1
        if si == begin or si == end:
            return
        left = len(nodes)
        nodes[ni][2] = left
        nodes.append([begin, si, 0, None, None])
        nodes.append([si, end, 0, None, None])
        build(left)
        build(left + 1)

    build(0)
    return nodes, faces


def pack_mesh_nodes(nodes, node_base=0, face_base=0):
    """The packed mesh nodes (scene.cpp:1317-1337): (min, faceBeginOrNode, max, faceEnd)."""
    out = []
    for b, e, child, mn, mx in nodes:
        if child > 0:
            out.append((mn, node_base + child, mx, 0))
        else:
            out.append((mn, face_base + b, mx, face_base + e))
    return out


def mat_vec(To: np.ndarray, v):
    """glm mat4 * vec4 (column-major To[c*4+r]): (m0*x + m1*y) + (m2*z + m3*w)."""
    m = To.reshape(4, 4)
    return [F32(F32(F32(m[0, r] * v[0]) + F32(m[1, r] * v[1])) + F32(F32(m[2, r] * v[2]) + F32(m[3, r] * v[3])))
            for r in range(4)]


def shape_bounds(shape, mesh_nodes):
    """ShapeBounds (scene.cpp:1031-1093)."""
    t = int(shape["Type"])
    if t == 0:                                   # SHAPE_TYPE_MESH_INSTANCE
        r = mesh_nodes[int(shape["MeshRootNodeIndex"])]
        mn, mx = r["Minimum"], r["Maximum"]
        corners = [(mn[0], mn[1], mn[2]), (mn[0], mn[1], mx[2]), (mn[0], mx[1], mn[2]), (mn[0], mx[1], mx[2]),
                   (mx[0], mn[1], mn[2]), (mx[0], mn[1], mx[2]), (mx[0], mx[1], mn[2]), (mx[0], mx[1], mx[2])]
    elif t == 1:                                 # SHAPE_TYPE_PLANE
        e = F32(1e-9)
        corners = [(-1e9, -1e9, -e), (1e9, -1e9, -e), (-1e9, 1e9, -e), (1e9, 1e9, -e),
                   (-1e9, -1e9, e), (1e9, -1e9, e), (-1e9, 1e9, e), (1e9, 1e9, e)]
    else:                                        # sphere, cube
        corners = [(-1, -1, -1), (1, -1, -1), (-1, 1, -1), (1, 1, -1), (-1, -1, 1), (1, -1, 1), (-1, 1, 1), (1, 1, 1)]
    wmin, wmax = [INF] * 3, [-INF] * 3
    To = np.asarray(shape["Transform"]["To"], dtype=F32)
    for c in corners:
        w = mat_vec(To, [F32(c[0]), F32(c[1]), F32(c[2]), F32(1)])
        wmin = [gmin(wmin[a], w[a]) for a in range(3)]
        wmax = [gmax(wmax[a], w[a]) for a in range(3)]
    return wmin, wmax


def build_tlas(shapes, mesh_nodes):
    """The shape BVH of PackSceneData (scene.cpp:1400-1493): one leaf per
    shape, then greedy mutual-best-match pairing by the reference's area
    expression (including its Size.z * Size.z term, scene.cpp:1437), the root
    moved to node 0.  Nodes: [min(3), childIndices, max(3), shapeIndex]."""
    pack = [None]                                                  # ShapeNodePack.resize(1)
    mp = []
    for i, sh in enumerate(shapes):
        mn, mx = shape_bounds(sh, mesh_nodes)
        mp.append(len(pack))
        pack.append([mn, 0, mx, i])

    def best(ia):
        mina, maxa = pack[mp[ia]][0], pack[mp[ia]][2]
        best_area, best_b = INF, 0xFFFF
        for ib in range(len(mp)):
            if ia == ib:
                continue
            minb, maxb = pack[mp[ib]][0], pack[mp[ib]][2]
            size = [F32(gmax(maxa[a], maxb[a]) - gmin(mina[a], minb[a])) for a in range(3)]
            with np.errstate(all="ignore"):
                area = F32(F32(F32(size[0] * size[1]) + F32(size[1] * size[2])) + F32(size[2] * size[2]))
            if area <= best_area:
                best_area, best_b = area, ib
        return best_b

    if shapes is not None and len(shapes):
        ia = 0
        ib = best(ia)
        while len(mp) > 1:
            ic = best(ib)
            if ia == ic:
                na, nb = pack[mp[ia]], pack[mp[ib]]
                node = [[gmin(na[0][a], nb[0][a]) for a in range(3)], (mp[ia] | (mp[ib] << 16)) & 0xFFFFFFFF,
                        [gmax(na[2][a], nb[2][a]) for a in range(3)], 0xFFFFFFFF]
                mp[ia] = len(pack)
                mp[ib] = mp[-1]
                mp.pop()
                if ia == len(mp):
                    ia = ib
                pack.append(node)
                ib = best(ia)
            else:
                ia, ib = ib, ic
        root = mp[ia]
        pack[0] = pack[root]
        pack[root] = pack[-1]
        pack.pop()
    return pack
