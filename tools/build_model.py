#!/usr/bin/env python3
"""Model compiler: UR5 + Robotiq-85 URDF and collision meshes -> constant C header.

Reads the reference's robot description (run in the build container only; the
generated header is committed so nothing here is needed on the GPU box):

  /root/reference/urgym/urdf/ur5_robotiq_85.urdf       (kinematic tree, masses, limits)
  /root/reference/urgym/meshes/ur5/collision/*.stl      (arm collision meshes)
  /root/reference/urgym/meshes/robotiq_85/collision/*   (gripper collision meshes)

and writes urgym_amd/csrc/model_data.h, included by both the CPU restatement
(oracle/) and the HIP kernels as *input data*.

Rules restated from PyBullet's URDF import ([ext]):
  * link order  = pre-order DFS from the root link `world`, children in joint
    declaration order  (gives ee_link = 7, fingers 9..18, as robot.py:180 and
    env_cubes_grasp_v0.py:207-208 assume);
  * a link without <inertial> gets mass 1 and an identity inertial frame,
    except the link named `world` (mass 0);
  * link inertia is NOT read from the URDF <inertia>: it is recomputed as the
    inertia of the box spanned by the AABB of the link's collision compound
    expressed in the inertial frame (btCompoundShape::calculateLocalInertia),
    collision margin 0.001 included in each child's AABB;
  * meshes become convex hulls of all their vertices; margin 0.001;
  * <mimic> is ignored (robot.py:190-211 builds gear constraints instead).

MI355X-side choice: links joined by fixed joints are merged into the moving
body that carries them (12 bodies, one per controllable joint). Their masses
and inertias are combined exactly (parallel-axis theorem); per-link data kept
for link damping, link queries (getLinkState / getAABB) and contact shapes.
"""
import math
import os
import struct
import sys
import xml.etree.ElementTree as ET

import numpy as np
from scipy.spatial import ConvexHull

REF = os.environ.get("URGYM_REFERENCE", "/root/reference")
# the robot: UR5Robotiq85 (robot.py:179-186, every registered env) or UR5Robotiq140 (robot.py:221-229) via
# URGYM_MODEL_URDF=urgym/urdf/ur5_robotiq_140.urdf (same tree shape and DFS order, its own meshes and limits)
URDF_REL = os.environ.get("URGYM_MODEL_URDF", "urgym/urdf/ur5_robotiq_85.urdf")
URDF = os.path.join(REF, URDF_REL)
OUT = os.environ.get("URGYM_MODEL_OUT",
                     os.path.join(os.path.dirname(__file__), "..", "urgym_amd", "csrc", "model_data.h"))
# collision-fidelity builds (tools/collision_fidelity.py; never the product): full hulls (URGYM_HULL_MAXV),
# a finer club-disc prism (URGYM_CYL_SEG) and the vertex loop of every hull face (URGYM_HULL_POLYS=1)
CYL_SEG = int(os.environ.get("URGYM_CYL_SEG", "16"))
HULL_POLYS = os.environ.get("URGYM_HULL_POLYS", "0") == "1"
MARGIN = 0.001  # gUrdfDefaultCollisionMargin [ext]


def rpy_to_mat(r, p, y):
    # URDF rpy: R = Rz(y) Ry(p) Rx(r)
    cr, sr, cp, sp, cy, sy = math.cos(r), math.sin(r), math.cos(p), math.sin(p), math.cos(y), math.sin(y)
    return np.array([
        [cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr],
        [sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr],
        [-sp, cp * sr, cp * cr]])


def origin_of(el):
    T = np.eye(4)
    if el is None:
        return T
    o = el.find("origin")
    if o is None:
        return T
    xyz = [float(v) for v in o.get("xyz", "0 0 0").split()]
    rpy = [float(v) for v in o.get("rpy", "0 0 0").split()]
    T[:3, :3] = rpy_to_mat(*rpy)
    T[:3, 3] = xyz
    return T


def read_stl(path):
    b = open(path, "rb").read()
    n = struct.unpack("<I", b[80:84])[0]
    v = []
    for i in range(n):
        off = 84 + 50 * i + 12
        tri = struct.unpack("<9f", b[off:off + 36])
        v.extend([tri[0:3], tri[3:6], tri[6:9]])
    return np.array(v, dtype=np.float64)


def read_dae(path):
    root = ET.parse(path).getroot()
    pts = []
    for fa in root.iter():
        if fa.tag.endswith("float_array") and "positions" in fa.get("id", ""):
            vals = np.array([float(x) for x in fa.text.split()])
            pts.append(vals.reshape(-1, 3))
    return np.concatenate(pts)


MAXV = int(os.environ.get("URGYM_HULL_MAXV", "48"))


def decimate(verts, maxv):
    """Farthest-point subset of the hull vertices (collision LOD)."""
    if len(verts) <= maxv:
        return verts
    c = verts.mean(0)
    sel = [int(np.argmax(np.linalg.norm(verts - c, axis=1)))]
    d = np.linalg.norm(verts - verts[sel[0]], axis=1)
    while len(sel) < maxv:
        k = int(np.argmax(d))
        sel.append(k)
        d = np.minimum(d, np.linalg.norm(verts - verts[k], axis=1))
    return verts[sorted(sel)]


def hull_planes(h):
    """the hull's facets with coplanar ones merged (unique planes), as n.x <= off (outward normal n, off = -d)"""
    planes = []
    for eq in h.equations:
        n, d = eq[:3], eq[3]
        dup = False
        for p in planes:
            if np.dot(p[:3], n) > 1 - 1e-6 and abs(p[3] - d) < 1e-6:
                dup = True
                break
        if not dup:
            planes.append(eq)
    return np.array([[p[0], p[1], p[2], -p[3]] for p in planes])


def spatial_chunks(verts, size=64):
    """vertex order for the full hulls: spatially coherent groups of <= size (recursive split of the group count
    along the longest extent), each group contiguous, so a 64-lane chunk has a tight bounding sphere (the kernel's
    exact chunk cull, team_hull_box_full).  Deterministic; returns the permutation."""
    def split(idx, k):
        if k == 1:
            return [idx]
        p = verts[idx]
        ax = int(np.argmax(p.max(0) - p.min(0)))
        o = idx[np.argsort(p[:, ax], kind="stable")]
        kl = k // 2
        nl = int(round(len(idx) * kl / k))
        return split(o[:nl], kl) + split(o[nl:], k - kl)
    n = len(verts)
    groups = split(np.arange(n), max(1, -(-n // size)))
    assert all(len(g) <= size for g in groups), [len(g) for g in groups]
    return np.concatenate([np.sort(g) for g in groups]), [len(g) for g in groups]


def hull_of(points):
    """(LOD vertices, LOD planes, full hull vertices, full hull planes): the collision LOD of the product's default
    geometry, and the convex hull of all mesh vertices that PyBullet builds (optimizeConvexHull) for the full mode"""
    h = ConvexHull(points)
    full = points[h.vertices]
    verts = decimate(full, MAXV)
    h = ConvexHull(verts)
    verts = verts[h.vertices]
    # report how far the dropped vertices lie outside the LOD hull
    out = np.max(full @ h.equations[:, :3].T + h.equations[:, 3], axis=1).max()
    print("  hull %d -> %d verts, max outside %.4f m" % (len(full), len(verts), out))
    planes = hull_planes(h)
    hf = ConvexHull(full)
    fverts = full[hf.vertices]
    fplanes = planes if len(fverts) == len(verts) and np.array_equal(fverts, verts) else hull_planes(hf)
    perm, sizes = spatial_chunks(fverts)
    return verts, planes, fverts[perm], fplanes, sizes


def face_loops(verts, planes):
    """vertex indices of each face, counter-clockwise about the outward normal (the face polygon)"""
    loops = []
    for p in planes:
        n, off = p[:3], p[3]
        on = np.where(np.abs(verts @ n - off) < 1e-6 * max(1.0, abs(off)) + 1e-9)[0]
        c = verts[on].mean(0)
        u = verts[on[0]] - c
        u /= np.linalg.norm(u)
        v = np.cross(n, u)
        ang = np.arctan2((verts[on] - c) @ v, (verts[on] - c) @ u)
        loops.append([int(i) for i in on[np.argsort(ang)]])
    return loops


def main():
    robot = ET.parse(URDF).getroot()
    links = {l.get("name"): l for l in robot.findall("link")}
    joints = robot.findall("joint")
    child_joints = {}
    parent_of = {}
    for j in joints:
        p = j.find("parent").get("link")
        c = j.find("child").get("link")
        child_joints.setdefault(p, []).append(j)
        parent_of[c] = j
    roots = [n for n in links if n not in parent_of]
    assert roots == ["world"], roots
    # pre-order DFS, children in joint declaration order
    order = []  # (link name, joint element)

    def dfs(name):
        for j in child_joints.get(name, []):
            c = j.find("child").get("link")
            order.append((c, j))
            dfs(c)
    dfs("world")
    assert len(order) == 19
    names = [n for n, _ in order]
    idx = {n: i for i, n in enumerate(names)}
    idx["world"] = -1

    mesh_dir = os.path.dirname(URDF)
    L = []
    for i, (name, j) in enumerate(order):
        lk = links[name]
        jt = j.get("type")
        parent = idx[j.find("parent").get("link")]
        Tj = origin_of(j)
        axis = np.array([float(v) for v in (j.find("axis").get("xyz").split() if j.find("axis") is not None else "1 0 0".split())])
        lim = j.find("limit")
        inert = lk.find("inertial")
        if inert is not None:
            mass = float(inert.find("mass").get("value"))
            Ti = origin_of(inert)
        else:
            mass = 1.0
            Ti = np.eye(4)
        shapes = []
        for col in lk.findall("collision"):
            Tc = origin_of(col)
            g = col.find("geometry")
            if g.find("box") is not None:
                size = np.array([float(v) for v in g.find("box").get("size").split()])
                shapes.append(dict(kind="box", T=Tc, half=size / 2))
            elif g.find("mesh") is not None:
                m = g.find("mesh")
                fn = os.path.normpath(os.path.join(mesh_dir, m.get("filename")))
                scale = np.array([float(v) for v in m.get("scale", "1 1 1").split()])
                pts = read_stl(fn) if fn.endswith(".stl") else read_dae(fn)
                pts = pts * scale
                verts, planes, full, fplanes, csizes = hull_of(pts)
                shapes.append(dict(kind="hull", T=Tc, verts=verts, planes=planes, full=full, fplanes=fplanes,
                                   csizes=csizes, file=os.path.basename(fn)))
        # compound AABB in inertial frame (child AABB includes margin; compound margin 0)
        Tinv = np.linalg.inv(Ti)
        lo = np.full(3, np.inf)
        hi = np.full(3, -np.inf)
        for s in shapes:
            T = Tinv @ s["T"]
            if s["kind"] == "box":
                h = s["half"]
                c = T[:3, 3]
                e = np.abs(T[:3, :3]) @ h  # btBoxShape AABB: halfExtents (margin inside)
                lo = np.minimum(lo, c - e)
                hi = np.maximum(hi, c + e)
            else:
                # inertia / getAABB use the full hull, not the collision LOD
                p = (T[:3, :3] @ s["full"].T).T + T[:3, 3]
                lo = np.minimum(lo, p.min(0) - MARGIN)
                hi = np.maximum(hi, p.max(0) + MARGIN)
        ext = hi - lo
        Idiag = mass / 12.0 * np.array([ext[1] ** 2 + ext[2] ** 2, ext[0] ** 2 + ext[2] ** 2, ext[0] ** 2 + ext[1] ** 2])
        L.append(dict(name=name, jname=j.get("name"), jtype=jt, parent=parent, Tj=Tj, axis=axis,
                      lower=float(lim.get("lower")) if lim is not None and lim.get("lower") else 0.0,
                      upper=float(lim.get("upper")) if lim is not None and lim.get("upper") else -1.0,
                      effort=float(lim.get("effort")) if lim is not None else 0.0,
                      vel=float(lim.get("velocity")) if lim is not None else 0.0,
                      mass=mass, Ti=Ti, Idiag=Idiag, shapes=shapes,
                      aabb_c=(lo + hi) / 2, aabb_h=(hi - lo) / 2))

    # controllable joints -> bodies
    dof_links = [i for i, l in enumerate(L) if l["jtype"] != "fixed"]
    assert dof_links == [1, 2, 3, 4, 5, 6, 9, 11, 13, 14, 16, 18], dof_links
    body_of = {}
    T_body_link = {}  # link frame expressed in its body frame
    for i, l in enumerate(L):
        if l["jtype"] != "fixed":
            body_of[i] = dof_links.index(i)
            T_body_link[i] = np.eye(4)
        else:
            p = l["parent"]
            if p == -1:
                body_of[i] = -1
                T_body_link[i] = l["Tj"]
            else:
                body_of[i] = body_of[p]
                T_body_link[i] = T_body_link[p] @ l["Tj"]
    NB = len(dof_links)
    bodies = []
    for b, li in enumerate(dof_links):
        l = L[li]
        pl = l["parent"]
        pb = body_of[pl]
        T_pb = T_body_link[pl] @ l["Tj"]  # joint frame in parent body frame (at q = 0)
        members = [i for i in range(19) if body_of[i] == b]
        m = 0.0
        mc = np.zeros(3)
        for i in members:
            Tc = T_body_link[i] @ L[i]["Ti"]
            m += L[i]["mass"]
            mc += L[i]["mass"] * Tc[:3, 3]
        com = mc / m
        I = np.zeros((3, 3))
        D = np.zeros((3, 3))
        for i in members:
            Tc = T_body_link[i] @ L[i]["Ti"]
            R = Tc[:3, :3]
            Ic = R @ np.diag(L[i]["Idiag"]) @ R.T
            D += Ic
            r = Tc[:3, 3] - com
            I += Ic + L[i]["mass"] * (np.dot(r, r) * np.eye(3) - np.outer(r, r))
        bodies.append(dict(link=li, parent=pb, T_pb=T_pb, axis=l["axis"], mass=m, com=com, I=I, D=D,
                           lower=l["lower"], upper=l["upper"], effort=l["effort"], vel=l["vel"], members=members))

    # ---- emit header ----
    out = []
    w = out.append

    def arr(name, a, ctype="double"):
        a = np.asarray(a, dtype=np.float64).ravel()
        if ctype == "int":
            body = ", ".join(str(int(x)) for x in a)
        else:
            body = ", ".join("%.17g" % x for x in a)
        w("UG_CONST %s %s[%d] = {%s};" % (ctype, name, len(a), body))

    def quat_of(R):
        # rotation matrix -> (x,y,z,w)
        t = np.trace(R)
        if t > 0:
            s = math.sqrt(t + 1.0) * 2
            return [(R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s, 0.25 * s]
        i = int(np.argmax(np.diag(R)))
        if i == 0:
            s = math.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
            return [0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s, (R[2, 1] - R[1, 2]) / s]
        if i == 1:
            s = math.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
            return [(R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s, (R[0, 2] - R[2, 0]) / s]
        s = math.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        return [(R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s, (R[1, 0] - R[0, 1]) / s]

    w("/* GENERATED by tools/build_model.py from %s and its collision meshes. Do not edit. */" % URDF_REL)
    w("/* Data, not code: shared as input by oracle/ (CPU restatement) and urgym_amd/csrc (HIP). */")
    w("#ifndef URGYM_MODEL_DATA_H")
    w("#define URGYM_MODEL_DATA_H")
    w("#ifndef UG_CONST")
    w("#define UG_CONST static const /* HIP translation units define it as __constant__ */")
    w("#endif")
    w("#define UG_NB %d          /* moving bodies = controllable joints (dofs) */" % NB)
    w("#define UG_NL 19          /* PyBullet link count (link index = DFS order) */")
    w("#define UG_EE_LINK 7")
    w("/* body b: joint frame in parent body frame at q=0 (rotation matrix row-major, translation) */")
    w("#define UG_BODY_PARENT_INIT {%s} /* also a compile-time table in the HIP code */"
      % ", ".join(str(int(b["parent"])) for b in bodies))
    w("UG_CONST int UG_BODY_PARENT[%d] = UG_BODY_PARENT_INIT;" % len(bodies))
    arr("UG_BODY_LINK", [b["link"] for b in bodies], "int")
    arr("UG_BODY_R", [b["T_pb"][:3, :3] for b in bodies])
    arr("UG_BODY_P", [b["T_pb"][:3, 3] for b in bodies])
    arr("UG_BODY_AXIS", [b["axis"] for b in bodies])
    arr("UG_BODY_MASS", [b["mass"] for b in bodies])
    arr("UG_BODY_COM", [b["com"] for b in bodies])
    arr("UG_BODY_I", [[b["I"][0, 0], b["I"][1, 1], b["I"][2, 2], b["I"][0, 1], b["I"][0, 2], b["I"][1, 2]] for b in bodies])
    arr("UG_BODY_DAMPI", [[b["D"][0, 0], b["D"][1, 1], b["D"][2, 2], b["D"][0, 1], b["D"][0, 2], b["D"][1, 2]] for b in bodies])
    arr("UG_DOF_LOWER", [b["lower"] for b in bodies])
    arr("UG_DOF_UPPER", [b["upper"] for b in bodies])
    arr("UG_DOF_MAXFORCE", [b["effort"] for b in bodies])
    arr("UG_DOF_MAXVEL", [b["vel"] for b in bodies])
    w("/* per PyBullet link: owning body (-1 = fixed base), link frame in body frame, COM frame in body frame */")
    arr("UG_LINK_BODY", [body_of[i] for i in range(19)], "int")
    arr("UG_LINK_R", [T_body_link[i][:3, :3] for i in range(19)])
    arr("UG_LINK_P", [T_body_link[i][:3, 3] for i in range(19)])
    arr("UG_LINK_COMR", [(T_body_link[i] @ L[i]["Ti"])[:3, :3] for i in range(19)])
    arr("UG_LINK_COMP", [(T_body_link[i] @ L[i]["Ti"])[:3, 3] for i in range(19)])
    arr("UG_LINK_MASS", [L[i]["mass"] for i in range(19)])
    w("/* compound-shape local AABB (centre, half) in the link inertial frame, margins included */")
    arr("UG_LINK_AABB_C", [L[i]["aabb_c"] for i in range(19)])
    arr("UG_LINK_AABB_H", [L[i]["aabb_h"] for i in range(19)])
    # angular motion disc of the link collider compound: bounding sphere radius + centre offset
    disc = [float(np.linalg.norm(L[i]["aabb_h"]) + np.linalg.norm(L[i]["aabb_c"])) for i in range(19)]
    arr("UG_LINK_DISC", disc)
    # collision shapes: flatten
    shp_link, shp_kind, shp_R, shp_P, shp_half, shp_v0, shp_nv, shp_f0, shp_nf = [], [], [], [], [], [], [], [], []
    V, F = [], []
    FV, FV0, FVN = [], [], []  # face polygons (HULL_POLYS): global vertex indices, per-face start / count
    for i in range(19):
        for s in L[i]["shapes"]:
            T = T_body_link[i] @ s["T"]  # shape frame in body frame
            shp_link.append(i)
            shp_R.append(T[:3, :3])
            shp_P.append(T[:3, 3])
            if s["kind"] == "box":
                shp_kind.append(0)
                shp_half.append(s["half"])
                shp_v0.append(0); shp_nv.append(0); shp_f0.append(0); shp_nf.append(0)
            else:
                shp_kind.append(1)
                vv = s["verts"]
                lo, hi = vv.min(0), vv.max(0)
                shp_half.append((hi - lo) / 2)  # unused for hulls except AABB sizing
                shp_v0.append(len(V)); shp_nv.append(len(vv)); shp_f0.append(len(F)); shp_nf.append(len(s["planes"]))
                if HULL_POLYS:
                    for lp in face_loops(vv, s["planes"]):
                        FV0.append(len(FV)); FVN.append(len(lp)); FV.extend(len(V) + i for i in lp)
                V.extend(vv.tolist())
                F.extend(s["planes"].tolist())
    # Golf club disc (env_golf_v0.py:293-305: GEOM_CYLINDER r 0.04, height 0.01, Z axis): a 16-sided prism
    # with the cylinder's safe margin (0.1 x min half extent) outside, so the outer extent is the cylinder's
    # (hull vertices on the circle of radius r - m; restated substitute for btCylinderShapeZ + GJK)
    cyl_r, cyl_h, cyl_m, nseg = 0.04, 0.005, 0.0005, CYL_SEG
    cyl_v0, cyl_f0 = len(V), len(F)
    rr, hh = cyl_r - cyl_m, cyl_h - cyl_m
    for zs in (-hh, hh):
        for k in range(nseg):
            th = 2.0 * np.pi * k / nseg
            V.append([rr * np.cos(th), rr * np.sin(th), zs])
    apo = rr * np.cos(np.pi / nseg)
    for k in range(nseg):
        th = 2.0 * np.pi * (k + 0.5) / nseg
        F.append([np.cos(th), np.sin(th), 0.0, apo])
    F.append([0.0, 0.0, 1.0, hh])
    F.append([0.0, 0.0, -1.0, hh])
    if HULL_POLYS:  # side k joins bottom k, k+1 and top k+1, k (outward ccw), then top and bottom caps
        for k in range(nseg):
            k1 = (k + 1) % nseg
            FV0.append(len(FV)); FVN.append(4)
            FV.extend([cyl_v0 + k, cyl_v0 + k1, cyl_v0 + nseg + k1, cyl_v0 + nseg + k])
        FV0.append(len(FV)); FVN.append(nseg); FV.extend(cyl_v0 + nseg + k for k in range(nseg))
        FV0.append(len(FV)); FVN.append(nseg); FV.extend(cyl_v0 + k for k in reversed(range(nseg)))
    # the full hulls (every vertex of PyBullet's convex hull of the mesh, every merged face) after the LOD data and
    # the prism, for the full-geometry mode (URGYM_FLAG_FULL_GEOMETRY): per-shape offsets into the same arrays
    shp_fv0, shp_fnv, shp_ff0, shp_fnf, shp_fc0 = [], [], [], [], []
    CS = []  # per 64-vertex chunk of a full hull: bounding sphere (centre in the shape frame, radius)
    for i in range(19):
        for sh in L[i]["shapes"]:
            if sh["kind"] == "box":
                shp_fv0.append(0); shp_fnv.append(0); shp_ff0.append(0); shp_fnf.append(0); shp_fc0.append(0)
            else:
                shp_fv0.append(len(V)); shp_fnv.append(len(sh["full"])); shp_ff0.append(len(F)); shp_fnf.append(len(sh["fplanes"]))
                shp_fc0.append(len(CS) // 4)
                for a in range(0, len(sh["full"]), 64):
                    cv = sh["full"][a:a + 64]
                    c = (cv.min(0) + cv.max(0)) / 2
                    r = float(np.linalg.norm(cv - c, axis=1).max())
                    CS.extend([c[0], c[1], c[2], r * (1 + 1e-12) + 1e-12])  # rounded up: an upper bound
                if HULL_POLYS:
                    for lp in face_loops(sh["full"], sh["fplanes"]):
                        FV0.append(len(FV)); FVN.append(len(lp)); FV.extend(len(V) + k for k in lp)
                V.extend(sh["full"].tolist())
                F.extend(sh["fplanes"].tolist())
    w("#define UG_CYL_V0 %d   /* golf club disc prism: 2 x %d vertices */" % (cyl_v0, nseg))
    w("#define UG_CYL_NV %d" % (2 * nseg))
    w("#define UG_CYL_F0 %d" % cyl_f0)
    w("#define UG_CYL_NF %d" % (nseg + 2))
    w("#define UG_CYL_R %.17g" % cyl_r)
    w("#define UG_CYL_HH %.17g" % cyl_h)
    w("#define UG_CYL_MARGIN %.17g" % cyl_m)
    w("#define UG_NSHAPE %d" % len(shp_link))
    w("#define UG_NHULLV %d" % len(V))
    w("#define UG_NHULLF %d" % len(F))
    w("/* shape kind: 0 box (half extents, margin inside), 1 convex hull (+margin 0.001 outside) */")
    arr("UG_SHAPE_LINK", shp_link, "int")
    arr("UG_SHAPE_KIND", shp_kind, "int")
    arr("UG_SHAPE_R", shp_R)
    arr("UG_SHAPE_P", shp_P)
    arr("UG_SHAPE_HALF", shp_half)
    arr("UG_SHAPE_V0", shp_v0, "int")
    arr("UG_SHAPE_NV", shp_nv, "int")
    arr("UG_SHAPE_F0", shp_f0, "int")
    arr("UG_SHAPE_NF", shp_nf, "int")
    w("/* full-geometry mode: the same shapes' full hulls (offsets into UG_HULL_V / UG_HULL_F) */")
    w("#define UG_FULL_HULL_MAXV %d" % max(shp_fnv))
    w("#define UG_FULL_HULL_MAXF %d" % max(shp_fnf))
    arr("UG_SHAPE_FV0", shp_fv0, "int")
    arr("UG_SHAPE_FNV", shp_fnv, "int")
    arr("UG_SHAPE_FF0", shp_ff0, "int")
    arr("UG_SHAPE_FNF", shp_fnf, "int")
    arr("UG_SHAPE_FC0", shp_fc0, "int")
    w("/* full hulls: bounding sphere (centre x y z, radius) of each 64-vertex chunk, vertices grouped spatially */")
    arr("UG_HULL_CS", CS)
    arr("UG_HULL_V", V)
    arr("UG_HULL_F", F)
    if HULL_POLYS:
        assert len(FV0) == len(F)
        w("#define UG_HULL_POLYS 1")
        w("#define UG_NHULLFV %d" % len(FV))
        arr("UG_HULL_FV", FV, "int")
        arr("UG_HULL_FV0", FV0, "int")
        arr("UG_HULL_FVN", FVN, "int")
    w("/* arm rest pose, robot.py:182-183 */")
    arr("UG_ARM_REST", [-1.5690622952052096, -1.5446774605904932, 1.343946009733127, -1.3708613585093699,
                        -1.5707970583733368, 0.0009377758247187636])
    w("#endif")
    open(OUT, "w").write("\n".join(out) + "\n")
    # report
    for b in bodies:
        print("body link %2d parent %2d mass %.5f members %s" % (b["link"], b["parent"], b["mass"], b["members"]))
    for i in range(19):
        print("link %2d %-28s shapes %s" % (i, L[i]["name"], [(s["kind"], len(s.get("verts", [])), len(s.get("planes", []))) for s in L[i]["shapes"]]))
    print("hull verts", len(V), "faces", len(F), "->", OUT)


if __name__ == "__main__":
    main()
