#!/usr/bin/env python3
"""Known-answer fixture for the model compiler (tools/build_model.py -> urgym_amd/csrc/model_data.h), written
independently of it from the reference's robot description (run in the build container only):

  /root/reference/urgym/urdf/ur5_robotiq_85.urdf  -- links, joints, <inertial> masses and origins, limits
  its collision meshes                            -- full convex hulls (scipy), summarised per link as the
                                                     support function h(d) = max_v d.v over a fixed direction
                                                     set and as the hull's AABB in the link's inertial frame

Writes tests/golden/urdf_model.json (data: URDF facts and mesh summaries).  tests/test_model_kat.py checks the
generated header against it: PyBullet's pre-order DFS link indices (robot.py:180 eef 7, grippers 9..18), masses
(1 kg for a link without <inertial>), merged-body masses / COMs, the collision-AABB box-inertia rule
 and the bound on the collision LOD (decimated hulls vs the full hulls).
"""
import json
import math
import os
import sys
import xml.etree.ElementTree as ET

import numpy as np
from scipy.spatial import ConvexHull

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("URGYM_REFERENCE", "/root/reference")
# URGYM_MODEL_URDF=urgym/urdf/ur5_robotiq_140.urdf writes the UR5Robotiq140 fixture (urdf_model_r140.json)
URDF_REL = os.environ.get("URGYM_MODEL_URDF", "urgym/urdf/ur5_robotiq_85.urdf")
URDF = os.path.join(REF, URDF_REL)
OUT = os.path.join(ROOT, "tests", "golden", "urdf_model_r140.json" if "140" in URDF_REL else "urdf_model.json")


def fib_dirs(n=64):
    """n unit directions on a Fibonacci sphere plus the 6 axes"""
    d = [[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]]
    g = math.pi * (3.0 - math.sqrt(5.0))
    for i in range(n):
        z = 1.0 - 2.0 * (i + 0.5) / n
        r = math.sqrt(1.0 - z * z)
        d.append([r * math.cos(g * i), r * math.sin(g * i), z])
    return np.array(d)


def rpy(r, p, y):
    """URDF fixed-axis roll, pitch, yaw: R = Rz(y) Ry(p) Rx(r)"""
    Rx = np.array([[1, 0, 0], [0, math.cos(r), -math.sin(r)], [0, math.sin(r), math.cos(r)]])
    Ry = np.array([[math.cos(p), 0, math.sin(p)], [0, 1, 0], [-math.sin(p), 0, math.cos(p)]])
    Rz = np.array([[math.cos(y), -math.sin(y), 0], [math.sin(y), math.cos(y), 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def origin(el):
    o = None if el is None else el.find("origin")
    xyz = [0.0, 0.0, 0.0] if o is None else [float(v) for v in o.get("xyz", "0 0 0").split()]
    r = [0.0, 0.0, 0.0] if o is None else [float(v) for v in o.get("rpy", "0 0 0").split()]
    return xyz, r


def mesh_points(path, scale):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from build_model import read_dae, read_stl  # plain file readers (binary STL / COLLADA float arrays)
    pts = read_stl(path) if path.endswith(".stl") else read_dae(path)
    return pts * np.asarray(scale)


def main():
    root = ET.parse(URDF).getroot()
    links = {l.get("name"): l for l in root.findall("link")}
    kids = {}
    for j in root.findall("joint"):
        kids.setdefault(j.find("parent").get("link"), []).append(j)
    order = []

    def visit(name):  # pybullet link index = pre-order depth-first, children in declaration order [ext]
        for j in kids.get(name, []):
            order.append(j)
            visit(j.find("child").get("link"))
    visit("world")
    dirs = fib_dirs()
    out = {"directions": dirs.tolist(), "links": []}
    names = [j.find("child").get("link") for j in order]
    for j in order:
        name = j.find("child").get("link")
        lk = links[name]
        inert = lk.find("inertial")
        mass = float(inert.find("mass").get("value")) if inert is not None else None
        ixyz, irpy = origin(inert)
        jxyz, jrpy = origin(j)
        ax = j.find("axis")
        rec = {"name": name, "joint": j.get("name"), "type": j.get("type"),
               "parent": names.index(j.find("parent").get("link")) if j.find("parent").get("link") in names else -1,
               "joint_xyz": jxyz, "joint_rpy": jrpy,
               "axis": [float(v) for v in ax.get("xyz").split()] if ax is not None else None,
               "mass": mass, "inertial_xyz": ixyz, "inertial_rpy": irpy, "collision": []}
        lim = j.find("limit")
        if lim is not None:
            rec["limit"] = {k: float(lim.get(k)) for k in ("lower", "upper", "effort", "velocity") if lim.get(k)}
        for col in lk.findall("collision"):
            cxyz, crpy = origin(col)
            g = col.find("geometry")
            c = {"xyz": cxyz, "rpy": crpy}
            if g.find("box") is not None:
                c["box"] = [float(v) for v in g.find("box").get("size").split()]
            else:
                m = g.find("mesh")
                path = os.path.normpath(os.path.join(os.path.dirname(URDF), m.get("filename")))
                scale = [float(v) for v in m.get("scale", "1 1 1").split()]
                pts = mesh_points(path, scale)
                full = pts[ConvexHull(pts).vertices]
                c["mesh"] = os.path.basename(path)
                c["hull_vertices"] = int(len(full))
                c["support"] = (full @ dirs.T).max(0).tolist()         # h(d) of the full hull, mesh frame
                # AABB of the full hull in the link's inertial frame (the inertia rule's input)
                Ri, pi = rpy(*irpy), np.array(ixyz)
                Rc, pc = rpy(*crpy), np.array(cxyz)
                p = ((Rc @ full.T).T + pc - pi) @ Ri                    # inertial-frame coordinates
                c["aabb_inertial"] = [p.min(0).tolist(), p.max(0).tolist()]
            rec["collision"].append(c)
        out["links"].append(rec)
    json.dump(out, open(OUT, "w"), indent=1)
    print("wrote", OUT, len(out["links"]), "links")


if __name__ == "__main__":
    main()
