#!/usr/bin/env python3
"""Geometry / contact-generation divergence table ("quantify the collision substitutes"; r2: the
reference-faithful geometry on the product path).

The product path (kernels and the parity oracle) defaults to the reference's geometry (robot hulls with every
vertex and face of PyBullet's mesh hulls, the club's disc as a true cylinder) and to PyBullet's own convex-convex
contact path: btConvexConvexAlgorithm -> btGjkPairDetector (GJK + EPA, one new point per pair and substep into the
persistent manifold), sphere-sphere / sphere-box / box-box keeping their dedicated algorithms.  This tool runs the
same seeded random-action rollouts from the same initial states through

  product   the default restatement (flags 0: GJK / EPA), the one the kernels match bit for bit
  floor     product with Bullet's own PGS arithmetic form (oracle pgs_bullet, ~1e-11 per substep): the growth of a
            rounding-level difference, i.e. the chaos floor of each task
  lod       the collision LOD (URGYM_FLAG_LOD_GEOMETRY: <= 48-vertex hulls, 16-gon disc prism), GJK / EPA contacts
  vih       rounds 1-3's contact generator (URGYM_FLAG_CONTACT_VIH: vertex-in-hull tests against the face planes,
            deepest + farthest-spread 4 points), full geometry
  sat       full hulls + a 128-gon disc prism + Bullet's polyhedral SAT path restated (oracle/ug_fidelity.h:
            separating axis over face normals and edge-edge cross products, incident-face clipping) -- what Bullet
            runs only for hulls loaded with URDF_INITIALIZE_SAT_FEATURES, which the reference never passes [ext]; a
            separate build (oracle/_fid/, test / measurement infrastructure, never shipped)

reporting, after 1, 10 and 100 env-steps, the divergence of each variant from `product`: max |dq| over the
12 robot dofs (rad), max object position difference (m), and the fraction of envs whose episode ended at a
different step.  Output: profiles/collision_fidelity.json and a markdown table on stdout.

usage: python tools/collision_fidelity.py [--envs 6] [--steps 100] [--tasks 0,1,2,3,4,5,6] [--jobs 8]
(CPU only, this container: the bullet build needs /root/reference for the full meshes)
"""
import argparse
import json
import multiprocessing as mp
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
FID = os.path.join(ROOT, "oracle", "_fid")
HDR = os.path.join(FID, "model_data.h")
LIBS = {"sat": os.path.join(FID, "libugoracle_fid.so")}
# creation flags per variant: the sat build's LOD slot holds the full hulls + 128-gon (URGYM_HULL_MAXV above) and its
# polyhedral path replaces the vertex-in-hull generator (8)
FLAGS = {"lod": 2, "vih": 8, "sat": 2 | 8}
CFLAGS = ["-O2", "-std=gnu99", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-mfma", "-Wall",
          "-Wno-unused-function", "-Wno-unknown-pragmas", "-shared"]
CHECK = (1, 10, 100)
NAMES = {0: "BallBalance", 1: "CubesPush", 2: "CubesGrasp", 3: "Golf", 4: "CubesPushDiff", 5: "GolfJoints",
         6: "TwoBallsBalance"}


def build():
    os.makedirs(FID, exist_ok=True)
    env = dict(os.environ, URGYM_MODEL_OUT=HDR, URGYM_HULL_MAXV="100000", URGYM_CYL_SEG="128", URGYM_HULL_POLYS="1")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "build_model.py")], env=env, check=True,
                   stdout=subprocess.DEVNULL)
    src = os.path.join(ROOT, "oracle", "ug_oracle.c")
    common = CFLAGS + ["-DMAXCAND=4096", "-DLOD_MAXCAND=4096", '-DUG_MODEL_DATA="_fid/model_data.h"']
    subprocess.run(["gcc"] + common + ["-DUG_FIDELITY", "-o", LIBS["sat"], src, "-lm"], check=True,
                   cwd=os.path.join(ROOT, "oracle"))


def actions(task, steps, seed):
    from urgym_amd.envs import spaces_for
    act = spaces_for(task)[1]
    rng = np.random.default_rng(seed)
    lo, hi = np.asarray(act.low, np.float64), np.asarray(act.high, np.float64)
    return rng.uniform(lo, hi, size=(steps, len(lo))).astype(np.float32)


def rollout(job):
    """one env of one task through one variant: states at the checkpoints (or the step its episode ended)"""
    task, env_i, variant, steps, s0 = job
    from oracle.pyoracle import OracleEnv
    from urgym_amd import layout as LY
    e = OracleEnv(task, 1000 + env_i, lib_path=LIBS.get(variant), flags=FLAGS.get(variant, 0))
    if variant == "floor":
        e.set_pgs_bullet(True)
    e.set_state(s0)
    acts = actions(task, steps, 7000 + 31 * task + env_i)
    out, ended = {}, None
    for t in range(steps):
        _, _, term, _, _ = e.step(acts[t])
        s = e.get_state()
        if t + 1 in CHECK:
            out[t + 1] = s[:LY.F_NMAN].copy()
        if term or not np.all(np.isfinite(s)):
            ended = t + 1
            break
    return (task, env_i, variant), out, ended


def initial_state(task, env_i):
    from oracle.pyoracle import OracleEnv
    e = OracleEnv(task, 1000 + env_i)
    e.reset()
    return e.get_state()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=6)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--tasks", default="0,1,2,3,4,5,6")
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--no-build", action="store_true")
    a = ap.parse_args()
    if not a.no_build:
        build()
    from urgym_amd import layout as LY
    tasks = [int(t) for t in a.tasks.split(",")]
    variants = ["product", "floor", "lod", "vih", "sat"]
    jobs = []
    for t in tasks:
        for i in range(a.envs):
            s0 = initial_state(t, i)
            for v in variants:
                jobs.append((t, i, v, a.steps, s0))
    with mp.get_context("fork").Pool(a.jobs) as pool:
        res = pool.map(rollout, jobs, chunksize=1)
    R = {k: (o, ended) for k, o, ended in res}
    obj = slice(LY.F_OBJ, LY.F_OBJ + LY.OBJ_DOUBLES * LY.MAXOBJ)
    table = {}
    for t in tasks:
        table[NAMES[t]] = {}
        for v in variants[1:]:
            row = {}
            for c in CHECK:
                dq, dp, n = [], [], 0
                for i in range(a.envs):
                    (po, pe), (vo, ve) = R[(t, i, "product")], R[(t, i, v)]
                    if c in po and c in vo:
                        n += 1
                        dq.append(float(np.abs(po[c][:12] - vo[c][:12]).max()))
                        d = (po[c][obj] - vo[c][obj]).reshape(LY.MAXOBJ, LY.OBJ_DOUBLES)[:, :3]
                        dp.append(float(np.abs(d).max()))
                ended_diff = sum(1 for i in range(a.envs)
                                 if (R[(t, i, "product")][1] or 10 ** 9) != (R[(t, i, v)][1] or 10 ** 9)
                                 and min(R[(t, i, "product")][1] or 10 ** 9, R[(t, i, v)][1] or 10 ** 9) <= c)
                row[str(c)] = {"envs_compared": n, "max_dq_rad": max(dq) if dq else None,
                               "median_dq_rad": float(np.median(dq)) if dq else None,
                               "max_dpos_m": max(dp) if dp else None,
                               "median_dpos_m": float(np.median(dp)) if dp else None,
                               "episode_end_differs": ended_diff}
            table[NAMES[t]][v] = row
    out = {"what": __doc__.split("\n\n")[0],
           "product": "full hulls + true cylinder disc (the default geometry), GJK / EPA contacts (the default)",
           "variants": {"floor": "product restatement with Bullet's PGS arithmetic form (rounding-level seed)",
                        "lod": "the collision LOD (<= 48-vertex hulls, 16-gon disc prism), GJK / EPA contacts",
                        "vih": "rounds 1-3's vertex-in-hull contact generator, full geometry",
                        "sat": "full hulls + 128-gon + Bullet's SAT polyhedral clipping (URDF_INITIALIZE_SAT_FEATURES "
                               "only, unused by the reference) (oracle/ug_fidelity.h)"},
           "envs_per_task": a.envs, "steps": a.steps, "checkpoints": list(CHECK),
           "action_sampling": "uniform in the action space, numpy PCG64 seed 7000 + 31 task + env",
           "initial_state": "OracleEnv(task, 1000 + env).reset(), shared by every variant", "tasks": table}
    with open(os.path.join(ROOT, "profiles", "collision_fidelity.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print("| task | variant | " + " | ".join(f"max dq / max dpos after {c}" for c in CHECK) + " |")
    print("|---|---|" + "---|" * len(CHECK))
    for tn, rows in table.items():
        for v, row in rows.items():
            cells = []
            for c in CHECK:
                r = row[str(c)]
                if r["max_dq_rad"] is None:
                    cells.append("ended")
                else:
                    cells.append(f"{r['max_dq_rad']:.1e} / {r['max_dpos_m']:.1e} ({r['envs_compared']})")
            print(f"| {tn} | {v} | " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main()
