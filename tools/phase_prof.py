#!/usr/bin/env python3
"""Per-phase cycle breakdown of the team kernels (development aid).

Needs the instrumented library: hipcc ... -DUG_PROF -o urgym_amd/_lib/liburgym_prof.so
(tools/build_prof.sh).  Runs a task (default BallBalance) x N envs with autoreset for K steps and prints
cycles per phase per env-step, plus substeps / rows / PGS iterations per substep.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("URGYM_LIB", os.path.join(ROOT, "urgym_amd", "_lib", "liburgym_prof.so"))

CALLS = ["team_gjk", "team_collide", "team_enumerate", "team_unit_solves", "team_robot_dynamics", "serial_pre",
         "serial_post", "serial_fk", "team_pgs", "glue", "team_reduce4_g"]  # ug_team.h CALL_* (buf[104 + k])
NAMES = ["collide", "dyn+enum", "rows", "pgs", "pgs_setup", "integrate", "glue", "total",
         "substeps", "nrows", "pgs_iters", "overlap_pairs", "hull_pairs", "manifolds", "pgs_sweeps", "hull_narrowphase",
         "robot_dynamics", "enumerate", "broadphase", "pair_narrowphase",
         "hullbox_vertices", "hullbox_corners", "hullbox_reduce", "fk", "lane0_ldl_objects", "unit_solves",
         "row_build", "rb_jacobians", "rb_solves", "rb_scalars", "pgs_mfma",
         "pgs_warm", "sw_nc", "sw_contact", "sw_finish", "sw_fric_prep", "sw_fric", "sw_res",
         "pr_lookup", "pr_narrow", "pr_manifold", "pr_store", "chunks", "nnc", "nn", "n_le64", "n_65_80", "n_81_96",
         "free_substeps", "free_collide", "free_dyn", "free_rows", "free_pgs", "free_integrate",
         "free_pgs_setup", "free_pgs_sweeps", "free_pgs_sweeps_plus_post", "pr_boxbox", "hull_sphere",
         "cyl_pairs", "cyl_pass1", "cyl_pass2", "cyl_survivors", "cyl_scan_iters"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--task", type=int, default=0)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--geometry", choices=("lod", "full"), default="full")
    ap.add_argument("--contact", choices=("gjk", "vih"), default="gjk")
    a = ap.parse_args()
    from urgym_amd._native import CONTACT_VIH, GEOM_LOD, Sim
    sim = Sim(a.task, a.envs, seed=20241220,
              flags=(GEOM_LOD if a.geometry == "lod" else 0) | (CONTACT_VIH if a.contact == "vih" else 0))
    from urgym_amd.envs import spaces_for
    _, asp = spaces_for(a.task)
    sim.set_autoreset(True, 500)
    buf = np.zeros(134, np.uint64)
    sim.reset()
    sim.sync()
    rc = sim.L.urgym_debug_prof(sim.h, buf.ctypes.data_as(ctypes.c_void_p), 1)
    assert rc == 0, "library not built with -DUG_PROF"
    r = {k: float(v) for k, v in zip(NAMES, buf[:len(NAMES)])}
    print("reset (cycles per substep):", json.dumps({k: round(r[k] / max(r["substeps"], 1), 1) for k in NAMES}))
    print("reset, contact-free substeps:", json.dumps({"fraction": r["free_substeps"] / max(r["substeps"], 1),
          **{k + "_cycles": round(r[k] / max(r["free_substeps"], 1), 1) for k in NAMES[-15:-7]}}))
    free_split = ["fk", "broadphase", "hull_narrowphase", "pr_lookup", "pr_narrow", "pr_manifold", "pr_store",
                  "pairs", "overlap_pairs", "hull_pairs", "robot_dynamics", "lane0_ldl_objects", "enumerate",
                  "unit_solves"]
    print("reset, quiescent substeps (collision skipped):", round(float(buf[115]) / max(r["substeps"], 1), 3))
    print("reset, calls per env:", json.dumps({k: round(float(buf[104 + i]) / a.envs, 2) for i, k in enumerate(CALLS)}))
    print("reset, contact-free substeps' sub-phases (cycles or counts per substep):",
          json.dumps({k: round(float(buf[64 + i]) / max(r["free_substeps"], 1), 1) for i, k in enumerate(free_split)}))
    rng = np.random.default_rng(1)
    for _ in range(a.steps):
        sim.step(rng.uniform(asp.low, asp.high, size=(a.envs, len(asp.low))).astype(np.float32))
    sim.sync()
    sim.L.urgym_debug_prof(sim.h, buf.ctypes.data_as(ctypes.c_void_p), 1)
    es = a.envs * a.steps
    d = {k: float(v) for k, v in zip(NAMES, buf[:len(NAMES)])}
    out = {"per_env_step_cycles": {k: d[k] / es for k in NAMES[:8]},
           "substeps_per_env_step": d["substeps"] / es,
           "rows_per_substep": d["nrows"] / max(d["substeps"], 1),
           "pgs_iters_per_substep": d["pgs_iters"] / max(d["substeps"], 1),
           "pgs_cycles_per_row_update": d["pgs"] / max(d["nrows"] * d["pgs_iters"] / max(d["substeps"], 1), 1),
           "collide_cycles_per_substep": d["collide"] / max(d["substeps"], 1),
           "overlap_pairs_per_substep": d["overlap_pairs"] / max(d["substeps"], 1),
           "hull_pairs_per_substep": d["hull_pairs"] / max(d["substeps"], 1),
           "manifolds_per_substep": d["manifolds"] / max(d["substeps"], 1)}
    out["pgs_sweep_cycles_per_row_update"] = d["pgs_sweeps"] / max(d["nrows"] * d["pgs_iters"] / max(d["substeps"], 1), 1)
    out["pgs_sweep_cycles_per_row_slot"] = d["pgs_sweeps"] / max(8 * d["chunks"], 1)  # chunk rows incl. neutral
    out["row_slots_per_sweep"] = 8 * d["chunks"] / max(d["pgs_iters"], 1)
    out["substep_fraction_rows_le64_65to80_81to96"] = [d[k] / max(d["substeps"], 1) for k in ("n_le64", "n_65_80", "n_81_96")]
    out["nc_normal_friction_rows_per_substep"] = [d["nnc"] / max(d["substeps"], 1), d["nn"] / max(d["substeps"], 1),
                                                  (d["nrows"] - d["nnc"] - d["nn"]) / max(d["substeps"], 1)]
    for k in ("dyn+enum", "rows", "pgs", "pgs_setup", "pgs_sweeps", "hull_narrowphase", "robot_dynamics",
              "enumerate", "broadphase", "pair_narrowphase", "hullbox_vertices", "hullbox_corners",
              "hullbox_reduce", "fk", "lane0_ldl_objects", "unit_solves", "row_build", "rb_jacobians", "rb_solves",
              "rb_scalars", "pgs_mfma", "pgs_warm", "sw_nc", "sw_contact", "sw_finish",
              "sw_fric_prep", "sw_fric", "sw_res", "pr_lookup", "pr_narrow", "pr_manifold", "pr_store", "integrate", "pr_boxbox", "hull_sphere",
              "cyl_pairs", "cyl_pass1", "cyl_pass2", "cyl_survivors", "cyl_scan_iters"):
        out[k + "_cycles_per_substep"] = d[k] / max(d["substeps"], 1)
    gj = dict(zip(["gjk_queries", "gjk_epa_queries", "gjk_iterations", "gjk_ccd_iterations", "gjk_hull_supports",
                   "gjk_hull_support_cycles", "epa_iterations", "gjk_cycles_reporting_queries", "gjk_penetration_cycles",
                   "gjk_ccd_cycles", "gjk_classic_cycles", "epa_gjk_cycles", "epa_setup_cycles", "epa_support_cycles",
                   "epa_expand_cycles", "epa_findbest_cycles", "ccd_support_cycles", "ccd_simplex_cycles",
                   "classic_support_cycles", "classic_simplex_cycles", "gjk_recertified"], [float(x) for x in buf[80:101]]))
    out["gjk_per_substep"] = {k: v / max(d["substeps"], 1) for k, v in gj.items()}
    out["gjk_cycles_per_hull_support"] = gj["gjk_hull_support_cycles"] / max(gj["gjk_hull_supports"], 1)
    # inside a support (cumulative from its start): the cell known, the cell's loads landed (forced wait)
    sc = dict(zip(["cell", "mem", "cells"], [float(x) for x in buf[101:104]]))
    out["hull_support_split"] = {"supports_through_a_cell": sc["cells"] / max(gj["gjk_hull_supports"], 1),
                                 "cycles_to_cell": sc["cell"] / max(gj["gjk_hull_supports"], 1),
                                 "cycles_to_reduced": sc["mem"] / max(sc["cells"], 1)}
    out["calls_per_env_step"] = {k: float(buf[104 + i]) / es for i, k in enumerate(CALLS)}
    out["quiescent_substeps_fraction"] = float(buf[115]) / max(d["substeps"], 1)
    # the calling convention's cost (ug_team.h PF_CS0): call + prologue (callee-saved saves) and epilogue (restores,
    # their wait, the return) of team_gjk / team_collide<full, gjk> / team_pgs, cycles per call and per substep
    cs = {}
    for i, (name, call) in enumerate((("team_gjk", 0), ("team_collide", 1), ("team_pgs", 8), ("serial_fk", 7),
                                      ("serial_pre", 5), ("serial_post", 6), ("team_unit_solves", 3),
                                      ("team_robot_dynamics", 4), ("team_enumerate", 2))):
        ncall = max(float(buf[104 + call]), 1.0)
        pro, epi = float(buf[116 + 2 * i]), float(buf[117 + 2 * i])
        cs[name] = {"calls_per_substep": ncall / max(d["substeps"], 1), "prologue_cycles_per_call": pro / ncall,
                    "epilogue_cycles_per_call": epi / ncall,
                    "prologue_plus_epilogue_cycles_per_substep": (pro + epi) / max(d["substeps"], 1)}
    # serial_pre's own figures include its two nested calls' (team_robot_dynamics, team_enumerate) only through its body
    tot = sum(v["prologue_plus_epilogue_cycles_per_substep"] for v in cs.values())
    cs["share_of_substep_cycles"] = tot / max(d["total"] / max(d["substeps"], 1), 1)
    out["call_save_restore"] = cs
    print(json.dumps(out, indent=1))
    sim.close()


if __name__ == "__main__":
    main()
