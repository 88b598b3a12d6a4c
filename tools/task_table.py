"""Markdown table of the per-task bench lines (DESIGN.md 'Current state'): python tools/task_table.py <dir> [prefix]"""
import json
import os
import sys

NAMES = {0: "BallBalance", 1: "CubesPush", 2: "CubesGrasp", 3: "Golf", 4: "CubesPushDiff", 5: "GolfJoints",
         6: "TwoBallsBalance", 7: "Box"}
R5 = {0: 189761, 1: 84902, 2: 27572, 3: 73578, 4: 84322, 5: 37842, 6: 156266, 7: 42008}  # BENCH_r05 / round5_final3 (50 x 3)


def main():
    d, pre = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "task"
    print("| task | envs | env-steps/s (median of 5 × 200) | rep range | ms / env-step | substeps / env-step | FP64-VALU frac | library | round 5 |")
    print("|---|---|---|---|---|---|---|---|---|")
    for t in range(8):
        p = os.path.join(d, f"{pre}{t}.json")
        if not os.path.exists(p):
            continue
        b = json.load(open(p))
        c = b["config"]
        rv = b["rep_values"]
        print(f"| {NAMES[t]}-v0 | {c['envs_per_gpu']} | **{b['value'] / 1e3:.1f} k** | {min(rv) / 1e3:.1f}–{max(rv) / 1e3:.1f} k | "
              f"{b['ms_per_step']:.2f} | {b['substeps_per_env_step']:.1f} | {b['roofline']['frac']:.4f} | "
              f"`{os.path.basename(c.get('library', ''))}` | {R5[t] / 1e3:.1f} k |")


if __name__ == "__main__":
    main()
