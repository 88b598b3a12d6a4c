"""Reduce rocprofv3 FETCH_SIZE / WRITE_SIZE passes to HBM bytes per k_step launch.

usage: python tools/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> <out.json>
       [--task T --envs N --steps K --warmup W --geometry G --contact C]

Units and corrections follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section): both counters are in
KB; on gfx950 FETCH_SIZE tallies 128-B requests at 64 B, so it is doubled; WRITE_SIZE is taken as is.
bench.py reads the output (profiles/traffic_k_step.json) to fill roofline.traffic for the same workload.
"""
import argparse
import csv
import json


def per_launch(path, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Kernel_Name"].startswith("k_step(") and r["Counter_Name"] == counter]
    if not vals:
        raise SystemExit(f"no k_step {counter} rows in {path}")
    return sum(vals) / len(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("out")
    ap.add_argument("--task", type=int, default=0)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--geometry", choices=("full", "lod"), default="full")
    ap.add_argument("--contact", choices=("gjk", "vih"), default="gjk")
    a, _ = ap.parse_known_args()
    f_kb, nf = per_launch(a.fetch, "FETCH_SIZE")
    w_kb, nw = per_launch(a.write, "WRITE_SIZE")
    fetch_b = 2.0 * f_kb * 1024.0  # gfx950: FETCH_SIZE reports half of the bytes read
    write_b = w_kb * 1024.0
    out = {"kernel": "k_step", "task": a.task, "envs": a.envs, "geometry": a.geometry, "contact": a.contact,
           "steps": a.steps, "warmup": a.warmup,
           "launches": [nf, nw], "fetch_size_kb_avg": f_kb, "write_size_kb_avg": w_kb,
           "hbm_bytes_per_launch": fetch_b + write_b, "read_bytes_per_launch": fetch_b,
           "write_bytes_per_launch": write_b,
           "correction": "FETCH_SIZE x2 (gfx950), KB -> bytes x1024; MI355X_MICROARCH.md HBM section"}
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
