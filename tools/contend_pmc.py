#!/usr/bin/env python3
"""Co-runner contention of k_step (development aid): the PMC passes of `tools/gpu.sh contend` at the
default wave slots (four waves per CU, one per SIMD) and at URGYM_SLOTS=256 (one wave per CU), summed over the
k_step dispatches and divided by the env-steps they ran (envs x dispatches; the same seeded work in both runs).
Reports, per env-step: wave cycles, cycles waiting on anything / on instruction issue, instruction fetches and I-cache
misses, L2 (TCC) hits and misses, the L1->L2 read latency per request, LDS bank conflicts; and TA busy.
usage: python tools/contend_pmc.py gpurun_out/<tag> [envs]"""
import collections
import csv
import glob
import os
import sys


def load(d):
    acc, disp = collections.defaultdict(float), collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_step" not in r["Kernel_Name"]:
                continue
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r["Dispatch_Id"])
    return acc, {k: len(v) for k, v in disp.items()}


def main():
    root = sys.argv[1]
    envs = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    runs = {}
    for sl in ("s0", "s256"):
        acc, nd = load(os.path.join(root, sl))
        per = {}
        for k, v in acc.items():
            es = envs * nd[k]
            per[k] = v / nd[k] if k.endswith("_avr") else v / es
        if "TCP_TCC_READ_REQ_sum" in acc and acc["TCP_TCC_READ_REQ_sum"]:
            per["l2_read_latency_cycles"] = acc["TCP_TCC_READ_REQ_LATENCY_sum"] / acc["TCP_TCC_READ_REQ_sum"]
        if acc.get("SQC_ICACHE_REQ"):
            per["icache_miss_frac"] = acc["SQC_ICACHE_MISSES"] / acc["SQC_ICACHE_REQ"]
        if acc.get("TCC_HIT_sum", 0) + acc.get("TCC_MISS_sum", 0):
            per["l2_hit_frac"] = acc["TCC_HIT_sum"] / (acc["TCC_HIT_sum"] + acc["TCC_MISS_sum"])
        runs[sl] = per
    keys = sorted(set(runs["s0"]) | set(runs["s256"]))
    print("%-32s %16s %16s %8s" % ("per env-step (k_step)", "4 waves / CU", "1 wave / CU", "ratio"))
    for k in keys:
        a, b = runs["s0"].get(k), runs["s256"].get(k)
        r = (a / b) if a is not None and b else float("nan")
        print("%-32s %16.4g %16.4g %8.3f" % (k, a if a is not None else float("nan"), b if b is not None else float("nan"), r))


if __name__ == "__main__":
    main()
