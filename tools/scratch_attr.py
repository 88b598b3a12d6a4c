#!/usr/bin/env python3
"""Attribution of k_step's vector-memory instructions (development aid): per __noinline__ function
of the product ISA, its static scratch / global / flat loads and stores, split into straight-line code (executed once
per call: the callee-saved saves and restores, the phase's own spills and its LDS-image / workspace accesses) and code
inside loops, times the calls per env-step the profiling build counts (tools/phase_prof.py "calls_per_env_step";
gjk_pair per GJK query).  The sum of the straight-line part is a lower bound on the dynamic count, which the PMC pass
measures directly (SQ_INSTS_VMEM_RD / _WR per wave = per env-step).
usage: python tools/scratch_attr.py isa.s phase.txt [pmc_counter_collection.csv [traffic_k_step.json]]
(isa.s: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -std=c++17 --cuda-device-only -S
 urgym_amd/csrc/ug_capi.hip)"""
import collections
import csv
import json
import re
import sys

MEM = re.compile(r"^\s*(scratch|global|flat)_(load|store)_(\w+)")
WIDTH = {"dword": 4, "dwordx2": 8, "dwordx3": 12, "dwordx4": 16, "ubyte": 1, "sbyte": 1, "byte": 1, "ushort": 2,
         "sshort": 2, "short": 2, "short_d16_hi": 2, "byte_d16_hi": 1}


def functions(lines):
    out, cur = [], None
    for i, l in enumerate(lines):
        m = re.match(r"^([_A-Za-z][\w.$]*):", l)
        if m and not l.startswith(".L"):
            cur = (m.group(1), i)
        if l.startswith(".Lfunc_end") and cur:
            out.append((cur[0], cur[1], i))
            cur = None
    return out


def loop_depth(body):
    labels = {}
    for j, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = j
    depth = [0] * len(body)
    for j, l in enumerate(body):
        m = re.search(r"s_(cbranch_\w+|branch)\s+(\.LBB\w+)", l)
        if m and m.group(2) in labels and labels[m.group(2)] < j:
            for k in range(labels[m.group(2)], j):
                depth[k] += 1
    return depth


def static_counts(path):
    lines = open(path).read().split("\n")
    res = {}
    for name, a, b in functions(lines):
        body = lines[a:b]
        depth = loop_depth(body)
        c = collections.Counter()
        for j, l in enumerate(body):
            m = MEM.match(l)
            if m:
                kind = "st" if m.group(2) == "store" else "ld"
                c[(m.group(1), kind, "loop" if depth[j] else "line")] += 1
                c[("bytes", kind, "loop" if depth[j] else "line")] += 64 * WIDTH.get(m.group(3), 4)
                if m.group(1) == "scratch":
                    c[("sbytes", kind, "loop" if depth[j] else "line")] += 64 * WIDTH.get(m.group(3), 4)
        res[name] = c
    return res


# the functions k_step runs (mangled prefixes; team_collide: the <full geometry, GJK> instance the default runs)
FUNCS = {"team_gjk": "_ZN3ugdL8team_gjkE", "gjk_pair": "_ZN3ugkL8gjk_pairE",
         "team_collide": "_ZN3ugdL12team_collideILb1ELb1EE", "glue": "_ZN3ugdL4glueE", "team_pgs": "_ZN3ugdL8team_pgsE",
         "team_unit_solves": "_ZN3ugdL16team_unit_solvesE", "serial_pre": "_ZN3ugdL10serial_preE",
         "serial_post": "_ZN3ugdL11serial_postE", "serial_fk": "_ZN3ugdL9serial_fkE",
         "team_robot_dynamics": "_ZN3ugdL19team_robot_dynamicsE", "team_enumerate": "_ZN3ugdL14team_enumerateE",
         "k_step": "_Z6k_step"}


def main():
    isa, phase = sys.argv[1], sys.argv[2]
    st = static_counts(isa)
    txt = open(phase).read()
    out = json.loads(txt[txt.index("{\n"):])
    calls = dict(out["calls_per_env_step"])
    calls["gjk_pair"] = out["gjk_per_substep"]["gjk_queries"] * out["substeps_per_env_step"]
    calls["k_step"] = 1.0
    rows, tot = [], collections.Counter()
    for fn, c in st.items():
        key = next((k for k, pre in FUNCS.items() if fn.startswith(pre)), None)
        if key is None or key not in calls:
            continue
        n = calls[key]
        ins = lambda k, w: sum(v for (s, kk, ww), v in c.items() if "bytes" not in s and kk == k and ww == w)
        ld, sto, ldl, stl = ins("ld", "line"), ins("st", "line"), ins("ld", "loop"), ins("st", "loop")
        scr = (c[("scratch", "ld", "line")], c[("scratch", "st", "line")])
        rows.append((key, n, ld, sto, ldl, stl, scr))
        tot["ld"] += n * ld
        tot["st"] += n * sto
        tot["scr_ld"] += n * scr[0]
        tot["scr_st"] += n * scr[1]
        tot["bytes_ld"] += n * c[("bytes", "ld", "line")]
        tot["bytes_st"] += n * c[("bytes", "st", "line")]
        tot["sbytes_ld"] += n * c[("sbytes", "ld", "line")]
        tot["sbytes_st"] += n * c[("sbytes", "st", "line")]
    print("%-22s %8s %7s %7s %7s %7s  %s" % ("function", "calls/es", "ld", "st", "ld(lp)", "st(lp)",
                                             "straight-line scratch ld/st"))
    for r in sorted(rows, key=lambda r: -(r[1] * (r[2] + r[3]))):
        print("%-22s %8.2f %7d %7d %7d %7d  %s" % r)
    print("straight-line, per env-step: loads %.0f (scratch %.0f), stores %.0f (scratch %.0f); bytes %.2f MB ld "
          "(scratch %.2f), %.2f MB st (scratch %.2f), full-wave widths"
          % (tot["ld"], tot["scr_ld"], tot["st"], tot["scr_st"], tot["bytes_ld"] / 1e6, tot["sbytes_ld"] / 1e6,
             tot["bytes_st"] / 1e6, tot["sbytes_st"] / 1e6))
    if len(sys.argv) > 3:
        acc, disp = collections.defaultdict(float), set()
        for r in csv.DictReader(open(sys.argv[3])):
            if "k_step" in r["Kernel_Name"]:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
                disp.add(r["Dispatch_Id"])
        waves = 4096 * len(disp)
        rd, wr = acc["SQ_INSTS_VMEM_RD"] / waves, acc["SQ_INSTS_VMEM_WR"] / waves
        print("PMC per env-step: loads %.0f, stores %.0f -> straight-line code accounts for %.0f %% / %.0f %% of the "
              "instructions" % (rd, wr, 100 * tot["ld"] / rd, 100 * tot["st"] / wr))
    if len(sys.argv) > 4:  # the FETCH_SIZE / WRITE_SIZE summary (tools/pmc_traffic.py)
        t = json.load(open(sys.argv[4]))
        r, w = t["read_bytes_per_launch"] / t["envs"], t["write_bytes_per_launch"] / t["envs"]
        print("HBM per env-step: %.2f MB read, %.2f MB written; the straight-line scratch accesses alone move %.2f / %.2f MB"
              % (r / 1e6, w / 1e6, tot["sbytes_ld"] / 1e6, tot["sbytes_st"] / 1e6))


if __name__ == "__main__":
    main()
