"""Summarise the tools/gpu.sh pmcmix passes: per counter, the average over k_step launches and per wave (4096 waves per
launch at the default bench size).  usage: python tools/pmc_mix_summary.py <pmc_mix outdir> <out.csv> [waves]"""
import collections
import csv
import glob
import sys

out_dir, out_csv = sys.argv[1], sys.argv[2]
waves = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
tot = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in sorted(glob.glob(out_dir + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if not r["Kernel_Name"].startswith("k_step"):
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
with open(out_csv, "w") as fo:
    fo.write("counter,avg_per_k_step_launch,per_wave\n")
    for k in sorted(tot):
        avg = tot[k] / len(disp[k])
        fo.write(f"{k},{avg:.1f},{avg / waves:.1f}\n")
print(open(out_csv).read())
