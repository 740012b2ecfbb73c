#!/usr/bin/env python3
"""Per-kernel averages of every counter in gpurun_out/pmc_<name>_*/run_counter_collection.csv."""
import csv, collections, glob, re, sys
name = sys.argv[1]
d = collections.defaultdict(list)
for f in sorted(glob.glob(f"gpurun_out/pmc_{name}_*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"])[:60]
        d[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(d.items()):
    if "rvcp" in k:
        print(f"{k:50s} {c:32s} {sum(v)/len(v):.4g}")
