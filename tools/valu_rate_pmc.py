#!/usr/bin/env python3
"""Per-kernel wave-instructions per SIMD per GRBM clock of tools/valu_rate.hip, from its
rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE pass (median over the
launches of each kernel).  GRBM_GUI_ACTIVE is summed over the 8 XCDs by rocprofv3.

  python tools/valu_rate_pmc.py run_counter_collection.csv [--simds 1024 --xcds 8]
"""
import argparse
import collections
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--simds", type=int, default=1024)
    ap.add_argument("--xcds", type=int, default=8)
    a = ap.parse_args()
    disp = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(a.csv)):
        d = r["Dispatch_Id"]
        disp[d][r["Counter_Name"]] += float(r["Counter_Value"])
        names[d] = r["Kernel_Name"].split("(")[0]
    per = collections.defaultdict(list)
    for d, c in disp.items():
        cyc = c["GRBM_GUI_ACTIVE"] / a.xcds
        per[names[d]].append(c["SQ_INSTS_VALU"] / (cyc * a.simds))
    for k, v in per.items():
        print(f"{k:12s} wave-instr/SIMD/clk {statistics.median(v):.4f}  cycles/instr "
              f"{1 / statistics.median(v):.2f}  (n={len(v)})")


if __name__ == "__main__":
    main()
