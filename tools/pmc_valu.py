#!/usr/bin/env python3
"""VALU issue utilisation of each kernel from a rocprofv3 SQ/GRBM PMC pass:

  valu_busy = SQ_INSTS_VALU x 2 cycles (a wave64 VALU instruction occupies a SIMD for two
              cycles on CDNA4, MI355X_MICROARCH.md) / (GRBM_GUI_ACTIVE per XCD x SIMDs)

  issue_frac = (SQ_INSTS_VALU / (cycles x SIMDs)) / 0.3888, the wave-instructions per SIMD
              per GRBM clock the chip sustains on independent v_fma_f32 streams with every SIMD
              full, measured in the same clock (tools/valu_rate.hip under the same PMC pass,
              profiles/history/r02_valu_rate_pmc.txt): how close the kernel is to the
              VALU issue rate actually reachable

  lane_utilisation = SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU), when the second pass
              holds both (the active lanes per VALU instruction; 0.998 on the C5 pool kernel,
              whose waves are full: DESIGN.md §4.7)

GRBM_GUI_ACTIVE is summed over the 8 XCDs by rocprofv3, so it is divided by 8 to get the
kernel's cycles.  Writes the JSON bench.py reads into roofline.valu_busy_pmc /
roofline.valu_issue_frac_pmc.

  python tools/pmc_valu.py SQ.csv GRBM.csv OUT.json --workload NAME [--simds 1024 --xcds 8]
         [--bench-log SQ_PASS.log GRBM_PASS.log]
"""
import argparse
import csv
import json
import re
from collections import defaultdict


def per_kernel(path, counter):
    vals = defaultdict(list)
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                vals[re.sub(r"\(.*", "", row["Kernel_Name"]).strip('"')].append(float(row["Counter_Value"]))
    return vals


def build_of(bench_logs):
    """The build the PMC passes measured: the `roofline.profile_binding.build` of the bench
    line each pass printed (bench.py, rvcp_internal_build_id + the specialised module's key);
    all passes must agree, else None (bench.py then treats the summary as stale)."""
    builds = []
    for path in bench_logs or []:
        lines = [l for l in open(path) if l.startswith("{")]
        if not lines:
            return None
        d = json.loads(lines[-1])
        builds.append(d.get("roofline", {}).get("profile_binding", {}).get("build"))
    if not builds or any(b != builds[0] for b in builds) or builds[0] is None:
        return None
    return builds[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sq_csv")
    ap.add_argument("grbm_csv")
    ap.add_argument("out_json")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--simds", type=int, default=1024)
    ap.add_argument("--xcds", type=int, default=8)
    ap.add_argument("--issue-peak", type=float, default=0.3888)
    ap.add_argument("--bench-log", nargs="*", default=[],
                    help="the bench.py output of each PMC pass: the build they measured")
    a = ap.parse_args()
    valu = per_kernel(a.sq_csv, "SQ_INSTS_VALU")
    grbm = per_kernel(a.grbm_csv, "GRBM_GUI_ACTIVE")
    thr = per_kernel(a.grbm_csv, "SQ_THREAD_CYCLES_VALU")
    act = per_kernel(a.grbm_csv, "SQ_ACTIVE_INST_VALU")
    out = {"workload": a.workload, "sources": [a.sq_csv, a.grbm_csv],
           "method": "SQ_INSTS_VALU x 2 / (GRBM_GUI_ACTIVE / xcds x simds), per launch; "
                     "issue_frac = SQ_INSTS_VALU / (cycles x simds) / measured issue peak",
           "issue_peak_per_simd_clk": a.issue_peak,
           "kernels": {}}
    for k in sorted(set(valu) & set(grbm)):
        v = sum(valu[k]) / len(valu[k])
        g = sum(grbm[k]) / len(grbm[k]) / a.xcds
        out["kernels"][k] = {"valu_insts": v, "cycles": g,
                             "valu_busy": round(2.0 * v / (g * a.simds), 4) if g else None,
                             "issue_frac": round(v / (g * a.simds) / a.issue_peak, 4) if g else None}
        if thr.get(k) and act.get(k) and sum(act[k]) > 0:
            out["kernels"][k]["lane_utilisation"] = round(sum(thr[k]) / (64.0 * sum(act[k])), 4)
    out["build"] = build_of(a.bench_log)
    out["bench_logs"] = list(a.bench_log)
    with open(a.out_json, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
