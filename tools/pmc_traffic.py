#!/usr/bin/env python3
"""Per-launch HBM traffic of each kernel from two rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE cannot share a pass on gfx950), corrected as MI355X_MICROARCH.md § HBM prescribes:
FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE counts half the bytes of wide reads, so
it is doubled.  The factor is checked here against kernels with known byte counts
(tools/traffic_calib.hip: coalesced reads count 0.5x at 4/16/48-B widths, coalesced writes 1x;
profiles/history/r02_traffic_calib.json).  Writes the JSON bench.py reads for
`roofline.traffic`.

  python tools/pmc_traffic.py FETCH.csv WRITE.csv OUT.json --workload NAME
         [--bench-log FETCH_PASS.log WRITE_PASS.log]
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
            if row["Counter_Name"] != counter:
                continue
            name = re.sub(r"\(.*", "", row["Kernel_Name"]).strip('"')
            vals[name].append(float(row["Counter_Value"]))
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
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("out_json")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--skip", type=int, default=1, help="warm-up launches to drop per kernel")
    ap.add_argument("--bench-log", nargs="*", default=[],
                    help="the bench.py output of each PMC pass: the build they measured")
    a = ap.parse_args()
    fetch = per_kernel(a.fetch_csv, "FETCH_SIZE")
    write = per_kernel(a.write_csv, "WRITE_SIZE")
    out = {"workload": a.workload,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                     "bytes = 2 x FETCH_SIZE KiB x 1024 + WRITE_SIZE KiB x 1024 (gfx950 "
                     "FETCH_SIZE correction, MI355X_MICROARCH.md § HBM)",
           "sources": [a.fetch_csv, a.write_csv], "kernels": {}}
    for name in sorted(set(fetch) | set(write)):
        f = fetch.get(name, [])[a.skip:] or fetch.get(name, [])
        w = write.get(name, [])[a.skip:] or write.get(name, [])
        fb = 2.0 * 1024.0 * sum(f) / len(f) if f else None
        wb = 1024.0 * sum(w) / len(w) if w else None
        out["kernels"][name] = {"launches": [len(f), len(w)],
                                "fetch_bytes": None if fb is None else round(fb),
                                "write_bytes": None if wb is None else round(wb),
                                "bytes": None if fb is None or wb is None else round(fb + wb)}
    out["build"] = build_of(a.bench_log)
    out["bench_logs"] = list(a.bench_log)
    with open(a.out_json, "w") as fo:
        json.dump(out, fo, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
