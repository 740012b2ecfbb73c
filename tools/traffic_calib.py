#!/usr/bin/env python3
"""Summarise tools/traffic_calib under rocprofv3: counter bytes / known bytes per kernel.

  python tools/traffic_calib.py FETCH.csv WRITE.csv [OUT.json]

FETCH_SIZE and WRITE_SIZE are KiB per dispatch (rocprofv3); the known byte counts are the
1-GiB buffers of tools/traffic_calib.hip (rec48: 22369621 records x 48 B).  The ratios are
the correction factors DESIGN.md §4.3 applies (tools/pmc_traffic.py)."""
import csv
import json
import re
import sys
from collections import defaultdict

KNOWN = {"read16": 1 << 30, "read4": 1 << 30, "rec48": (1 << 30) // 48 * 48,
         "write16": 1 << 30, "write4": 1 << 30, "scat4": 1 << 30}


def load(path, counter):
    v = defaultdict(list)
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                v[re.sub(r"\(.*", "", row["Kernel_Name"]).strip('"')].append(float(row["Counter_Value"]))
    return v


def main():
    fetch, write = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k, b in KNOWN.items():
        f = [x * 1024.0 / b for x in fetch.get(k, [])]
        w = [x * 1024.0 / b for x in write.get(k, [])]
        out[k] = {"known_bytes": b, "fetch_size_over_known": [round(x, 4) for x in f],
                  "write_size_over_known": [round(x, 4) for x in w]}
        print(f"{k:8s} FETCH_SIZE/known {['%.3f' % x for x in f]}  WRITE_SIZE/known {['%.3f' % x for x in w]}")
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as fo:
            json.dump(out, fo, indent=1)


if __name__ == "__main__":
    main()
