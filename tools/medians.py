#!/usr/bin/env python3
"""Median / min kernel_ms per labelled group of tools/frames.py JSON lines (stdin or file)."""
import json
import sys

cur = None
src = open(sys.argv[1]) if len(sys.argv) > 1 else sys.stdin


def show(c):
    if c and c[1]:
        v = sorted(c[1])
        print(f"{c[0]:24s} median {v[len(v) // 2]:.3f} min {v[0]:.3f} n {len(v)}")


for line in src:
    line = line.strip()
    if not line or "amdgpu.ids" in line:
        continue
    if line.startswith("{"):
        cur[1].append(json.loads(line)["kernel_ms"])
    else:
        show(cur)
        cur = (line, [])
show(cur)
