#!/usr/bin/env python3
"""Same-box A/B driver: every measurement of a variant against another runs through this.

A case is `label=ENV=v,ENV2=w::runner args`: the environment it runs with (RVCP_LIB to pick a
library build -- tools/build_variant.sh builds variants, the debug build holds the
experiment knobs; RVCP_JIT_FLAGS for hipRTC -D options of the specialised module), and the
arguments of the runner.  Cases run interleaved, pass after pass, each under its own time
limit; one line per (pass, case), then the median per case.

Runners:
  bench     python bench.py --no-cpu-baseline --launch-pass 0 --interactive-pass 0 --steps 40
            --warmup 5 ARGS
            (ms_per_step, the driver's figure: frames in flight and batches as the bench
            picks them unless ARGS fix them; --field picks another key of the line, e.g.
            config.frame_latency_ms_alone with ARGS --launch-pass 40)
  frames    python tools/frames.py --frames 20 ARGS  (one frame at a time, path-kernel ms:
            median of the frames after the first 3)
  share     python tools/rank_share.py ARGS  (rank 0's share of the N-GPU C4 frame alone)

  python tools/ab.py --runner bench --passes 2 \\
      "base=::--workload c3" "v2=RVCP_LIB=tools/build/var_v2/librvcp.so::--workload c3"
  python tools/ab.py --runner frames "s3=::--variant 3" "s10=::--variant 10 --tris 2000"
  python tools/ab.py --cases-file tools/ab_cases/c3_lib.txt      (one case per line)
"""
import argparse
import json
import os
import shlex
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUNNERS = {
    "bench": [sys.executable, "bench.py", "--no-cpu-baseline", "--launch-pass", "0",
              "--interactive-pass", "0", "--steps", "40", "--warmup", "5"],
    "frames": [sys.executable, "tools/frames.py", "--frames", "20"],
    "share": [sys.executable, "-u", "tools/rank_share.py"],
}


def stale_macros(env):
    """-D macros a case passes to hipRTC (RVCP_JIT_FLAGS) that no kernel source names any more:
    re-running such a case would build the same module under another label."""
    import re
    names = re.findall(r"-D\s*([A-Za-z_][A-Za-z0-9_]*)", env.get("RVCP_JIT_FLAGS", ""))
    csrc = os.path.join(ROOT, "rvcp-real-time-path-tracer_amd", "csrc")
    text = "".join(open(os.path.join(csrc, f)).read() for f in os.listdir(csrc)
                   if f.endswith((".hip", ".h", ".cpp")))
    return [n for n in names if n not in text]


def parse_case(text):
    label, _, rest = text.partition("=")
    envs, _, args = rest.partition("::")
    env = {}
    for kv in filter(None, envs.split(",")):
        k, _, v = kv.partition("=")
        env[k] = v
    return label, env, shlex.split(args)


def measure(runner, out, field="ms_per_step"):
    """The case's figure from the runner's stdout (ms); `field`: the bench line's key, dotted
    for nested ones (config.frame_latency_ms_alone)."""
    lines = [l for l in out.splitlines() if l.startswith("{")]
    if runner == "bench":
        v = json.loads(lines[-1])
        for k in field.split("."):
            v = v[k]
        return v
    if runner == "frames":
        ms = sorted(json.loads(l)["kernel_ms"] for l in lines[3:] or lines)
        return ms[len(ms) // 2]
    vals = [json.loads(l).get("ms_per_frame") for l in lines]
    return [v for v in vals if v is not None][-1]


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--runner", choices=sorted(RUNNERS), default="bench")
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--timeout", type=int, default=200)
    ap.add_argument("--field", default="ms_per_step",
                    help="bench runner: the figure to compare (several: comma-separated, the first "
                         "one the headline of each line)")
    ap.add_argument("--cases-file", help="cases one per line (# comments), after the positional ones; "
                    "$DBG is the debug library")
    ap.add_argument("cases", nargs="*")
    a = ap.parse_args()
    texts = list(a.cases)
    if a.cases_file:
        dbg = "rvcp-real-time-path-tracer_amd/csrc/build/librvcp_debug.so"
        for line in open(os.path.join(ROOT, a.cases_file)):
            line = line.strip()
            if line and not line.startswith("#"):
                texts.append(line.replace("$DBG", dbg))
    if not texts:
        ap.error("no cases")
    cases = [parse_case(c) for c in texts]
    for label, env, _ in cases:
        stale = stale_macros(env)
        if stale:
            sys.exit(f"case {label}: {', '.join(stale)} no longer exist in the kernel sources -- a "
                     "historical case file, not re-runnable (it would measure noise as an effect)")
    fields = a.field.split(",") if a.runner == "bench" else [a.field]
    got = {label: [] for label, _, _ in cases}
    extra = {(label, f): [] for label, _, _ in cases for f in fields[1:]}
    for p in range(1, a.passes + 1):
        for label, env, args in cases:
            cmd = ["timeout", "-k", "10", str(a.timeout)] + RUNNERS[a.runner] + args
            r = subprocess.run(cmd, cwd=ROOT, env=dict(os.environ, **env), capture_output=True,
                               text=True)
            if r.returncode != 0:
                print(f"pass {p} {label:>24}  FAILED rc={r.returncode}: {r.stderr[-400:]}", flush=True)
                if r.returncode >= 124:      # time limit / signal: stop here
                    sys.exit(r.returncode)
                continue
            v = measure(a.runner, r.stdout, fields[0])
            got[label].append(v)
            more = ""
            for f in fields[1:]:
                x = measure(a.runner, r.stdout, f)
                extra[(label, f)].append(x)
                more += f"  {f}={x:.4f}"
            print(f"pass {p} {label:>24}  {v:.4f} ms{more}", flush=True)
    for label, vals in got.items():
        if vals:
            print(f"median {label:>24}  {statistics.median(vals):.4f} ms  (n={len(vals)}, "
                  f"min {min(vals):.4f})", flush=True)
            for f in fields[1:]:
                xs = extra[(label, f)]
                print(f"median {label:>24}  {f} {statistics.median(xs):.4f}  (min {min(xs):.4f})",
                      flush=True)


if __name__ == "__main__":
    main()
