#!/usr/bin/env python3
"""Benchmark: Msamples/s of the path-tracing hot path (BASELINE.json metric), Cornell box.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c4|c5]

One step = one frame: every rank renders its 8-row stripes of the frame with the HIP kernel
(rvcp_render_shard_async), the stripes are gathered to rank 0 over RCCL (torch.distributed
'nccl' backend) and rank 0 assembles the frame on the device.  Scene and camera are uploaded
once, before timing (inputs resident in HBM).

Workloads (per BASELINE.json configs; the N=1 default is the headline C3):
  c3: Cornell 1024x1024 SPP=30.  For N>1 the frame grows with N at fixed SPP
      (side = round8(1024*sqrt(N))), so per-GPU work stays ~C3: "scaling": "weak".
  c1: Cornell 128x128 SPP=1 (BASELINE configs[0], the CPU plumbing case; its cpu_baseline is
      the whole frame).
  c2: Cornell 384x384 SPP=10 (README benchmark row).
  c4: Cornell 2048x2048 SPP=64, fixed frame sharded over N GPUs ("scaling": "strong").
  c5: Cornell + 100k random triangles, 1024x1024 SPP=30.
  spheres: integrator mode 2 (ray_tracer.comp) on the deprecated host's sphere room,
      1024x1024 at its SPP=5 (not a BASELINE config; reported for coverage).

Rank 0 prints ONE JSON line.  `roofline` is for the dominant kernel (the path-tracing kernel,
>99% of the frame's GPU time): algorithmic bytes = its reference-algorithm traversals x F x
36 B per launch (the primary rays the pre-pass traces once are the only
traversals not attributed to it) over its HIP-event time (rvcp_stats_t.main_kernel_ms,
events on the launch stream).  `traffic` is the same kernel's measured HBM bytes per launch
from the rocprofv3 PMC summary committed under profiles/ (tools/pmc_traffic.py), when one
exists for the workload; `valu_busy_pmc` / `valu_issue_frac_pmc` are that kernel's VALU issue
utilisation from the committed SQ counter passes (tools/pmc_valu.py: at 2 cycles per wave64
instruction, and as a fraction of the issue rate tools/valu_rate.hip measures) -- the bound
that actually limits this FP32 kernel.  `cpu_baseline` times the scalar C oracle (oracle/rvcp_oracle.c, the
CPU re-execution of the same kernel) on a bounded sample of the workload, rank 0 at N=1 only.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
# the reference's published C3 row (README.md:26, 3 fps on an RTX 3060) and
# C2 row (README.md:22, 51 fps), as Msamples/s
REFERENCE_MSAMPLES = {"c3": 94.4, "c2": 75.2}
FP32_PEAK_TFLOPS = 157.3       # MI355X FP32 vector peak (spec)
FLOP_PER_TEST = 52


def workload(name, n_gpus):
    if name == "c3":
        side = 1024 if n_gpus == 1 else int(round(1024 * math.sqrt(n_gpus) / 8.0)) * 8
        return dict(workload="cornell_1024sq_spp30" if n_gpus == 1 else
                    f"cornell_{side}sq_spp30_weak", W=side, H=side, spp=30, extra_tris=0,
                    scaling="weak")
    if name == "c1":
        return dict(workload="cornell_128sq_spp1", W=128, H=128, spp=1, extra_tris=0,
                    scaling="strong")
    if name == "c2":
        return dict(workload="cornell_384sq_spp10", W=384, H=384, spp=10, extra_tris=0,
                    scaling="strong")
    if name == "c4":
        return dict(workload="cornell_2048sq_spp64", W=2048, H=2048, spp=64, extra_tris=0,
                    scaling="strong")
    if name == "c5":
        return dict(workload="cornell_plus_100k_tris_1024sq_spp30", W=1024, H=1024, spp=30,
                    extra_tris=100000, scaling="strong")
    if name == "spheres":
        return dict(workload="spheres_mode2_1024sq_spp5", W=1024, H=1024, spp=5, extra_tris=0,
                    scaling="strong", integrator=1)
    raise SystemExit(f"unknown workload {name}")


def load_valu_busy(workload_name, kernel_substr):
    """VALU issue utilisation of the dominant kernel from the newest committed SQ PMC summary:
    (busy at 2 cycles per wave64 instruction, fraction of the measured issue peak)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_valu_{workload_name}.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    for name, k in d.get("kernels", {}).items():
        if kernel_substr in name:
            return k.get("valu_busy"), k.get("issue_frac")
    return None, None


def load_traffic(workload_name, kernel_substr):
    """HBM bytes per launch of the dominant kernel from the newest committed PMC summary."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_traffic_{workload_name}.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    for name, k in d.get("kernels", {}).items():
        if kernel_substr in name and k.get("bytes"):
            return float(k["bytes"]), os.path.relpath(files[-1], ROOT)
    return None, None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(sc, cfg_kw, W, H, threads):
    """Time the CPU oracle (scalar C re-execution) on a bounded sample of the workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import rvcp_amd
    O.build()
    cfg = rvcp_amd.abi.make_config(**cfg_kw)
    arrays = dict(materials=sc.aligned_materials(), vertices=sc.mesh.aligned_vertices(),
                  faces=sc.mesh.aligned_faces(), lum_face_ids=sc.luminous_face_ids(),
                  spheres=sc.aligned_spheres())
    push = sc.push_constant(123.0)
    rows = list(range(0, H, 8))
    O.render(arrays, push, cfg, W, H, rect=(0, H // 2, min(W, 64), 1), threads=threads,
             want_linear=False)                                   # warm-up (page-in, threads)
    if len(arrays["faces"]) > 1000:          # C5 on CPU: 128^2 SPP=1 frame only
        t0 = time.perf_counter()
        O.render(arrays, push, rvcp_amd.abi.make_config(**dict(cfg_kw, spp=1)), 128, 128,
                 threads=threads, want_linear=False)
        dt = time.perf_counter() - t0
        return dict(value=128 * 128 / dt / 1e6, unit="Msamples/s", cores=threads, kind="port",
                    sample="128x128 SPP=1 frame of the same scene", seconds=round(dt, 3),
                    cpu=cpu_model())
    # the whole frame on `threads` threads (a few seconds), then a single-thread figure on
    # every 64th row
    t0 = time.perf_counter()
    O.render(arrays, push, cfg, W, H, threads=threads, want_linear=False)
    dt = time.perf_counter() - t0
    samples = W * H * cfg_kw["spp"]
    rows1 = list(range(0, H, 64 if H >= 256 else 8))
    t1 = time.perf_counter()
    for y in rows1:
        O.render(arrays, push, cfg, W, H, rect=(0, y, W, 1), threads=1, want_linear=False)
    dt1 = time.perf_counter() - t1
    return dict(value=samples / dt / 1e6, unit="Msamples/s", cores=threads, kind="port",
                sample=f"the full {W}x{H} SPP={cfg_kw['spp']} frame on {threads} threads",
                seconds=round(dt, 3),
                single_thread_value=round(len(rows1) * W * cfg_kw["spp"] / dt1 / 1e6, 4),
                single_thread_sample=f"every {64 if H >= 256 else 8}th row ({len(rows1)} rows), 1 thread",
                single_thread_seconds=round(dt1, 3), cpu=cpu_model())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c3", choices=["c1", "c2", "c3", "c4", "c5", "spheres"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "0") or 0))
    ap.add_argument("--save-frame", default="")
    ap.add_argument("--accel", default="none", choices=["none", "bvh"],
                    help="bvh: the opt-in BVH (not the parity path; never the default line)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import rvcp_amd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run")
    # Rehearsal (RVCP_BENCH_REHEARSAL=1): every rank on device 0 and a gloo gather through host
    # memory, to exercise the N>1 code path on a 1-GPU box.  Never used for reported numbers.
    rehearsal = os.environ.get("RVCP_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local_rank = 0
    torch.cuda.set_device(local_rank)
    if world > 1:
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    wl = workload(args.workload, world)
    W, H, spp = wl["W"], wl["H"], wl["spp"]
    legacy = wl.get("integrator", 0) == 1
    sc = rvcp_amd.scene.sphere_scene() if legacy else rvcp_amd.Scene.default()
    if wl["extra_tris"]:
        sc = rvcp_amd.scene.with_random_triangles(sc, wl["extra_tris"])
    cfg_kw = dict(spp=spp, device=local_rank)
    if legacy:
        cfg_kw["integrator"] = 1
    if args.accel == "bvh":
        cfg_kw["accel"] = 1
    rt = rvcp_amd.RayTracer(**cfg_kw)
    rt.upload_scene(sc)
    push = sc.push_constant(123.0)
    n_faces = len(sc.mesh.aligned_faces())
    n_spheres = len(sc.spheres) if legacy else 0

    rows = rvcp_amd.shard_rows(H, rank, world)
    slot = max(rvcp_amd.shard_rows(H, k, world) for k in range(world))
    dev = torch.device("cuda", local_rank)
    shard_buf = torch.zeros((slot, W), dtype=torch.int32, device=dev)
    frame = torch.zeros((H, W), dtype=torch.int32, device=dev) if rank == 0 else None
    gat_flat = torch.zeros((world, slot, W), dtype=torch.int32, device=dev) if (world > 1 and rank == 0) else None
    stream = torch.cuda.current_stream().cuda_stream

    def step():
        if world == 1:
            rt.render_shard_async(push, W, H, 0, 1, frame.data_ptr(), stream=stream)
            st = rt.sync_stats()
            return st
        rt.render_shard_async(push, W, H, rank, world, shard_buf.data_ptr(), stream=stream)
        st = rt.sync_stats()
        if rehearsal:
            got = rvcp_amd.frame.gather_shards(shard_buf.cpu(), rank, world, dst=0)
            if rank == 0:
                gat_flat.copy_(torch.stack(got))
        else:
            rvcp_amd.frame.gather_shards(shard_buf, rank, world, dst=0, out=gat_flat)   # RCCL
        if rank == 0:
            rt.assemble_frame_async(gat_flat.data_ptr(), slot, W, H, world, frame.data_ptr(),
                                    stream=stream)
        return st

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    kernel_ms, main_ms, trav, trav_exec = [], [], 0, 0
    t0 = time.perf_counter()
    step_ms = []
    for _ in range(args.steps):
        ts = time.perf_counter()
        st = step()
        step_ms.append((time.perf_counter() - ts) * 1000.0)
        kernel_ms.append(float(st["kernel_ms"]))
        main_ms.append(float(st["main_kernel_ms"]))
        trav += int(st["traversals"])
        trav_exec += int(st["traversals_executed"])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if rehearsal else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    samples_total = W * H * spp * args.steps
    value = samples_total / elapsed / 1e6
    ms_per_step = elapsed * 1000.0 / args.steps

    # roofline for the dominant kernel (this rank's launches).  The pre-pass (variants 3/4,
    # games101 only) traces each pixel's primary ray once; every other reference-algorithm
    # traversal -- including the reused primary hits of samples 2..SPP -- belongs to the
    # path kernel.
    avg_frame_s = (sum(kernel_ms) / len(kernel_ms)) / 1000.0
    avg_kernel_s = (sum(main_ms) / len(main_ms)) / 1000.0
    prepass = 0 if legacy else rows * W
    units = trav / args.steps - prepass                     # traversals per path-kernel launch
    # a traversal tests F triangles (36 B each) and, in mode 2, S spheres (16 B each)
    bytes_per_launch = units * (n_faces * 36 + n_spheres * 16)
    achieved_gbs = bytes_per_launch / avg_kernel_s / 1e9
    tests_per_s = units * (n_faces + n_spheres) / avg_kernel_s
    exec_tests_per_s = (trav_exec / args.steps - prepass) * (n_faces + n_spheres) / avg_kernel_s
    kname = ("legacy_kernel" if legacy else "games101_bvh_path_kernel" if args.accel == "bvh"
             else "games101_tiled_single_kernel" if n_faces >= 256 else "games101_path_kernel")
    traffic, traffic_src = load_traffic(wl["workload"], kname)
    valu_busy, valu_issue_frac = load_valu_busy(wl["workload"], kname)

    frame_check = None
    if world > 1 and rank == 0:
        # the assembled N-rank frame must be bit-identical to a 1-rank render (outside timing)
        single = torch.zeros((H, W), dtype=torch.int32, device=dev)
        rt.render_shard_async(push, W, H, 0, 1, single.data_ptr(), stream=stream)
        rt.sync_stats()
        torch.cuda.synchronize()
        frame_check = bool(torch.equal(single, frame))

    if args.save_frame and rank == 0:
        np.save(args.save_frame, frame.cpu().numpy().view(np.uint8).reshape(H, W, 4))

    if rank == 0:
        out = {
            "metric": "Msamples/sec (pixels*SPP/s) + frame ms, Cornell Box 1024^2 SPP=30",
            "value": round(value, 2),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "fps": round(1000.0 / ms_per_step, 2),
            "frame_ms_median": round(float(np.median(step_ms)), 4),
            "higher_is_better": True,
            "scaling": wl["scaling"],
            "vs_baseline": (round(value / REFERENCE_MSAMPLES[args.workload], 2)
                            if args.workload in REFERENCE_MSAMPLES else None),
            "dtype": "f32",
            "data": ("synthetic (the reference's deprecated sphere-room scene, integrator mode 2, "
                     "fixed time seed 123.0)" if legacy else
                     "synthetic (the reference's built-in Cornell box scene, fixed time seed 123.0)"),
            "config": {"workload": wl["workload"], "width": W, "height": H, "spp": spp,
                       "faces": n_faces, "parallelism": f"pixel-stripes x{world}",
                       "accel": args.accel,
                       "gather": ("gloo-rehearsal" if rehearsal else "rccl") if world > 1 else "none"},
            "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                         "traffic": None if traffic is None else round(traffic),
                         "traffic_source": traffic_src,
                         "kernel": kname,
                         "kernel_ms": round(avg_kernel_s * 1000.0, 4),
                         "frame_kernels_ms": round(avg_frame_s * 1000.0, 4),
                         "algorithmic_bytes_per_launch": round(bytes_per_launch),
                         "definition": "reference-algorithm traversals of the path kernel x "
                                       "(F x 36 B + S x 16 B) per launch / its HIP-event time "
                                       "(SURVEY.md §8(d))",
                         "traversals_per_sample": round(trav / args.steps / (W * H * spp / world), 4)
                         if world == 1 else None,
                         "executed_traversal_frac": round(trav_exec / max(trav, 1), 4),
                         "valu_tflops": round(tests_per_s * FLOP_PER_TEST / 1e12, 2),
                         "valu_frac": round(tests_per_s * FLOP_PER_TEST / 1e12 / FP32_PEAK_TFLOPS, 4),
                         "valu_busy_pmc": valu_busy,
                         "valu_issue_frac_pmc": valu_issue_frac,
                         "executed_tests_per_s": round(exec_tests_per_s, 1)},
            "cpu_baseline": None,
        }
        if frame_check is not None:
            out["config"]["assembled_frame_bitexact_vs_1gpu"] = frame_check
        if world == 1 and not args.no_cpu_baseline:
            threads = args.cpu_threads or min(16, os.cpu_count() or 1)
            out["cpu_baseline"] = cpu_baseline(sc, cfg_kw, W, H, threads)
        print(json.dumps(out), flush=True)

    rt.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
