#!/usr/bin/env python3
"""Benchmark: Msamples/s of the path-tracing hot path (BASELINE.json metric), Cornell box.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c4|c5|...]

`--gpus N` (N > 1) without a launcher starts its N ranks itself (torch.distributed.run on
127.0.0.1, see self_launch); under torch.distributed.run it is one rank.

One step = one frame, each with its own time seed (123.0 + frame index, as the reference
re-stamps `time` every frame): every rank renders its 8-row stripes of the frame with the HIP kernel
(rvcp_render_shard_async), the stripes are gathered to rank 0 over RCCL
(rvcp_gather_frame_async: ncclGather inside librvcp) and rank 0 assembles the frame on the
device.  Two frames are in flight (--frames-in-flight, default 2): two contexts, each on its
own stream, render consecutive frames, so a frame's start overlaps the previous frame's tail
(DESIGN.md §4.8); every step still renders its whole frame.  Scene and camera are uploaded
once, before timing (inputs resident in HBM).

Workloads (per BASELINE.json configs; the N=1 default is the headline C3):
  c3: Cornell 1024x1024 SPP=30 (the N=1 default).  With --workload c3 at N>1 the frame
      grows with N at fixed SPP (side = round8(1024*sqrt(N))): "scaling": "weak".
  c1: Cornell 128x128 SPP=1 (BASELINE configs[0], the CPU plumbing case; its cpu_baseline is
      the whole frame).
  c2: Cornell 384x384 SPP=10 (README benchmark row).
  c4: Cornell 2048x2048 SPP=64, fixed frame sharded over N GPUs ("scaling": "strong"): the
      BASELINE.json 8-GPU config and the default for N>1.  Rank 0 also renders the same frame
      alone after the timed region (bit-exactness check, and `one_gpu_ms` for the speedup).
  c5: Cornell + 100k random triangles, 1024x1024 SPP=30.
  c6: Cornell + 310 random triangles (342 faces, 998 vertices: the largest unshared-vertex
      scene within the reference's own 1000-vertex / 1000-face buffers,
      ray_tracer_games101_branch.comp:18-19), 1024x1024 SPP=30.
  spheres: integrator mode 2 (ray_tracer.comp) on the deprecated host's sphere room,
      1024x1024 at its SPP=5 (not a BASELINE config; reported for coverage).
  c3m2: the C3 frame (Cornell 1024x1024 SPP=30) through integrator mode 2 (ray_tracer.comp,
      the shader north_star names) instead of the games101 branch the current host binds.
  c3rot: the C3 frame of the Cornell box turned off-axis with its camera (scene.rotated_scene):
      no exact-zero triangle component is left for the scene-specialised scan to drop.
  c3gen: the C3 frame with the generic scan (rvcp_config_t.specialize = OFF).

Rank 0 prints ONE JSON line.  `roofline` is for the dominant kernel (the path-tracing kernel,
>99% of the frame's GPU time), whose bound is FP32 VALU issue:
  * `achieved` / `frac`: useful FLOP per frame (52 per reference-algorithm ray-triangle test,
    25 per ray-sphere test) / `ms_per_step` (the driver-comparable wall time
    per frame) / `peak` = 157.3 TFLOP/s FP32 vector;
  * `frac_executed`: the same with the traversals the kernels execute (the primary hit is
    traced once per pixel, not once per sample);
  * `per_launch`: useful FLOP / the path kernel's HIP-event time with ONE frame in flight, from
    a short pass after the timed region (with frames in flight a launch's event time includes
    the other frame's work); the rocprofv3 summary of the same command is committed under
    profiles/ and must agree;
  * `valu_issue_frac_pmc_guide`: VALU wave-instructions per SIMD-cycle from the committed SQ
    counter passes (tools/pmc_valu.py) over the guide's 0.5 (2 cycles per wave64 instruction);
    `valu_issue_frac_wall`: that pass's instructions per frame over the issue slots of
    `ms_per_step` at `shader_clock_ghz`, the clock THIS run's path kernel measured on itself
    (per-wave s_memtime / s_memrealtime stamps);
  * `traffic`: the kernel's measured HBM bytes per launch (rocprofv3 PMC, tools/pmc_traffic.py);
    `hbm_algorithmic`: SURVEY.md §8(d)'s HBM-read figure (36 algorithmic bytes per triangle
    test), which exceeds the HBM peak because the scene is served on-chip.
  With --accel bvh the work is not the brute-force scan's, so `frac` is null (the traversal is
  bound by dependent node loads).
`cpu_baseline` times the scalar C port of the shader (oracle/rvcp_oracle.c; the image has no
Rust toolchain for a Rust re-execution) on the CPUs this process is granted (the cgroup quota,
16 per GPU on the box; `cores`), with one thread timed beside it, rank 0 at N=1 only.
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
FLOP_PER_SPHERE_TEST = 25      # ray_tracer.comp:300-321
# the reference's published C3 row (README.md:26, 3 fps on an RTX 3060) and
# C2 row (README.md:22, 51 fps), as Msamples/s
REFERENCE_MSAMPLES = {"c3": 94.4, "c2": 75.2}
FP32_PEAK_TFLOPS = 157.3       # MI355X FP32 vector peak (spec)
# VALU issue: 1,024 SIMDs (256 CUs x 4) issuing one wave64 instruction per 2 cycles
# (MI355X_MICROARCH.md) at the shader clock this run measured (the path kernel's own per-wave
# s_memtime / s_memrealtime stamps, rvcp_stats_t.shader_clock_ghz)
N_SIMDS = 1024
VALU_ISSUE_PER_CLK = 0.5
FLOP_PER_TEST = 52
C6_EXTRA_TRIS = 310            # Cornell + 310 = 342 faces, 998 vertices (workload c6)
# the time seed of frame 0 (the tests' fixed seed); frame f renders with
# TIME0 + f, as the reference re-stamps `time` every frame (vulkan.rs:418-421)
TIME0 = 123.0


BASELINE_METRIC = "Msamples/sec (pixels*SPP/s) + frame ms, Cornell Box 1024^2 SPP=30"


def metric_name(wl, world):
    """BASELINE.json's metric for the headline (C3 on one GPU); other workloads name their own
    frame, and N > 1 names the GPU count the frame is sharded over."""
    if wl["workload"] == "cornell_1024sq_spp30" and world == 1:
        return BASELINE_METRIC
    what = f"{wl['W']}^2 SPP={wl['spp']}, {wl['workload']}"
    if world > 1:
        what += (f", frame sharded over {world} GPUs" if wl["scaling"] == "strong" else
                 f", {world} GPUs (weak scaling)")
    return f"Msamples/sec (pixels*SPP/s) + frame ms, {what}"


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
    if name == "c6":
        # the largest unshared-vertex scene the reference itself can load: its shader caps the
        # buffers at 1000 vertices and 1000 faces (ray_tracer_games101_branch.comp:18-19), so
        # Cornell (68 vertices) + 310 random triangles (930) = 998 vertices, 342 faces
        return dict(workload="cornell_plus_310_tris_1024sq_spp30", W=1024, H=1024, spp=30,
                    extra_tris=C6_EXTRA_TRIS, scaling="strong")
    if name == "spheres":
        return dict(workload="spheres_mode2_1024sq_spp5", W=1024, H=1024, spp=5, extra_tris=0,
                    scaling="strong", integrator=1, scene="spheres")
    if name == "c3rot":
        return dict(workload="cornell_rotated_1024sq_spp30", W=1024, H=1024, spp=30, extra_tris=0,
                    scaling="strong", rotate=True)
    if name == "c3gen":
        return dict(workload="cornell_generic_scan_1024sq_spp30", W=1024, H=1024, spp=30,
                    extra_tris=0, scaling="strong", specialize_off=True)
    if name == "c3m2":
        return dict(workload="cornell_mode2_1024sq_spp30", W=1024, H=1024, spp=30, extra_tris=0,
                    scaling="strong", integrator=1, scene="cornell")
    raise SystemExit(f"unknown workload {name}")


def profile_summary(kind, workload_name, kernel_name):
    """The newest committed PMC summary of `kind` ("valu": tools/pmc_valu.py, "traffic":
    tools/pmc_traffic.py) for the workload: (the dominant kernel's record or None, the file
    relative to the repo or None, the build it measured -- {"source", "module"} from the PMC
    pass's own bench line, tools/pmc_*.py --bench-log -- or None for a summary without one)."""
    import glob
    # profiles/ holds this round's summaries, profiles/history/ the earlier rounds'; the tag
    # (r01 ... r06...) sorts by round, so the newest is the last by file name
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{kind}_{workload_name}.json")) +
                   glob.glob(os.path.join(ROOT, "profiles", "history", f"*_{kind}_{workload_name}.json")),
                   key=os.path.basename)
    if not files:
        return None, None, None
    with open(files[-1]) as f:
        d = json.load(f)
    rec = next((k for name, k in d.get("kernels", {}).items() if kernel_name in name), None)
    return rec, os.path.relpath(files[-1], ROOT), d.get("build")


def load_valu_busy(workload_name, kernel_name, want_insts=False):
    """VALU issue utilisation of the dominant kernel from the newest committed SQ PMC summary:
    (busy at 2 cycles per wave64 instruction, fraction of the measured issue peak), and with
    want_insts also (wave64 VALU instructions per launch, summary file).  Whatever build the
    summary measured (bench.py checks that with profile_summary's build)."""
    k, src, _ = profile_summary("valu", workload_name, kernel_name)
    if k is None:
        return (None, None, None, None) if want_insts else (None, None)
    if want_insts:
        return k.get("valu_busy"), k.get("issue_frac"), k.get("valu_insts"), src
    return k.get("valu_busy"), k.get("issue_frac")


def load_traffic(workload_name, kernel_name):
    """HBM bytes per launch of the dominant kernel from the newest committed PMC summary."""
    k, src, _ = profile_summary("traffic", workload_name, kernel_name)
    if k is None or not k.get("bytes"):
        return None, None
    return float(k["bytes"]), src


def build_identity(rt):
    """What this run executes: the library's source identity (SHA-256 prefix of the sources it
    was built from, rvcp_internal_build_id) and the key of rt's scene-specialised module
    (hipRTC version, options, embedded sources and generated scan; None when the generic
    kernels run).  PMC-derived roofline fields are reported only from a summary of this same
    build."""
    import ctypes
    L = rvcp_amd_abi().load()
    L.rvcp_internal_build_id.restype = ctypes.c_char_p
    L.rvcp_internal_module_key.restype = ctypes.c_uint64
    L.rvcp_internal_module_key.argtypes = [ctypes.c_void_p]
    key = int(L.rvcp_internal_module_key(rt.handle))
    return {"source": L.rvcp_internal_build_id().decode(), "module": f"{key:016x}" if key else None}


def rvcp_amd_abi():
    import rvcp_amd
    return rvcp_amd.abi


def bound_profile(kind, workload_name, kernel_name, build):
    """profile_summary's record when it measured `build`, else None; and the binding record the
    line carries: {source file, its build, match}."""
    rec, src, pbuild = profile_summary(kind, workload_name, kernel_name)
    match = None if rec is None else (pbuild is not None and pbuild == build)
    return (rec if match else None), {"source": src, "build": pbuild, "build_match": match}


def vs_baseline_loop_shape(wname, world, samples_per_frame, interactive_ms):
    """vs_baseline on the reference's own loop shape: the interactive pass's Msamples/s (one
    frame per launch, pushes stamped at submission, at most 3 in flight) over the reference's
    published Msamples/s for the same frame; None without a published row or without the pass."""
    if world != 1 or wname not in REFERENCE_MSAMPLES or not interactive_ms:
        return None
    return round(samples_per_frame / (interactive_ms / 1000.0) / 1e6 / REFERENCE_MSAMPLES[wname], 2)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def host_threads():
    """Hardware threads this process may run on (the whole host)."""
    try:
        return len(os.sched_getaffinity(0)) or 1
    except AttributeError:
        return os.cpu_count() or 1


def cgroup_cpu_quota():
    """CPUs granted by the cgroup v2 quota (cpu.max), or None when unlimited/unknown."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(period), 2)
    except (OSError, ValueError):
        return None


def granted_cpus():
    """The CPUs this process can actually use: the cgroup quota (rounded down) when there is
    one, else the affinity mask."""
    q = cgroup_cpu_quota()
    n = host_threads()
    return max(1, min(n, int(q))) if q else n


def cpu_baseline(sc, cfg_kw, W, H, threads):
    """Time the CPU port (scalar C re-execution of the shader) on a bounded sample of the
    workload: the whole frame on `threads` threads (the granted CPUs), and 1 thread on a row
    sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import rvcp_amd
    O.build()
    cfg = rvcp_amd.abi.make_config(**cfg_kw)
    arrays = dict(materials=sc.aligned_materials(), vertices=sc.mesh.aligned_vertices(),
                  faces=sc.mesh.aligned_faces(), lum_face_ids=sc.luminous_face_ids(),
                  spheres=sc.aligned_spheres())
    push = sc.push_constant(123.0)
    common = dict(unit="Msamples/s", cores=threads, kind="port",
                  implementation="C port of the shader (oracle/rvcp_oracle.c, gcc -O3 "
                                 "-ffp-contract=off); the image has no Rust toolchain, so not a "
                                 "Rust re-execution",
                  host_threads=host_threads(), cgroup_cpu_quota=cgroup_cpu_quota(),
                  cpu=cpu_model())
    O.render(arrays, push, cfg, W, H, rect=(0, H // 2, min(W, 64), 1), threads=threads,
             want_linear=False, o3=True)                                   # warm-up (page-in, threads)
    if len(arrays["faces"]) > 1000:          # C5 on CPU: 128^2 SPP=1 frame only
        t0 = time.perf_counter()
        O.render(arrays, push, rvcp_amd.abi.make_config(**dict(cfg_kw, spp=1)), 128, 128,
                 threads=threads, want_linear=False, o3=True)
        dt = time.perf_counter() - t0
        return dict(value=round(128 * 128 / dt / 1e6, 4), sample="128x128 SPP=1 frame of the same scene",
                    seconds=round(dt, 3), **common)
    # the whole frame on `threads` threads (a few seconds), then a single-thread figure on
    # every 64th row
    t0 = time.perf_counter()
    O.render(arrays, push, cfg, W, H, threads=threads, want_linear=False, o3=True)
    dt = time.perf_counter() - t0
    samples = W * H * cfg_kw["spp"]
    rows1 = list(range(0, H, 64 if H >= 256 else 8))
    t1 = time.perf_counter()
    for y in rows1:
        O.render(arrays, push, cfg, W, H, rect=(0, y, W, 1), threads=1, want_linear=False, o3=True)
    dt1 = time.perf_counter() - t1
    return dict(value=round(samples / dt / 1e6, 4),
                sample=f"the full {W}x{H} SPP={cfg_kw['spp']} frame on {threads} threads",
                seconds=round(dt, 3),
                single_thread_value=round(len(rows1) * W * cfg_kw["spp"] / dt1 / 1e6, 4),
                single_thread_sample=f"every {64 if H >= 256 else 8}th row ({len(rows1)} rows), 1 thread",
                single_thread_seconds=round(dt1, 3), **common)


def _all_ok(dist, ok, why):
    """Agree over the control plane: (True, None) if every rank is ok, else (False, reasons)."""
    got = [None] * dist.get_world_size()
    dist.all_gather_object(got, (bool(ok), why))
    bad = [w for o, w in got if not o]
    return (not bad), (None if not bad else "; ".join(str(w) for w in bad))


def negotiate_gather(dist, rank, n_comms, make_id, init_comm, probe_render=None,
                     probe_gather=None):
    """Decide, on every rank alike, whether the frame moves over RCCL or through host memory.

    1. every rank creates RCCL ids (a local call that loads librccl: a rank without a usable
       RCCL fails here, before any collective RCCL call could block the others); agreed over
       the control plane (gloo);
    2. rank 0's ids are broadcast and every rank joins each communicator (init_comm(i, id));
       agreed;
    3. `probe_render()` (a tiny frame's render on every context, local); agreed -- so that no
       rank enters the collective gather while another rank's render already failed (its
       peers would wait in the gather forever);
    4. `probe_gather()` (the tiny frame's RCCL gather + rank 0's check); agreed.
    Any failure on any rank sends every rank to the host gather, with the reasons.  The
    communicator is created non-blocking and polled against a deadline (rvcp_rccl_init,
    rvcp_rccl_set_timeout), and so is every gather wait: when one rank's init fails at once,
    its peers' inits end with RVCP_E_TIMEOUT instead of waiting inside RCCL, and the all-gather
    of step 2 sees every rank's outcome.
    Returns ("rccl", None) or ("host", reason)."""
    ids, why = None, None
    try:
        ids = [make_id() for _ in range(n_comms)]
    except Exception as e:              # noqa: BLE001 -- reported in the JSON line
        why = f"rank {rank}: rccl id: {e!r}"
    ok, reason = _all_ok(dist, why is None, why)
    if not ok:
        return "host", reason
    got = [ids if rank == 0 else None]
    dist.broadcast_object_list(got, src=0)
    try:
        for i, uid in enumerate(got[0]):
            init_comm(i, uid)
    except Exception as e:              # noqa: BLE001
        why = f"rank {rank}: rccl init: {e!r}"
    ok, reason = _all_ok(dist, why is None, why)
    if not ok:
        return "host", reason
    for stage, fn in (("probe render", probe_render), ("gather probe", probe_gather)):
        if fn is None:
            continue
        try:
            fn()
        except Exception as e:          # noqa: BLE001
            why = f"rank {rank}: {stage}: {e!r}"
        ok, reason = _all_ok(dist, why is None, why)
        if not ok:
            return "host", reason
    return "rccl", None


def auto_pipeline(pixels, spp, legacy, small_scene, hw_queues, accel="none", steps=0):
    """Frames in flight, the path kernel's grid per frame (rvcp_config_t.grid_waves_per_simd,
    0 = every resident slot) and frames per path kernel (rvcp_render_frames_async) for a
    rank-frame of `pixels` pixels.

    `fif` contexts render consecutive launches on their own streams, so launch f+1's pre-pass
    and path kernel fill the CUs that launch f's tail leaves idle -- the per-image fences of the
    reference's swapchain loop (vulkan.rs:367-369).  A context holds one launch at a time
    (rvcp.h), so launch f waits, at its enqueue, for the one its context ran fif launches
    earlier.  A pixel is a serial chain of SPP samples: a frame of P surface pixels on L
    resident lanes ends in a tail once P/L is small (C3: ~2.6 pixels per lane, the N=8 share of
    C4: ~1.3).  Two remedies, measured (profiles/history/r03zt_batch_sweep.log, r03zu_batch_sweep2.log,
    r03zp_grid_bench_ab.log): a batch of frames in one path kernel, whose lanes take frame k+1's
    pixels while frame k's last chains finish (games101 pre-pass schedules), and else a smaller
    grid per frame with a third frame beside it, whose waves start in the tail:
      - games101, brute-force scan of a small scene or the opt-in BVH, up to 1.5 Mpixel or
        below 4 Msamples: batches of about 3 Mpixel, 4 Mpixel for frames of 1 Mpixel and more
        (at most 32 frames -- 16 before round 4, C2 0.1652 -> 0.1606 / 0.1596 ms with 20 / 25,
        r04c2b2_ab_c2batch2.log -- and at most a quarter of the timed steps), 2 in flight.  Round 4
        (profiles/history/r04b20b_ab_b20b.log, r04shb_ab_share_b.log, r04c5b_ab_c5b.log): C3 2.910 ->
        2.871 ms at 20 frames and 2.819 -> 2.799 at 60 with 4 frames instead of 3, the N=4
        share 5.990 -> 5.961 ms, C5 with the BVH 70.32 -> 69.21 ms; the N=8 share keeps 6
        (3.020 vs 3.034 ms with 8).  Batches of 3 against 3 single frames in flight on
        3 waves per SIMD: C3 3.31 -> 3.20 ms, the N=8 share of C4 3.65 -> 3.46 ms, C2
        0.232 -> 0.208 ms (batches of 2: 3.24 / 3.56 / 0.226); deeper batches for smaller
        launches (r03zx_batch_sweep3.log): the N=8 share 3.42 / 3.37 / 3.33 ms with 3 / 4 / 6
        frames, C2 0.195 / 0.173 / 0.162 / 0.158 ms with 3 / 6 / 10 / 16; C5 with the BVH
        97.6 -> 92.0 ms with 3 (profiles/history/r03zw_bvh_batch_ab.log); and 2 for larger frames
        (r03zze_batch_sweep4.log): the N=2 share of C4 13.47 -> 13.29-13.36 ms, the whole C4
        frame 26.28-26.30 -> 26.13-26.15 ms;
      - runs with too few steps for a batch (fewer than 8): frames up to 1.5 Mpixel as mode 2
        below;
      - mode 2 (no pre-pass), up to 1.5 Mpixel and at least 16 Msamples per frame: batches of
        up to 8 frames (at most a quarter of the timed steps), 2 in flight, full grid -- round 4,
        mode 2 on the C3 frame 1.667 -> 1.595 ms at 40 frames, 1.710 -> 1.633 ms at 20 with 5
        (profiles/history/r04m2p2_ab_m2pipe2.log);
      - other mode-2 frames up to 1.5 Mpixel: 3 in flight on 3 waves per SIMD -- mode 2 on the
        C3 frame 1.96 -> 1.88 ms, sphere room 0.308 -> 0.269 ms (round 4: batches of 4 / 8 for
        the sphere room 0.2654 / 0.2621 vs 0.2544 ms with 2 in flight on the full grid,
        r04m2p_ab_m2pipe.log) -- and since round 6 in batches of up to 8 frames (at most a
        quarter of the timed steps): the sphere room 0.2363 -> 0.2194 ms at 60 frames (batches
        of 2 / 4 / 6 / 10: 0.2308 / 0.2253 / 0.2261 / 0.2242, on 2 waves per SIMD 0.2241),
        0.2603 -> 0.2558 ms at 20 with 5 (profiles/r06v_ab_m2pipe6.log, r06w_ab_m2pipe7.log,
        r06x_ab_m2pipe8.log, r06za_ab_m2pipe9.log);
      - larger mode-2 frames and meshes: full grid, one frame per launch, 2 in flight (3 in
        mode 2: one kernel per frame, no pre-pass);
      - other small frames (below 4 Msamples): 4 in flight (C2 0.59/0.32/0.27/0.33 ms for
        1/2/3/4 in flight, profiles/history/r02_fif_sweep.log).
    Contexts beyond the hardware queues minus one contend for queues."""
    if not legacy and (small_scene or accel == "bvh"):
        # about 3 Mpixel per launch (4 for frames of 1 Mpixel and more) and at least 2 frames,
        # at most 32 frames, and at least 4 launches in the run
        per_launch = (4 if pixels >= 1024 * 1024 else 3) * 1024 * 1024
        batch = max(1, min(max(2, -(-per_launch // max(1, pixels))), 32,
                           steps // 4 if steps else 32))
        fif, grid = 2, 0
        if batch == 1 and pixels <= 1536 * 1024:
            fif, grid = 3, 3        # too few steps for batches: single frames, smaller grid
    elif pixels * spp < (4 << 20):
        fif, grid, batch = 4, 0, 1
    elif (legacy and small_scene and pixels <= 1536 * 1024 and pixels * spp >= (16 << 20)
          and (steps == 0 or steps >= 8)):
        # mode 2 with long pixel chains (the C3 frame): batches of up to 8 frames, 2 in flight
        fif, grid, batch = 2, 0, min(8, steps // 4 if steps else 8)
    elif small_scene and pixels <= 1536 * 1024:
        # (mode 2 only: games101 small scenes took the first branch) batches of up to 8 frames
        fif, grid, batch = 3, 3, max(1, min(8, steps // 4 if steps else 8))
    else:
        fif, grid, batch = (3 if legacy else 2), 0, 1
    try:
        fif = max(1, min(fif, int(hw_queues) - 1))
    except ValueError:
        pass
    return fif, grid, batch


class CallSchedule:
    """The bench's call schedule: `n` frames as calls of `batch` frames
    (the last one shorter) dealt round-robin to `fif` contexts; a context holds one call at a
    time (rvcp.h), so call c waits, before its enqueue, for the call its context ran `fif`
    calls earlier.  Frame f of the whole run (warm-up frames first) renders with the time seed
    TIME0 + f.  `run(n)` returns the stats of every call it made, each exactly once, in
    completion order; `slot_time[i][j]` is the seed of the frame in context i's slot j and
    `done_t` the (host time, frames) of each completed call of the last run.

    enqueue(i, pushes, nb) starts a call of nb frames on context i; finish(i, nb) waits for it
    and returns its stats.  Pure host logic: tests/test_bench_cpu.py drives it with a stub."""

    def __init__(self, fif, batch, enqueue, finish, push_of, clock=time.perf_counter):
        assert fif >= 1 and batch >= 1
        self.fif, self.batch = fif, batch
        self._enqueue, self._finish, self._push_of, self._clock = enqueue, finish, push_of, clock
        self.pending = [0] * fif            # frames of the call in flight on each context
        self.frames_run = 0                 # frames enqueued so far (the next frame's index)
        self.slot_time = [[None] * batch for _ in range(fif)]
        self.done_t = []

    def calls(self, n):
        """n frames as calls of `batch` frames (the last one shorter)."""
        return [self.batch] * (n // self.batch) + ([n % self.batch] if n % self.batch else [])

    def _finish_ctx(self, i):
        nb, self.pending[i] = self.pending[i], 0
        st = self._finish(i, nb)
        self.done_t.append((self._clock(), nb))
        return st

    def run(self, n):
        """Render n frames; returns the stats of each call (all of them, drained)."""
        self.done_t = []
        stats = []
        for c, nb in enumerate(self.calls(n)):
            i = c % self.fif
            if self.pending[i]:
                stats.append(self._finish_ctx(i))
            ts = [TIME0 + float(self.frames_run + j) for j in range(nb)]
            self.frames_run += nb
            self.slot_time[i][:nb] = ts
            self._enqueue(i, [self._push_of(t) for t in ts], nb)
            self.pending[i] = nb
        stats += [self._finish_ctx(i) for i in range(self.fif) if self.pending[i]]
        return stats


def report_failure(rank, world, wl, stage, err):
    """A rank's library error during the run (e.g. RVCP_E_TIMEOUT from a gather whose peer never
    came): one labelled JSON line on stdout (rank 0: the line the driver reads; other ranks: the
    same record), naming the rank and the stage, before the non-zero exit."""
    rec = {"metric": metric_name(wl, world), "value": None, "unit": "Msamples/s",
           "n_gpus": world, "higher_is_better": True,
           "error": {"rank": rank, "stage": stage, "code": getattr(err, "code", None),
                     "message": str(err)}}
    print(json.dumps(rec), flush=True, file=sys.stdout if rank == 0 else sys.stderr)
    return rec


def free_port():
    """A TCP port on 127.0.0.1 that is free right now (for the ranks' rendezvous)."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(n, argv, script=None):
    """`bench.py --gpus N` (N > 1) started as a plain process: start the N ranks as a
    torch.distributed.run child (one process per GPU, rendezvous on 127.0.0.1) and return its
    exit status -- non-zero when any rank failed.  This process never imports torch, so it
    never touches the GPU (no HIP initialisation before the ranks start, and no exec from a
    process that holds the GPU); the ranks inherit stdout, so rank 0's one JSON line is this
    command's output."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={free_port()}",
           script or os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    print(f"bench: self-launch of {n} ranks (parent pid {os.getpid()}, "
          f"torch imported: {'torch' in sys.modules})", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 60 frames by default: the pipeline's fill and drain (the last launch's tail, which no
    # later frame overlaps) spread over 60 frames instead of 20 -- C3 2.848 / 2.775 / 2.750 ms
    # per frame at 20 / 40 / 60 (profiles/history/r05zt_ab_steps.log); the run still takes well under
    # a second of GPU time
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default=None, choices=["c1", "c2", "c3", "c4", "c5", "c6", "spheres", "c3m2", "c3rot", "c3gen"],
                    help="default: c3 at N=1 (headline), c4 at N>1 (BASELINE's 8-GPU config)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="oracle threads for cpu_baseline (default: the CPUs this process is "
                         "granted -- the cgroup quota, else the affinity mask)")
    ap.add_argument("--save-frame", default="")
    ap.add_argument("--frames-in-flight", type=int, default=0,
                    help="contexts rendering consecutive frames concurrently (1 = one frame "
                         "at a time; 0 = auto, see auto_pipeline; N>1 rehearsals always use 1)")
    ap.add_argument("--accel", default="none", choices=["none", "bvh"],
                    help="bvh: the opt-in BVH (not the parity path; never the default line)")
    ap.add_argument("--schedule", type=int, default=0,
                    help="rvcp_config_t.kernel_variant (0 = the library's automatic choice)")
    ap.add_argument("--batch", type=int, default=0,
                    help="frames per path kernel (rvcp_render_frames_async; 1 = one frame per "
                         "rvcp_render_shard_async call; 0 = auto, see auto_pipeline)")
    ap.add_argument("--grid-waves", type=int, default=-1,
                    help="rvcp_config_t.grid_waves_per_simd: the path kernel's persistent grid "
                         "per frame in waves per SIMD (0 = every resident slot; -1 = auto, "
                         "chosen with the frames in flight)")
    ap.add_argument("--comm-timeout-ms", type=int, default=60000,
                    help="N>1: deadline of the RCCL communicator's creation and of each gather "
                         "wait (rvcp_rccl_set_timeout); past it the rank aborts its communicator "
                         "-- at creation every rank then takes the labelled host gather, during "
                         "the run the command exits non-zero with a line naming rank and stage")
    ap.add_argument("--interactive-pass", type=int, default=60,
                    help="N=1: frames of the post-timing pass in the reference's own loop shape "
                         "(one frame per launch, one in flight per swapchain image -- at most 3, "
                         "vulkan.rs:213 -- each frame's push made just before its submission: "
                         "ray_tracer.rs:80-98, vulkan.rs:367-369) -> "
                         "config.interactive_ms_per_step (0 = skip)")
    ap.add_argument("--interactive-frames-in-flight", type=int, default=0,
                    help="the interactive pass's frames in flight (1-3; 0 = auto_pipeline's "
                         "single-frame choice); for A/Bs")
    ap.add_argument("--interactive-grid-waves", type=int, default=-1,
                    help="the interactive pass's grid per frame in waves per SIMD (0 = every "
                         "resident slot; -1 = auto_pipeline's single-frame choice); for A/Bs")
    ap.add_argument("--launch-pass", type=int, default=10,
                    help="frames (at most --steps) of the post-timing one-frame-in-flight pass "
                         "that measures the path kernel's isolated launch time "
                         "(roofline.per_launch; 0 = skip)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # the driver's form `python bench.py --gpus N`: start the ranks ourselves, before
        # anything here touches the GPU
        sys.exit(self_launch(args.gpus, sys.argv[1:]))

    # Hardware queues per process: the process's own setting, else HIP's default of 4 (what the
    # GPU box runs).  No override: frames in flight are sized to the queues
    # (auto_pipeline keeps them below the queue count), and contexts sharing a queue would run
    # their frames one after another.  The value used is in the line.
    hw_queues = os.environ.get("GPU_MAX_HW_QUEUES", "4")

    import torch
    import torch.distributed as dist
    import rvcp_amd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} launched with WORLD_SIZE={world}")
    # Rehearsal (RVCP_BENCH_REHEARSAL=1): every rank on device 0 and the gather through host
    # memory over gloo (RCCL refuses two ranks on one GPU), to exercise the N>1 code path on
    # a 1-GPU box.  Never used for reported numbers.
    rehearsal = os.environ.get("RVCP_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local_rank = 0
    torch.cuda.set_device(local_rank)
    if world > 1:
        # control plane only (barriers, the max-over-ranks time, the RCCL ids, agreement on
        # the gather mode); the frame itself moves over RCCL inside librvcp
        # (rvcp_gather_frame_async)
        # (a bounded control plane too: a rank that died leaves its peers' gloo calls waiting
        # this long at most, torch.distributed.run ending them sooner)
        import datetime
        dist.init_process_group("gloo", timeout=datetime.timedelta(
            seconds=max(300, 3 * args.comm_timeout_ms // 1000)))

    wname = args.workload or ("c3" if world == 1 else "c4")
    wl = workload(wname, world)
    W, H, spp = wl["W"], wl["H"], wl["spp"]
    legacy = wl.get("integrator", 0) == 1
    sc = rvcp_amd.scene.sphere_scene() if wl.get("scene") == "spheres" else rvcp_amd.Scene.default()
    if wl["extra_tris"]:
        sc = rvcp_amd.scene.with_random_triangles(sc, wl["extra_tris"])
    if wl.get("rotate"):
        sc = rvcp_amd.scene.rotated_scene(sc)
    cfg_kw = dict(spp=spp, device=local_rank)
    if wl.get("specialize_off"):
        cfg_kw["specialize"] = 1
    if legacy:
        cfg_kw["integrator"] = 1
    if args.accel == "bvh":
        cfg_kw["accel"] = 1
    if args.schedule:
        cfg_kw["kernel_variant"] = args.schedule
    # Frames in flight: `fif` contexts render consecutive frames on their own
    # streams, so frame f+1's pre-pass and path kernel fill the CUs that frame f's tail leaves
    # idle -- the per-image fences of the reference's swapchain loop (vulkan.rs:367-369).  A
    # context holds one frame at a time (rvcp.h), so frame f waits, at its enqueue, for the
    # frame its context rendered fif steps earlier.
    # (measured, profiles/history/r02_fif_sweep.log: C3 1/2/3/4 in flight 4.35/3.83/3.83/3.95 ms,
    # C2 0.59/0.32/0.27/0.33 ms -- a small frame is mostly tail, so it gains from a third)
    # (mode 2 -- one kernel per frame, no pre-pass -- gains from a third frame at every size:
    # C3 frame 2.84/2.40/2.29/2.46 ms for 1/2/3/4 in flight, profiles/history/r02_m2_fif_sweep.log)
    # (small frames, 8 hardware queues: C2 4 in flight 0.269 ms vs 3 in flight 0.284 ms,
    # profiles/history/r02_hwq_fif_sweep.log; C3 2 and 3 equal)
    small_scene = args.accel == "none" and not wl["extra_tris"]
    # from the largest shard's size, so that every rank picks the same pipeline: the contexts'
    # communicators must see the ranks' gathers in the same order
    fif_auto, grid_auto, batch_auto = auto_pipeline(W * rvcp_amd.shard_rows(H, 0, world), spp,
                                                    legacy, small_scene, hw_queues, args.accel,
                                                    args.steps)
    fif = 1 if rehearsal else (args.frames_in_flight or fif_auto)
    batch = args.batch or batch_auto
    # (the smaller grid leaves room for frames beside it: with fewer in flight, the full grid)
    grid_waves = args.grid_waves if args.grid_waves >= 0 else (grid_auto if fif >= 3 else 0)
    cfg_kw["grid_waves_per_simd"] = grid_waves
    rts = [rvcp_amd.RayTracer(**cfg_kw) for _ in range(fif)]
    cc0 = rvcp_amd.abi.code_cache_counts()
    t_up = time.perf_counter()
    rts[0].upload_scene(sc)              # includes the scene-specialised compile (§4.7)
    upload_s = time.perf_counter() - t_up
    cc1 = rvcp_amd.abi.code_cache_counts()
    # where the upload's specialised module came from: the on-disk code-object cache
    # (rvcp_set_code_cache_dir; a verified entry of this exact compile), a hipRTC compile, or
    # none (the generic kernels; or the process's own in-memory cache)
    upload_module = ("disk cache" if cc1["loads"] > cc0["loads"] else
                     "compiled" if cc1["compiles"] > cc0["compiles"] else "none")
    build = build_identity(rts[0])
    for r in rts[1:]:
        r.upload_scene(sc)               # (the compiled module is cached per process)
    rt = rts[0]
    push = sc.push_constant(TIME0)
    n_faces = len(sc.mesh.aligned_faces())
    n_spheres = len(sc.spheres) if legacy else 0

    rows = rvcp_amd.shard_rows(H, rank, world)
    slot = rvcp_amd.shard_rows(H, 0, world)          # shard 0 has the most rows
    dev = torch.device("cuda", local_rank)
    # frame k of a context's batch at [k] (rvcp_render_frames_async's layout: shard slots of the
    # largest shard's rows)
    shard_bufs = [torch.zeros((batch, slot, W), dtype=torch.int32, device=dev) for _ in range(fif)]
    frames = [torch.zeros((batch, H, W), dtype=torch.int32, device=dev) if rank == 0 else None
              for _ in range(fif)]
    gat_flats = [torch.zeros((world, slot, W), dtype=torch.int32, device=dev)
                 if (world > 1 and rank == 0) else None for _ in range(fif)]

    # The gather mode, agreed by every rank (negotiate_gather): RCCL (one communicator per
    # context) when every rank can load RCCL, join the communicators and pass a probe gather;
    # otherwise every rank gathers through host memory over gloo, labelled in the JSON line.
    gather_mode, gather_error = ("none", None) if world == 1 else ("host", "rehearsal")
    if world > 1 and not rehearsal:
        # a tiny frame (8 rows per rank) rendered on every context, gathered and checked
        # against rank 0's own render of it
        pW, pH = 16, 8 * world
        p_slot = rvcp_amd.shard_rows(pH, 0, world)
        p_shards = [torch.zeros((p_slot, pW), dtype=torch.int32, device=dev) for _ in rts]

        def probe_render():
            for r, p_shard in zip(rts, p_shards):
                r.render_shard_async(push, pW, pH, rank, world, p_shard.data_ptr())
                r.sync_stats()
            torch.cuda.synchronize()

        def probe_gather():
            p_gat = torch.zeros((world, p_slot, pW), dtype=torch.int32, device=dev) if rank == 0 else None
            p_frame = torch.zeros((pH, pW), dtype=torch.int32, device=dev) if rank == 0 else None
            for r, p_shard in zip(rts, p_shards):
                r.gather_frame_async(p_shard.data_ptr(), pW, pH,
                                     p_gat.data_ptr() if rank == 0 else 0,
                                     p_frame.data_ptr() if rank == 0 else 0)
                r.gather_wait()
                if rank == 0:
                    ref = torch.zeros((pH, pW), dtype=torch.int32, device=dev)
                    r.render_shard_async(push, pW, pH, 0, 1, ref.data_ptr())
                    r.sync_stats()
                    torch.cuda.synchronize()
                    if not torch.equal(ref, p_frame):
                        raise RuntimeError("probe frame differs from the 1-rank render")
            torch.cuda.synchronize()
        def init_comm(i, uid):
            # non-blocking creation polled against the deadline: a peer that never joins
            # gives RVCP_E_TIMEOUT here (communicator aborted), not a rank blocked in RCCL
            rts[i].rccl_set_timeout(args.comm_timeout_ms)
            rts[i].rccl_init(uid, world, rank)
        gather_mode, gather_error = negotiate_gather(
            dist, rank, fif, rvcp_amd.rccl_unique_id, init_comm, probe_render, probe_gather)
    host_gather = world > 1 and gather_mode != "rccl"
    torch.cuda.synchronize()
    # Every frame has its own time seed, as the reference re-stamps `time` in the push
    # constant of every frame it submits (vulkan.rs:418-421): frame f (warm-up frames first,
    # then the timed ones, the same numbering on every rank) renders with time TIME0 + f, so
    # no two frames of the run share an RNG stream.
    gather_ms = []

    def enqueue(i, pushes, nb):
        """Enqueue nb frames (one call) on context i's own stream (stream 0 = its stream)."""
        r, shard_buf, gat_flat = rts[i], shard_bufs[i], gat_flats[i]
        out = frames[i] if world == 1 else shard_buf
        k, n = (0, 1) if world == 1 else (rank, world)
        if batch == 1:
            r.render_shard_async(pushes[0], W, H, k, n, out.data_ptr())
        else:
            r.render_frames_async(pushes, W, H, k, n, out.data_ptr())
        if world == 1 or host_gather:
            return
        # RCCL gather + device assembly of each frame, enqueued behind the render without a
        # host sync (the gathers of a batch reuse gat_flat in stream order)
        for j in range(nb):
            r.gather_frame_async(shard_buf[j].data_ptr(), W, H,
                                 gat_flat.data_ptr() if rank == 0 else 0,
                                 frames[i][j].data_ptr() if rank == 0 else 0)

    def finish(i, nb):
        """Wait for context i's call of nb frames; return its stats."""
        st = rts[i].sync_stats()
        if world > 1 and not host_gather:
            gather_ms.append(rts[i].gather_wait()[0])
        if host_gather:    # gloo gather through host memory (rehearsal / no usable RCCL)
            for j in range(nb):
                got = rvcp_amd.frame.gather_shards(shard_bufs[i][j].cpu(), rank, world, dst=0)
                if rank == 0:
                    gat_flats[i].copy_(torch.stack(got))
                    rts[i].assemble_frame_async(gat_flats[i].data_ptr(), slot, W, H, world,
                                                frames[i][j].data_ptr())
                    torch.cuda.synchronize()
        return st

    sched = CallSchedule(fif, batch, enqueue, finish, lambda t: sc.push_constant(t))

    # Warm-up: at least one full batch on every context, so that each context's surface list,
    # accumulator and camera buffers have their full size before timing (growing one inside the
    # timed region frees device memory, which synchronises the device and drains the other
    # context's frames)
    warm = max(args.warmup, fif * batch)
    warm = -(-warm // batch) * batch
    stage = ["warm-up frames"]
    try:
        sched.run(warm)
        gather_ms.clear()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        stage[0] = "timed frames"
        t0 = time.perf_counter()
        stats = sched.run(args.steps)
        # (a copy: the post-timing passes below render into the same buffers)
        frame = frames[0][0].clone() if rank == 0 else None
        frame_time = sched.slot_time[0][0]
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
    except rvcp_amd.abi.RvcpError as e:
        # a gather that timed out (a peer rank missing or failed: RVCP_E_TIMEOUT, the
        # communicator aborted) or any other library error: a labelled line and a non-zero exit
        # instead of a hang; torch.distributed.run then ends the other ranks
        report_failure(rank, world, wl, stage[0], e)
        raise SystemExit(3)
    kernel_ms = [float(st["kernel_ms"]) for st in stats]
    main_ms = [float(st["main_kernel_ms"]) for st in stats]
    trav = sum(int(st["traversals"]) for st in stats)
    trav_exec = sum(int(st["traversals_executed"]) for st in stats)
    variant = int(stats[-1]["kernel_variant"])
    # every timed frame rendered exactly once (CallSchedule; tests/test_bench_cpu.py sweeps
    # steps x batch x frames in flight against a stub)
    assert sum(int(st["samples"]) for st in stats) == args.steps * W * rows * spp, \
        (len(stats), [int(st["samples"]) for st in stats], args.steps, batch, fif)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    done_t = [(t0, 0)] + sched.done_t
    intervals = [(b[0] - a[0]) * 1000.0 / b[1] for a, b in zip(done_t, done_t[1:]) if b[1]]
    samples_total = W * H * spp * args.steps
    value = samples_total / elapsed / 1e6
    ms_per_step = elapsed * 1000.0 / args.steps

    # Isolated launch time (after the timed region): the path kernel with ONE frame in flight,
    # so its HIP-event time is its own (roofline.per_launch), on the full resident grid -- the
    # launch a one-frame-at-a-time caller makes (a grid left partly free for the next frame,
    # grid_waves_per_simd, only pays off with frames beside it)
    iso_ms, latency_ms, iso_clk = [], [], []
    if args.launch_pass > 0:
        rt_iso = rt if grid_waves == 0 else rvcp_amd.RayTracer(**dict(cfg_kw, grid_waves_per_simd=0))
        if rt_iso is not rt:
            rt_iso.upload_scene(sc)
        for f in range(max(1, min(args.launch_pass, args.steps))):
            tl = time.perf_counter()
            rt_iso.render_shard_async(sc.push_constant(TIME0 + float(f)), W, H, rank, world,
                                      (frames[0] if world == 1 else shard_bufs[0]).data_ptr())
            st_iso = rt_iso.sync_stats()
            iso_ms.append(float(st_iso["main_kernel_ms"]))
            iso_clk.append(float(st_iso["shader_clock_ghz"]))
            latency_ms.append((time.perf_counter() - tl) * 1000.0)
        if rt_iso is not rt:
            rt_iso.close()

    # The reference's own loop shape (after the timed region and the launch pass): one frame
    # per submission, the push constant of each frame stamped just before it is submitted
    # (ray_tracer.rs:80-98), one frame in flight per swapchain image behind per-image fences
    # (vulkan.rs:367-369) -- min_image_count + 1 images (vulkan.rs:213), 3 on common drivers --
    # no batches, nothing enqueued ahead.  Its pipeline is auto_pipeline's for single frames
    # (frames up to 1.5 Mpixel: 3 in flight on 3 waves per SIMD), at most 3 in flight; its ms
    # per frame is config.interactive_ms_per_step beside ms_per_step.
    interactive_ms = None
    fif_i = grid_i = None
    if args.interactive_pass > 0 and world == 1:
        fif_i, grid_i, _ = auto_pipeline(W * H, spp, legacy, small_scene, hw_queues, args.accel, 1)
        fif_i = min(args.interactive_frames_in_flight or fif_i, 3)
        if args.interactive_grid_waves >= 0:
            grid_i = args.interactive_grid_waves
        reuse = fif == fif_i and grid_waves == grid_i
        if reuse:
            rts_i = rts[:fif_i]
        else:
            # the timed contexts are not used again at world 1: freed first, so that the new
            # ones get hardware queues of their own (GPU_MAX_HW_QUEUES is 4; contexts sharing a
            # queue run their frames one after another: C3 3.66 vs 2.91 ms per frame,
            # profiles/history/r05zn_ovli.log; 3 in flight on 3 waves per SIMD: 2.82 ms,
            # r05zzj_ab_c3interactive.log)
            for r in rts:
                r.close()
            rts_i = [rvcp_amd.RayTracer(**dict(cfg_kw, grid_waves_per_simd=grid_i))
                     for _ in range(fif_i)]
            for r in rts_i:
                r.upload_scene(sc)
        bufs_i = [torch.zeros((H, W), dtype=torch.int32, device=dev) for _ in range(fif_i)]
        sch_i = CallSchedule(
            fif_i, 1, lambda i, pushes, nb: rts_i[i].render_shard_async(pushes[0], W, H, 0, 1,
                                                                       bufs_i[i].data_ptr()),
            lambda i, nb: rts_i[i].sync_stats(), lambda t: sc.push_constant(t))
        sch_i.run(2 * fif_i)
        torch.cuda.synchronize()
        ti = time.perf_counter()
        sch_i.run(args.interactive_pass)
        torch.cuda.synchronize()
        interactive_ms = (time.perf_counter() - ti) * 1000.0 / args.interactive_pass
        if not reuse:
            for r in rts_i:
                r.close()

    # roofline of the dominant kernel (this rank's launches).  The pre-pass (schedules 3-6,
    # games101 only) traces each pixel's primary ray once; every other reference-algorithm
    # traversal -- including the reused primary hits of samples 2..SPP -- belongs to the
    # path kernel.
    avg_frame_s = (sum(kernel_ms) / len(kernel_ms)) / 1000.0
    avg_kernel_s = (sum(main_ms) / len(main_ms)) / 1000.0
    prepass = 0 if legacy else rows * W
    units = trav / args.steps - prepass                     # traversals per path-kernel launch
    units_exec = trav_exec / args.steps - prepass
    tri_tests = units * n_faces
    flop_per_launch = tri_tests * FLOP_PER_TEST + units * n_spheres * FLOP_PER_SPHERE_TEST
    flop_exec = units_exec * (n_faces * FLOP_PER_TEST + n_spheres * FLOP_PER_SPHERE_TEST)
    wall_s = ms_per_step / 1000.0
    # (at N>1 each rank's FLOP over the max-over-ranks wall time per frame)
    achieved_tflops = flop_per_launch / wall_s / 1e12
    # 36 algorithmic bytes per triangle test (16 per sphere test)
    bytes_per_launch = units * (n_faces * 36 + n_spheres * 16)
    algo_gbs = bytes_per_launch / wall_s / 1e9
    kname = rvcp_amd.abi.KERNEL_NAMES.get(variant, "?")
    # the committed PMC summaries count only when they measured this build (the library's
    # sources and, for the specialised scan, the module): else their fields are null and the
    # line says which summary is stale
    trec, traffic_bind = bound_profile("traffic", wl["workload"], kname, build)
    vrec, valu_bind = bound_profile("valu", wl["workload"], kname, build)
    traffic = float(trec["bytes"]) if trec and trec.get("bytes") else None
    traffic_src = traffic_bind["source"]
    valu_busy = vrec.get("valu_busy") if vrec else None
    valu_insts = vrec.get("valu_insts") if vrec else None
    lane_util = vrec.get("lane_utilisation") if vrec else None
    valu_src = valu_bind["source"]
    # the shader clock of THIS run: the path kernel's own per-wave s_memtime / s_memrealtime
    # stamps (rvcp_stats_t.shader_clock_ghz), averaged over the timed calls by kernel time
    clk = [(float(st["shader_clock_ghz"]), float(st["main_kernel_ms"])) for st in stats]
    clk_w = sum(w for c, w in clk if c > 0)
    clock_ghz = (sum(c * w for c, w in clk if c > 0) / clk_w) if clk_w > 0 else None
    # the committed PMC pass's VALU instructions per frame (one frame per launch there) over
    # the issue slots of one timed frame at this run's clock: how close the wall clock is to the
    # issue floor (the guide's 0.5 wave-instructions per SIMD-cycle)
    valu_wall = (None if not valu_insts or world != 1 or not clock_ghz else
                 valu_insts / (ms_per_step * 1e-3 * clock_ghz * 1e9 * N_SIMDS * VALU_ISSUE_PER_CLK))
    bvh = args.accel == "bvh"
    iso_s = (float(np.mean(iso_ms)) / 1000.0) if iso_ms else None

    frame_check, one_gpu_ms = None, None
    if world > 1 and rank == 0:
        # the assembled N-rank frame must be bit-identical to a 1-rank render of the same frame
        # (outside timing); the same frame rendered by this GPU alone, pipelined the way a
        # one-GPU run of that frame is (auto_pipeline for the whole frame, unless the command
        # line fixed fif / grid for both), is the single-GPU reference for the speedup
        fif1, grid1, batch1 = auto_pipeline(W * H, spp, legacy, small_scene, hw_queues,
                                            args.accel, 3 * 4 * 2)
        fif1 = args.frames_in_flight or fif1
        grid1 = args.grid_waves if args.grid_waves >= 0 else (grid1 if fif1 >= 3 else 0)
        batch1 = args.batch or batch1
        if (fif1, grid1) == (fif, grid_waves):
            rts1, own1 = rts, False
        else:
            rts1 = [rvcp_amd.RayTracer(**dict(cfg_kw, grid_waves_per_simd=grid1)) for _ in range(fif1)]
            for r in rts1:
                r.upload_scene(sc)
            own1 = True
        singles = [torch.zeros((batch1, H, W), dtype=torch.int32, device=dev) for _ in range(fif1)]

        def render1(i, f0, nb=batch1):
            # frames f0 .. f0 + nb - 1 of the one-GPU run, each with its own time seed
            pushes = [sc.push_constant(TIME0 + float(f0 + j)) for j in range(nb)]
            if nb == 1:
                rts1[i].render_shard_async(pushes[0], W, H, 0, 1, singles[i].data_ptr())
            else:
                rts1[i].render_frames_async(pushes, W, H, 0, 1, singles[i].data_ptr())
        n1 = 3 * fif1                                      # launches of batch1 frames
        for i in range(fif1):                              # warm-up, one per context
            render1(i, 0)
        for i in range(fif1):
            rts1[i].sync_stats()
        torch.cuda.synchronize()
        busy = [False] * fif1
        ts = time.perf_counter()
        for f in range(n1):
            i = f % fif1
            if busy[i]:
                rts1[i].sync_stats()
            render1(i, f * batch1)
            busy[i] = True
        for i in range(fif1):
            if busy[i]:
                rts1[i].sync_stats()
        torch.cuda.synchronize()
        one_gpu_ms = (time.perf_counter() - ts) * 1000.0 / (n1 * batch1)
        # the check: the assembled frame of context 0's slot 0 against this GPU's render of
        # the same time seed
        rts1[0].render_shard_async(sc.push_constant(frame_time), W, H, 0, 1, singles[0].data_ptr())
        rts1[0].sync_stats()
        torch.cuda.synchronize()
        frame_check = bool(torch.equal(singles[0][0], frame))
        if own1:
            for r in rts1:
                r.close()

    per_rank = None
    if world > 1:
        mine = dict(rank=rank, path_kernel_ms=round(avg_kernel_s * 1000.0, 4),
                    frame_kernels_ms=round(avg_frame_s * 1000.0, 4),
                    isolated_path_kernel_ms=None if iso_s is None else round(iso_s * 1000.0, 4),
                    gather_ms=round(float(np.mean(gather_ms)), 4) if gather_ms else None,
                    rows=rows)
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
        dist.barrier()

    if args.save_frame and rank == 0:
        np.save(args.save_frame, frame.cpu().numpy().view(np.uint8).reshape(H, W, 4))

    if rank == 0:
        out = {
            "metric": metric_name(wl, world),
            "value": round(value, 2),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "fps": round(1000.0 / ms_per_step, 2),
            # median of the intervals between consecutive calls' completions (host clock),
            # per frame of the later call: the pipelined frame interval, not a frame latency
            # (that is config.frame_latency_ms_alone)
            "frame_interval_ms_median": round(float(np.median(intervals)), 4) if intervals else None,
            "higher_is_better": True,
            "scaling": wl["scaling"],
            # the reference's published rows are single-GPU (RTX 3060) C3 / C2 frames, timed by
            # its own loop (one frame per submission, a push per frame made just before it,
            # ray_tracer.rs:80-98): compared on that loop shape here (the interactive pass), not
            # on the batched pipeline's rate, which the reference's loop cannot run
            "vs_baseline": vs_baseline_loop_shape(wname, world, W * H * spp, interactive_ms),
            "vs_baseline_batched": (round(value / REFERENCE_MSAMPLES[wname], 2)
                                    if world == 1 and wname in REFERENCE_MSAMPLES else None),
            "vs_baseline_definition": (
                "Msamples/s of the reference's loop shape (config.interactive_ms_per_step: one "
                "frame per launch, one in flight per swapchain image, push stamped at submission) "
                "/ the reference's published row (README.md:19-26, RTX 3060); "
                "vs_baseline_batched: value (batched pipeline) / the same row"),
            "dtype": "f32",
            "data": ("synthetic (the reference's deprecated sphere-room scene, integrator mode 2"
                     if wl.get("scene") == "spheres" else
                     "synthetic (the reference's built-in Cornell box scene, integrator mode 2"
                     if legacy else
                     "synthetic (the reference's built-in Cornell box scene") +
                    f"{', rotated off-axis' if wl.get('rotate') else ''}; time seed {TIME0} + frame "
                    "index, a new RNG stream every frame)",
            "config": {"workload": wl["workload"], "width": W, "height": H, "spp": spp,
                       "faces": n_faces, "parallelism": f"pixel-stripes x{world}",
                       "accel": args.accel, "kernel_schedule": variant & ~rvcp_amd.abi.VARIANT_SPECIALIZED,
                       "scan": ("scene-specialised (hipRTC at upload, DESIGN.md §4.7)"
                                if variant & rvcp_amd.abi.VARIANT_SPECIALIZED else "generic"),
                       "upload_s": round(upload_s, 3),
                       "upload_module": upload_module,
                       # warm-up frames actually run: at least one full batch per context
                       "warmup_frames": warm,
                       "frames_in_flight": fif, "grid_waves_per_simd": grid_waves,
                       "frames_per_launch": batch,
                       # one frame alone, enqueue to completion (the latency of a synchronous
                       # rvcp_render of this rank's frame; ms_per_step is the pipelined rate)
                       "frame_latency_ms_alone": (round(float(np.median(latency_ms)), 4)
                                                  if latency_ms else None),
                       # the reference's loop shape: one frame per launch, one in flight per
                       # swapchain image (at most 3), a push per frame made just before its
                       # submission (ray_tracer.rs:80-98, vulkan.rs:213, 367-369); ms_per_step
                       # is the batched pipeline's rate.  vs_baseline is quoted on this one.
                       "interactive_ms_per_step": (None if interactive_ms is None else
                                                   round(interactive_ms, 4)),
                       "interactive_msamples_s": (None if not interactive_ms else
                                                  round(W * H * spp / (interactive_ms / 1000.0) / 1e6, 2)),
                       "interactive_frames": args.interactive_pass if interactive_ms else 0,
                       "interactive_frames_in_flight": fif_i,
                       "interactive_grid_waves_per_simd": grid_i,
                       "gpu_max_hw_queues": hw_queues,
                       "gather": ("none" if world == 1 else
                                  "gloo-rehearsal (all ranks on GPU 0)" if rehearsal else
                                  "rccl ncclGather via rvcp_gather_frame_async" if not host_gather
                                  else f"gloo through host memory (RCCL not usable: {gather_error})")},
            "roofline": {"bound": "latency (dependent BVH node loads)" if bvh else "valu",
                         "achieved": None if bvh else round(achieved_tflops, 2),
                         "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": None if bvh else round(achieved_tflops / FP32_PEAK_TFLOPS, 4),
                         "definition": (
                             "BVH: the brute-force scan's FLOP are not executed; no FLOP roofline "
                             "(DESIGN.md §4.6)" if bvh else
                             f"useful FP32 FLOP per frame ({FLOP_PER_TEST} per reference-"
                             f"algorithm ray-triangle test, {FLOP_PER_SPHERE_TEST} per ray-sphere "
                             "test) / ms_per_step / peak"),
                         "frac_executed": None if bvh else round(flop_exec / wall_s / 1e12 / FP32_PEAK_TFLOPS, 4),
                         "frac_executed_definition": "FLOP of the traversals the kernels execute "
                                                     "(primary hit once per pixel) / ms_per_step / peak",
                         "per_launch": None if (bvh or iso_s is None) else {
                             "kernel_ms": round(iso_s * 1000.0, 4),
                             "kernel_ms_min": round(min(iso_ms), 4),
                             "achieved": round(flop_per_launch / iso_s / 1e12, 2),
                             "frac": round(flop_per_launch / iso_s / 1e12 / FP32_PEAK_TFLOPS, 4),
                             # the honest kernel fraction: only the
                             # traversals the kernel executes (the primary hit once per pixel)
                             "frac_executed": round(flop_exec / iso_s / 1e12 / FP32_PEAK_TFLOPS, 4),
                             "frames": len(iso_ms),
                             "grid_waves_per_simd": 0,
                             "definition": "useful FLOP / the path kernel's HIP-event time with "
                                           "one frame in flight on the full resident grid "
                                           "(post-timing pass)"},
                         "kernel": kname,
                         "kernel_ms_in_flight": round(avg_kernel_s * 1000.0, 4),
                         "frames_per_launch": batch,
                         "frame_kernels_ms_in_flight": round(avg_frame_s * 1000.0, 4),
                         "traffic": None if traffic is None else round(traffic),
                         "traffic_source": traffic_src,
                         "traffic_hbm_frac": None if (traffic is None or iso_s is None) else
                         round(traffic / iso_s / 1e9 / HBM_PEAK_GBS, 5),
                         "tests_per_launch": round(tri_tests),
                         "hbm_algorithmic": {
                             "bytes_per_launch": round(bytes_per_launch),
                             "achieved_gbs": round(algo_gbs, 1),
                             "frac_of_peak": round(algo_gbs / HBM_PEAK_GBS, 4),
                             "definition": "SURVEY.md §8(d): reference-algorithm traversals x "
                                           "(F x 36 B + S x 16 B) per frame / ms_per_step; > 1 "
                                           "= on-chip reuse (scene in scalar cache / LDS)"},
                         "traversals_per_sample": round(trav / args.steps / (W * H * spp / world), 4)
                         if world == 1 else None,
                         "executed_traversal_frac": round(trav_exec / max(trav, 1), 4),
                         "valu_issue_frac_pmc_guide": valu_busy,
                         "lane_utilisation_pmc": lane_util,
                         # the build this run executes and the summaries' own: PMC-derived
                         # fields are null unless the summary measured this same build
                         "profile_binding": {"build": build, "valu": valu_bind,
                                             "traffic": traffic_bind},
                         "stale_profile": any(b["build_match"] is False
                                              for b in (valu_bind, traffic_bind)),
                         "valu_insts_per_frame_pmc": None if not valu_insts else round(valu_insts),
                         "shader_clock_ghz": None if clock_ghz is None else round(clock_ghz, 4),
                         "shader_clock_ghz_isolated": (round(float(np.mean(iso_clk)), 4)
                                                       if iso_clk and min(iso_clk) > 0 else None),
                         "shader_clock_definition": (
                             "this run's path-kernel waves: sum of s_memtime ticks / sum of "
                             "s_memrealtime ticks x 100 MHz, start to end of each wave (timed "
                             "calls, weighted by kernel time; _isolated: the one-frame pass)"),
                         "valu_issue_frac_wall": None if valu_wall is None else round(valu_wall, 4),
                         "valu_issue_frac_wall_definition": (
                             "PMC SQ_INSTS_VALU of the dominant kernel per frame (" + str(valu_src) +
                             f") / (ms_per_step x shader_clock_ghz x {N_SIMDS} SIMDs x "
                             f"{VALU_ISSUE_PER_CLK} wave-instructions per SIMD-cycle: the guide's "
                             "issue rate)")},
            "cpu_baseline": None,
        }
        if world > 1:
            out["config"]["per_rank"] = per_rank
        if args.save_frame:
            out["config"]["saved_frame_time"] = frame_time      # the saved frame's time seed
        if frame_check is not None:
            out["config"]["assembled_frame_bitexact_vs_1gpu"] = frame_check
            out["config"]["one_gpu_ms"] = round(one_gpu_ms, 4)
            out["config"]["one_gpu_frames_in_flight"] = fif1
            out["config"]["one_gpu_grid_waves_per_simd"] = grid1
            out["config"]["one_gpu_frames_per_launch"] = batch1
            out["config"]["speedup_vs_one_gpu_same_frame"] = round(one_gpu_ms / ms_per_step, 3)
            # the same frame's Msamples/s on this GPU alone: value / one_gpu_value is the
            # scaling curve of this frame
            out["config"]["one_gpu_value"] = round(W * H * spp / (one_gpu_ms / 1000.0) / 1e6, 2)
            if rehearsal:
                out["config"]["physical_gpus"] = 1
        if world == 1 and not args.no_cpu_baseline:
            threads = args.cpu_threads or granted_cpus()
            out["cpu_baseline"] = cpu_baseline(sc, cfg_kw, W, H, threads)
        print(json.dumps(out), flush=True)

    for r in rts:
        r.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
