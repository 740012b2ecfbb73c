"""bench.py host logic on CPU: the workload table against BASELINE.json's configs, the roofline
constants, and the loaders of the committed PMC summaries (no GPU, nothing rendered)."""
import json
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_workloads_match_baseline_configs():
    """C1-C5 sizes are BASELINE.json configs[0..4]; N=1 defaults to C3, N>1 C4 is strong."""
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        configs = json.load(f)["configs"]
    want = {"c1": (128, 1), "c2": (384, 10), "c3": (1024, 30), "c4": (2048, 64), "c5": (1024, 30)}
    for (name, (side, spp)), text in zip(want.items(), configs):
        wl = bench.workload(name, 1)
        assert (wl["W"], wl["H"], wl["spp"]) == (side, side, spp)
        assert f"{side}" in text and f"SPP={spp}" in text
    assert bench.workload("c5", 1)["extra_tris"] == 100000
    c6 = bench.workload("c6", 1)                   # the reference's own scene-size limit
    assert (c6["W"], c6["spp"], 32 + c6["extra_tris"], 68 + 3 * c6["extra_tris"]) == (1024, 30, 342, 998)
    assert bench.workload("c4", 8)["scaling"] == "strong"
    assert bench.workload("c4", 8)["W"] == 2048                 # fixed frame at any N
    assert bench.workload("c3", 1)["workload"] == "cornell_1024sq_spp30"
    assert bench.workload("c3", 4)["W"] == 2048                 # weak-scaled C3 side
    m2 = bench.workload("c3m2", 1)
    assert (m2["W"], m2["spp"], m2["integrator"], m2["scene"]) == (1024, 30, 1, "cornell")
    assert bench.workload("spheres", 1)["scene"] == "spheres"
    with pytest.raises(SystemExit):
        bench.workload("nope", 1)


def test_auto_pipeline():
    """Frames in flight, grid per frame and frames per launch: games101 on a
    small scene (or the BVH) in batches of about 3 Mpixel (4 from 1-Mpixel frames) and at least 2 frames (at most 32,
    at most a quarter of the timed steps), 2 in flight; mode 2 up to 1.5 Mpixel with at least 16
    Msamples per frame in batches of up to 8, 2 in flight, other mode-2 frames up to 1.5 Mpixel
    3 in flight on 3 waves per SIMD in batches of up to 8; larger mode-2 frames and meshes the full grid, one frame per launch;
    never more contexts than the hardware queues minus one."""
    ap = bench.auto_pipeline
    assert ap(1024 * 1024, 30, False, True, "4", "none", 20) == (2, 0, 4)          # C3
    assert ap(1024 * 1024, 30, False, True, "4") == (2, 0, 4)
    assert ap(2048 * 256, 64, False, True, "4", "none", 40) == (2, 0, 6)           # C4, N=8 share
    assert ap(2048 * 256, 64, False, True, "4", "none", 20) == (2, 0, 5)
    assert ap(2048 * 512, 64, False, True, "4", "none", 20) == (2, 0, 4)           # C4, N=4 share
    assert ap(2048 * 1024, 64, False, True, "4", "none", 20) == (2, 0, 2)          # C4, N=2 share
    assert ap(2048 * 2048, 64, False, True, "4", "none", 20) == (2, 0, 2)          # C4, one GPU
    assert ap(2048 * 2048, 64, False, True, "4", "none", 4) == (2, 0, 1)           # 4 steps
    assert ap(384 * 384, 10, False, True, "4", "none", 200) == (2, 0, 22)          # C2
    assert ap(384 * 384, 10, False, True, "4", "none", 100) == (2, 0, 22)
    assert ap(256 * 256, 10, False, True, "4", "none", 400) == (2, 0, 32)
    assert ap(384 * 384, 10, False, True, "4", "none", 20) == (2, 0, 5)
    assert ap(384 * 384, 10, False, True, "4", "none", 3) == (3, 3, 1)             # too few steps
    assert ap(1024 * 1024, 30, False, True, "4", "none", 5) == (3, 3, 1)
    assert ap(1024 * 1024, 30, True, True, "4", "none", 20) == (2, 0, 5)           # mode 2, C3 frame
    assert ap(1024 * 1024, 30, True, True, "4", "none", 40) == (2, 0, 8)
    assert ap(1024 * 1024, 30, True, True, "4", "none", 5) == (3, 3, 1)            # too few steps
    assert ap(1024 * 1024, 5, True, True, "4", "none", 20) == (3, 3, 5)            # sphere room
    assert ap(1024 * 1024, 5, True, True, "4", "none", 60) == (3, 3, 8)
    assert ap(1024 * 1024, 5, True, True, "4", "none", 8) == (3, 3, 2)
    assert ap(1024 * 1024, 5, True, True, "4", "none", 3) == (3, 3, 1)             # too few steps
    assert ap(384 * 384, 5, True, True, "8", "none", 20) == (4, 0, 1)              # small mode-2 frame
    assert ap(384 * 384, 5, True, True, "4", "none", 20) == (3, 0, 1)              # ... on 4 queues
    assert ap(1024 * 1024, 30, False, False, "4", "none", 20) == (2, 0, 1)         # C5 (mesh)
    assert ap(1024 * 1024, 30, False, False, "4", "bvh", 20) == (2, 0, 4)          # C5 with the BVH
    assert ap(1024 * 1024, 30, False, True, "2", "none", 20) == (1, 0, 4)
    assert ap(1024 * 1024, 30, False, True, "x", "none", 20) == (2, 0, 4)


def test_interactive_pipeline():
    """The reference's loop shape (bench.py's interactive pass): auto_pipeline for single
    frames (steps = 1: no batches), at most 3 in flight -- one per swapchain image,
    min_image_count + 1 (vulkan.rs:213)."""
    ap = bench.auto_pipeline
    assert ap(1024 * 1024, 30, False, True, "4", "none", 1) == (3, 3, 1)           # C3
    assert ap(384 * 384, 10, False, True, "4", "none", 1) == (3, 3, 1)             # C2
    assert ap(1024 * 1024, 5, True, True, "4", "none", 1) == (3, 3, 1)             # sphere room
    assert ap(1024 * 1024, 30, False, False, "4", "bvh", 1) == (3, 3, 1)           # C5, BVH
    assert ap(1024 * 1024, 30, False, False, "4", "none", 1) == (2, 0, 1)          # c6 / C5 mesh
    assert ap(2048 * 2048, 64, False, True, "4", "none", 1) == (2, 0, 1)           # C4 frame


def test_roofline_constants():
    assert bench.FLOP_PER_TEST == 52 and bench.FP32_PEAK_TFLOPS == 157.3
    assert bench.REFERENCE_MSAMPLES["c3"] == pytest.approx(1024 * 1024 * 30 * 3 / 1e6, rel=0.01)
    assert bench.REFERENCE_MSAMPLES["c2"] == pytest.approx(384 * 384 * 10 * 51 / 1e6, rel=0.01)


def test_vs_baseline_uses_the_reference_loop_shape():
    """vs_baseline is the reference loop shape's rate (one frame per launch,
    interactive_ms_per_step) over the published row, not the batched pipeline's."""
    # C2 at the round-5 loop-shape time 0.237 ms: x83, not the batched x125
    assert bench.vs_baseline_loop_shape("c2", 1, 384 * 384 * 10, 0.237) == pytest.approx(82.7, abs=0.1)
    assert bench.vs_baseline_loop_shape("c3", 1, 1024 * 1024 * 30, 2.81) == pytest.approx(118.6, abs=0.1)
    # no published row (C4, mode 2), N > 1, or no interactive pass: null
    assert bench.vs_baseline_loop_shape("c4", 1, 2048 * 2048 * 64, 22.0) is None
    assert bench.vs_baseline_loop_shape("c3", 2, 1024 * 1024 * 30, 2.81) is None
    assert bench.vs_baseline_loop_shape("c3", 1, 1024 * 1024 * 30, None) is None


def test_committed_pmc_summaries_load():
    """The bench line's traffic / VALU fields come from these summaries: they exist for the
    headline C3 kernel and the C5 tiled kernel, and carry per-launch numbers."""
    for wl, kname in [("cornell_1024sq_spp30", "rvcp_spec_path_kernel5"),
                      ("cornell_plus_100k_tris_1024sq_spp30", "games101_tiled_pool_kernel")]:
        traffic, src = bench.load_traffic(wl, kname)
        assert traffic and traffic > 0 and src.startswith("profiles/")
        busy, frac = bench.load_valu_busy(wl, kname)
        assert 0 < busy <= 1 and 0 < frac <= 1
    busy, frac = bench.load_valu_busy("cornell_mode2_1024sq_spp30", "rvcp_spec_legacy_kernel")
    assert 0 < busy <= 1 and 0 < frac <= 1


def test_pmc_fields_bound_to_the_build(monkeypatch):
    """a PMC summary counts only for the build it measured (the library's
    source identity and the specialised module's key, recorded from the PMC passes' own bench
    lines); any other build gets null fields and build_match False."""
    rec = {"valu_insts": 2.8e9, "valu_busy": 0.7}
    mine = {"source": "15761ae75e2389d3", "module": "00000000deadbeef"}
    for pbuild, want in [(dict(mine), True), (dict(mine, module="0000000000000001"), False),
                         (dict(mine, source="0"), False), (None, False)]:
        monkeypatch.setattr(bench, "profile_summary", lambda *a, pb=pbuild: (rec, "profiles/x.json", pb))
        got, bind = bench.bound_profile("valu", "w", "k", mine)
        assert bind["build_match"] is want and (got is rec) == want and bind["source"] == "profiles/x.json"
    monkeypatch.setattr(bench, "profile_summary", lambda *a: (None, None, None))
    got, bind = bench.bound_profile("valu", "w", "k", mine)
    assert got is None and bind["build_match"] is None


def test_pmc_summary_build_from_bench_logs(tmp_path):
    """tools/pmc_valu.py / pmc_traffic.py take the build from the passes' bench lines; passes
    that disagree (or a log without a line) give None, which bench.py treats as stale."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("pmc_valu", os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "pmc_valu.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    b = {"source": "a", "module": "b"}
    logs = []
    for i, build in enumerate([b, b, dict(b, module="c")]):
        p = tmp_path / f"p{i}.log"
        p.write_text("noise\n" + json.dumps({"roofline": {"profile_binding": {"build": build}}}) + "\n")
        logs.append(str(p))
    assert m.build_of(logs[:2]) == b
    assert m.build_of(logs) is None
    empty = tmp_path / "e.log"
    empty.write_text("no line\n")
    assert m.build_of([str(empty)]) is None and m.build_of([]) is None


def _negotiate_worker(rank, world, port, outdir):
    """One rank of bench.py's N>1 control flow (negotiate_gather) over gloo, with the RCCL
    calls replaced by stand-ins that fail on chosen ranks."""
    import torch.distributed as dist
    import rvcp_amd
    RVCP_E_TIMEOUT, RvcpError = rvcp_amd.abi.RVCP_E_TIMEOUT, rvcp_amd.abi.RvcpError
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    results = {}
    try:
        for case, bad_rank, stage in [("ok", -1, ""), ("id", 3, "id"), ("init", 5, "init"),
                                      ("render", 6, "render"), ("probe", 7, "probe"),
                                      ("init_all", -2, "init"), ("init_timeout", 4, "init_t"),
                                      ("probe_timeout", 2, "probe_t")]:
            inited = []
            gathered = []

            def fails(st):
                return stage == st and (bad_rank == rank or bad_rank == -2)

            def make_id():
                if fails("id"):
                    raise RuntimeError("cannot load librccl.so.1")
                return bytes([rank]) * 128

            def init_comm(i, uid):
                if fails("init"):
                    raise RuntimeError("ncclCommInitRank: unhandled system error")
                if stage == "init_t":
                    # the asymmetric case a blocking init could not survive: rank 4 fails at
                    # once, its peers' non-blocking inits run into the deadline
                    # (rvcp_rccl_init -> RVCP_E_TIMEOUT, communicator aborted)
                    if rank == bad_rank:
                        raise RuntimeError("ncclCommInitRankConfig: invalid usage")
                    raise RvcpError(RVCP_E_TIMEOUT, "ncclCommInitRankConfig: no progress within "
                                    "60000 ms (a peer rank missing or failed)")
                assert uid == bytes([0]) * 128          # every rank joins rank 0's ids
                inited.append(i)

            def probe_render():
                if fails("render"):
                    raise RuntimeError("render: out of memory")

            def probe_gather():
                gathered.append(True)
                if fails("probe"):
                    raise RuntimeError("ncclGather: internal error")
                if stage == "probe_t" and rank != bad_rank:
                    # rank 2 never enters the gather: every other rank's wait hits the deadline
                    raise RvcpError(RVCP_E_TIMEOUT, "gather not complete within 60000 ms")

            mode, why = bench.negotiate_gather(dist, rank, 2, make_id, init_comm, probe_render,
                                               probe_gather)
            results[case] = (mode, why, inited, gathered)
        import pickle
        with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
            pickle.dump(results, f)
    finally:
        dist.destroy_process_group()


def test_negotiate_gather_world8_injected_failures(tmp_path):
    """bench.py at N=8: a failure on ANY rank (no loadable RCCL, communicator init, the probe
    gather) sends EVERY rank to the same host-memory gather, with the failing rank named; with
    no failure every rank takes RCCL.  (gloo, world size 8, on CPU)"""
    import pickle
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_negotiate_worker, args=(8, port, str(tmp_path)), nprocs=8, join=True)
    res = []
    for r in range(8):
        with open(tmp_path / f"r{r}.pkl", "rb") as f:
            res.append(pickle.load(f))
    for r in range(8):
        assert res[r]["ok"][0] == "rccl" and res[r]["ok"][1] is None and res[r]["ok"][2] == [0, 1]
        for case, bad in [("id", "rank 3"), ("init", "rank 5"), ("render", "rank 6"),
                          ("probe", "rank 7")]:
            mode, why, _, _ = res[r][case]
            assert mode == "host" and bad in why, (r, case, why)
        mode, why, _, _ = res[r]["init_all"]
        assert mode == "host" and all(f"rank {k}" in why for k in range(8))
        # an injected deadline: every rank agrees on the host gather, the failing rank and the
        # timed-out ones are all named, and nobody was left inside a collective
        mode, why, _, _ = res[r]["init_timeout"]
        assert mode == "host" and "rank 4" in why and "invalid usage" in why
        assert all(f"rank {k}" in why for k in range(8)) and "error -7" in why
        mode, why, _, gathered = res[r]["probe_timeout"]
        assert mode == "host" and "error -7" in why and "rank 2" not in why
        assert gathered == [True]
        # a render failure on one rank keeps EVERY rank out of the collective gather (its
        # peers would otherwise wait in it forever)
        assert res[r]["render"][3] == [] and res[r]["ok"][3] == [True]
    # the id failure stops before any communicator is joined
    assert all(res[r]["id"][2] == [] for r in range(8))


_RANK_STUB = '''
import json, os, sys
import torch
import torch.distributed as dist
dist.init_process_group("gloo")
r, w = dist.get_rank(), dist.get_world_size()
t = torch.tensor([float(r)])
dist.all_reduce(t)
if r == 0:
    print(json.dumps({"n_gpus": w, "sum": float(t.item()), "argv": sys.argv[1:],
                      "master": os.environ["MASTER_ADDR"]}), flush=True)
fail = os.environ.get("STUB_FAIL_RANK")
dist.destroy_process_group()
if fail is not None and int(fail) == r:
    sys.exit(3)
'''


def _self_launch(tmp_path, extra_env=None):
    import subprocess
    import sys
    stub = tmp_path / "rank_stub.py"
    stub.write_text(_RANK_STUB)
    code = ("import sys, bench\n"
            f"rc = bench.self_launch(2, ['--gpus', '2', '--steps', '3'], script={str(stub)!r})\n"
            "print('PARENT_TORCH', 'torch' in sys.modules, flush=True)\n"
            "sys.exit(rc)\n")
    env = dict(os.environ, **(extra_env or {}))
    env.pop("WORLD_SIZE", None)
    return subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True,
                          text=True, timeout=180, env=env)


def test_self_launch_relays_rank0_line(tmp_path):
    """`python bench.py --gpus N` without a launcher (the driver's form): bench.self_launch
    starts N ranks under torch.distributed.run on 127.0.0.1 and its stdout carries rank 0's
    one JSON line; the parent never imports torch, so it never initialises the GPU (here the
    ranks are a gloo stand-in for bench.py's own main)."""
    r = _self_launch(tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["sum"] == 1.0 and d["master"] == "127.0.0.1"
    assert d["argv"] == ["--gpus", "2", "--steps", "3"]
    assert "PARENT_TORCH False" in r.stdout


def test_self_launch_fails_with_a_rank(tmp_path):
    """A failing rank makes the whole command fail (non-zero exit status)."""
    r = _self_launch(tmp_path, {"STUB_FAIL_RANK": "1"})
    assert r.returncode != 0


class _StubTracer:
    """Stand-in for a RayTracer context: one call in flight at a time, stats of the last call."""

    def __init__(self, log, i):
        self.log, self.i, self.inflight = log, i, None

    def enqueue(self, pushes, nb):
        assert self.inflight is None, "a context holds one call at a time (rvcp.h)"
        assert len(pushes) == nb
        self.inflight = list(pushes)
        self.log.extend(pushes)

    def finish(self, nb):
        assert self.inflight is not None and len(self.inflight) == nb
        st = {"samples": nb * 7, "frames": self.inflight}
        self.inflight = None
        return st


def test_call_schedule_accounts_every_frame_once():
    """bench.CallSchedule (the warm-up and timed calls of bench.py) over
    steps x frames per launch x frames in flight: every frame is enqueued exactly once with its
    own time seed, every call's stats come back exactly once (so `sum(samples)` is exact), no
    context ever holds two calls, and the seeds continue from warm-up into the timed run."""
    for fif in (1, 2, 3, 4):
        for batch in (1, 2, 3, 4, 5, 7, 8, 16, 22, 32):
            for steps in list(range(1, 41)) + [63, 64, 65, 100, 129]:
                log = []
                tr = [_StubTracer(log, i) for i in range(fif)]
                sched = bench.CallSchedule(fif, batch, lambda i, p, nb: tr[i].enqueue(p, nb),
                                           lambda i, nb: tr[i].finish(nb), lambda t: t)
                warm = -(-max(3, fif * batch) // batch) * batch
                w_stats = sched.run(warm)
                assert sum(s["samples"] for s in w_stats) == warm * 7
                assert all(t.inflight is None for t in tr) and sched.pending == [0] * fif
                stats = sched.run(steps)
                assert sum(s["samples"] for s in stats) == steps * 7, (fif, batch, steps)
                assert len(stats) == len(sched.calls(steps)) == len(sched.done_t)
                assert sum(nb for _, nb in sched.done_t) == steps
                want = [bench.TIME0 + f for f in range(warm + steps)]
                assert log == want                       # every seed once, in order
                got = sorted(t for s in stats for t in s["frames"])
                assert got == want[warm:]                # each timed call's stats exactly once
                assert all(t.inflight is None for t in tr)
                # slot 0 of context 0 holds the first frame of the last call made on it
                c0 = [c for c in range(len(sched.calls(steps))) if c % fif == 0][-1]
                assert sched.slot_time[0][0] == bench.TIME0 + warm + sum(sched.calls(steps)[:c0])


def test_report_failure_names_rank_and_stage(capsys):
    """A library error during the run (a gather's RVCP_E_TIMEOUT) becomes one labelled JSON line
    naming the rank, the stage and the code (rank 0 on stdout, the driver's line)."""
    import rvcp_amd
    RVCP_E_TIMEOUT, RvcpError = rvcp_amd.abi.RVCP_E_TIMEOUT, rvcp_amd.abi.RvcpError
    wl = bench.workload("c4", 8)
    err = RvcpError(RVCP_E_TIMEOUT, "gather not complete within 60000 ms")
    rec = bench.report_failure(0, 8, wl, "timed frames", err)
    line = capsys.readouterr().out.strip()
    assert json.loads(line) == rec
    assert rec["value"] is None and rec["n_gpus"] == 8
    assert rec["error"] == {"rank": 0, "stage": "timed frames", "code": -7,
                            "message": "rvcp error -7: gather not complete within 60000 ms"}
    bench.report_failure(3, 8, wl, "warm-up frames", err)
    cap = capsys.readouterr()
    assert cap.out == "" and json.loads(cap.err)["error"]["rank"] == 3
