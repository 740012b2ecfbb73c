"""Interactive caller (rvcp_amd.interactive): the camera update of
src/ray_tracer/ray_tracer.rs:104-164, the FPS counter of :80-87, the per-frame time seed and
a headless frame loop with image dumps.  CPU tests use a recording stand-in for the tracer;
the GPU test drives the real RayTracer and checks the last frame against the oracle."""
import os
import zlib

import numpy as np
import pytest

import oracle as O
import rvcp_amd
from conftest import scene_arrays

I = rvcp_amd.interactive
f32 = np.float32


def _cam():
    return rvcp_amd.Scene.default().camera


def test_camera_new_yaw_pitch_f32():
    c = _cam()                                   # forward (0, 0, 1): yaw 90, pitch 0
    assert np.array_equal(c.forward, np.array([0, 0, 1], dtype=f32))
    assert f32(c.yaw) == f32(f32(np.pi / 2) * I.DEGS_PER_RAD) and c.pitch == 0.0
    s = rvcp_amd.scene.sphere_scene().camera      # looking down at the origin
    assert -90.0 < s.pitch < 0.0 and f32(s.yaw) == f32(s.yaw)


@pytest.mark.parametrize("key,sign,axis", [("W", 1, "forward"), ("S", -1, "forward"),
                                           ("D", 1, "right"), ("A", -1, "right"),
                                           ("E", 1, "Y"), ("Q", -1, "Y")])
def test_keys_move_camera(key, sign, axis):
    c = _cam()
    p0 = c.position.copy()
    info = I.RuntimeInfo()
    info.key(key, True)
    assert I.update_camera_state(info, c, 0.25)
    v = rvcp_amd.scene.Y if axis == "Y" else getattr(c, axis)
    step = (v * f32(f32(c.move_speed) * f32(0.25))).astype(f32)
    exp = (p0 + step).astype(f32) if sign > 0 else (p0 - step).astype(f32)
    assert np.array_equal(c.position, exp)


def test_no_input_no_change():
    c = _cam()
    p0, f0 = c.position.copy(), c.forward.copy()
    info = I.RuntimeInfo()
    info.key("W", False)
    assert not I.update_camera_state(info, c, 1.0)
    assert np.array_equal(c.position, p0) and np.array_equal(c.forward, f0)


def test_mouse_rotation_and_pitch_clamp():
    c = _cam()
    info = I.RuntimeInfo(window_size=(384, 384))
    info.mouse_right(True)
    info.cursor(192 + 10, 192 - 4)               # right and up
    yaw0, pitch0 = c.yaw, c.pitch
    assert I.update_camera_state(info, c, 0.5)
    rv = f32(f32(c.rotate_speed) * f32(0.5))
    assert f32(c.yaw) == f32(f32(yaw0) + f32(f32(10) * rv))
    assert f32(c.pitch) == f32(f32(pitch0) + f32(f32(4) * rv))
    assert abs(float(np.linalg.norm(c.forward.astype(np.float64))) - 1.0) < 1e-6
    assert abs(float(np.dot(c.forward, c.right))) < 1e-6
    assert info.mouse_cur_position == (192.0, 192.0)          # cursor re-centred
    info.cursor(192, 192 - 100000)                             # huge upward drag
    I.update_camera_state(info, c, 1.0)
    assert c.pitch == 89.0
    info.cursor(192, 192 + 100000)
    I.update_camera_state(info, c, 1.0)
    assert c.pitch == -89.0


def test_zero_drag_keeps_direction():
    c = _cam()
    f0 = c.forward.copy()
    info = I.RuntimeInfo()
    info.mouse_right(True)                        # cursor at the centre: dx = dy = 0
    I.update_camera_state(info, c, 0.1)
    assert np.allclose(c.forward, f0, atol=1e-6)


def test_image_writers(tmp_path):
    rgba = np.random.default_rng(0).integers(0, 256, (5, 7, 4), dtype=np.uint8)
    I.write_ppm(str(tmp_path / "a.ppm"), rgba)
    assert np.array_equal(I.read_ppm(str(tmp_path / "a.ppm")), rgba[..., :3])
    I.write_png(str(tmp_path / "a.png"), rgba)
    data = (tmp_path / "a.png").read_bytes()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    idat = data.index(b"IDAT")
    n = int.from_bytes(data[idat - 4:idat], "big")
    raw = zlib.decompress(data[idat + 4:idat + 4 + n])
    rows = np.frombuffer(raw, dtype=np.uint8).reshape(5, 1 + 7 * 4)
    assert (rows[:, 0] == 0).all()
    assert np.array_equal(rows[:, 1:].reshape(5, 7, 4), rgba)


class _Recorder:
    """Stand-in for RayTracer on CPU: records the camera and time of every frame."""
    def __init__(self, scene):
        self.scene, self.calls = scene, []

    def render(self, w, h, t):
        self.calls.append((self.scene.camera.position.copy(), self.scene.camera.forward.copy(), t))
        return np.zeros((h, w, 4), dtype=np.uint8)


def test_headless_loop_scripted(tmp_path):
    sc = rvcp_amd.Scene.default()
    rec = _Recorder(sc)
    events = [(1, "key", ("W", True)), (3, "key", ("W", False)),
              (4, "mouse_right", (True,)), (4, "cursor", (40.0, 32.0)),
              (5, "mouse_right", (False,))]
    out = I.run_headless(rec, sc, 6, 64, 64, events=events, fixed_dt=0.1,
                         time_seed=lambda i: 100.0 + i, dump_dir=str(tmp_path), on_fps=lambda n: None)
    assert out["camera_moved"] == [False, True, True, False, True, False]
    pos = [c[0] for c in rec.calls]
    assert np.array_equal(pos[0], pos[1 - 1]) and not np.array_equal(pos[1], pos[0])
    assert np.array_equal(pos[3], pos[4]) and np.array_equal(pos[4], pos[5])
    assert not np.array_equal(rec.calls[4][1], rec.calls[3][1])     # rotated at frame 4
    assert [c[2] for c in rec.calls] == [100.0 + i for i in range(6)]
    assert sorted(os.listdir(tmp_path)) == [f"frame_{i:05d}.ppm" for i in range(6)]


def test_headless_loop_default_time_seed():
    sc = rvcp_amd.Scene.default()
    rec = _Recorder(sc)
    I.run_headless(rec, sc, 2, 8, 8, on_fps=lambda n: None)
    for _, _, t in rec.calls:                     # unix_secs % 1000 as f32 (vulkan.rs:418-421)
        assert 0.0 <= t < 1000.0 and f32(t) == t


@pytest.mark.gpu
def test_headless_loop_gpu_matches_oracle(tmp_path):
    sc = rvcp_amd.Scene.default()
    cfg = rvcp_amd.abi.make_config(spp=2)
    events = [(0, "key", ("W", True)), (2, "key", ("W", False)), (2, "key", ("D", True)),
              (3, "mouse_right", (True,)), (3, "cursor", (20.0, 40.0))]
    with rvcp_amd.RayTracer(cfg) as rt:
        rt.upload_scene(sc)
        out = I.run_headless(rt, sc, 5, 48, 40, events=events, fixed_dt=0.05,
                             time_seed=lambda i: 10.0 + i, dump_dir=str(tmp_path),
                             on_fps=lambda n: None)
        last = I.read_ppm(str(tmp_path / "frame_00004.ppm"))
    assert all(out["camera_moved"])
    _, o_rgba, _ = O.render(scene_arrays(sc), sc.push_constant(14.0), cfg, 48, 40)
    assert np.array_equal(last, o_rgba[..., :3])
