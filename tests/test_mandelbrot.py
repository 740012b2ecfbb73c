"""The Mandelbrot operator (assets/shaders/mandelbrot.comp) behind rvcp_mandelbrot.

CPU: the C oracle against a pure-Python float32 restatement of the shader on sampled pixels,
plus known answers (a point inside the set runs the full loop; a far point escapes at once).
GPU: librvcp bit-exact against the oracle (escape value bitwise, RGBA8 equal)."""
import numpy as np
import pytest

import oracle as O
import rvcp_amd

M = rvcp_amd.mandelbrot
F = np.float32


def _py_pixel(push, W, H, x, y):
    """mandelbrot.comp:12-33 in numpy float32 scalars, no contraction."""
    nx = F(F(F(x) + F(0.5)) / F(W))
    ny = F(F(F(y) + F(0.5)) / F(H))
    cx = F(F(nx - F(0.5)) * F(2.0))
    cy = F(F(ny - F(0.5)) * F(2.0))
    cx = F(F(cx / F(push["scale"])) + F(push["position"][0]))
    cy = F(F(cy / F(push["scale"])) + F(push["position"][1]))
    cx = F(cx - F(1.0))
    cy = F(cy - F(0.0))
    zx = zy = F(0.0)
    i = F(0.0)
    with np.errstate(all="ignore"):
        while i < F(1.0):
            nzx = F(F(F(zx * zx) - F(zy * zy)) + cx)
            nzy = F(F(F(zy * zx) + F(zx * zy)) + cy)
            zx, zy = nzx, nzy
            if F(np.sqrt(F(F(zx * zx) + F(zy * zy)))) > F(4.0):
                break
            i = F(i + F(0.005))
    return i


PUSHES = [M.Config().push_constant(),
          M.Config([0.3, -0.2], 3.5).push_constant(),
          M.Config([-0.74, 0.12], 40.0).push_constant()]


@pytest.mark.parametrize("k", range(len(PUSHES)))
def test_oracle_vs_python(k):
    push = PUSHES[k]
    W, H = 37, 29
    rgba, val = O.mandelbrot(push, W, H)
    rng = np.random.default_rng(k)
    for x, y in zip(rng.integers(0, W, 40), rng.integers(0, H, 40)):
        assert val[y, x].view(np.uint32) == _py_pixel(push, W, H, int(x), int(y)).view(np.uint32)
    u = np.array([O.unorm_u8(float(v)) for v in val.ravel()], dtype=np.uint8).reshape(H, W)
    assert np.array_equal(rgba[..., 0], u) and np.array_equal(rgba[..., 1], u)
    assert (rgba[..., 3] == 255).all()


def test_known_answers():
    push = M.Config().push_constant()
    # 2x2 frame: pixel centres at norm 0.25/0.75 -> c = (-1.5 or -0.5, -0.5 or 0.5)
    rgba, val = O.mandelbrot(push, 2, 2)
    assert val[0, 1] >= 1.0 and rgba[0, 1, 0] == 255           # c = (-0.5, -0.5): inside
    far = M.Config([100.0, 100.0], 1.0).push_constant()
    rgba, val = O.mandelbrot(far, 3, 3)
    assert (val == 0.0).all() and (rgba[..., :3] == 0).all()     # escapes on the first step


def test_keyboard_state():
    cfg = M.Config()
    assert not M.update_keyboard_state({}, cfg, 0.1)
    assert M.update_keyboard_state({"D": True, "E": True}, cfg, 0.1)
    assert cfg.camera_position[0] == float(F(F(F(1.0) * F(0.5)) * F(0.1)))
    assert cfg.camera_scale == float(F(F(1.0) + F(F(F(1.0) * F(0.5)) * F(0.1))))
    M.update_keyboard_state({"W": True}, cfg, 0.1)
    assert cfg.camera_position[1] < 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(PUSHES)))
@pytest.mark.parametrize("W,H", [(64, 64), (37, 29), (1, 1), (1000, 3)])
def test_gpu_bitexact(k, W, H):
    push = PUSHES[k]
    o_rgba, o_val = O.mandelbrot(push, W, H)
    with rvcp_amd.RayTracer(spp=1) as rt:
        rgba, val = rt.mandelbrot(push, W, H, want_value=True)
        assert rt.last_stats["kernel_ms"] > 0.0
        only = rt.mandelbrot(push, W, H)
    assert np.array_equal(val.view(np.uint32), o_val.view(np.uint32))
    assert np.array_equal(rgba, o_rgba) and np.array_equal(only, o_rgba)
