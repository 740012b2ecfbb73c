"""The shadow rays' early end (shadow_stop, csrc/rvcp_kernels.hip) against
a float32 model of resolve A (ray_tracer_games101_branch.comp:438-449 as the kernel computes it):
for a hit at any t <= stop, the computed |hp - p| must leave the light sample blocked,
|dist - |hp - p|| >= eps, so the first such hit decides the sample as the nearest one would.
Random shading points, light points, directions and eps over scene scales 2^-20 .. 2^38 (the
fuzz suite's range), checked at t = stop itself (the boundary) and at random t below it."""
import numpy as np
import pytest

f32 = np.float32


def _fma(a, b, c):
    # float32 fma via float64 (the product of two float32 is exact in float64; the sum rounds
    # once there and once to float32 -- a double rounding the bound's 4x margin absorbs)
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(f32)


def _dot(a, b):       # the kernel's dot: fma(z, z', fma(y, y', x * x'))
    return _fma(a[..., 2], b[..., 2], _fma(a[..., 1], b[..., 1], (a[..., 0] * b[..., 0]).astype(f32)))


def _stop(eps, p, dist):
    M = (np.max(np.abs(p), axis=-1) + eps).astype(f32)
    M = (M + dist).astype(f32)
    marg = (f32(2.0 ** -18) * ((M + dist).astype(f32) + eps).astype(f32)).astype(f32)
    return ((dist - (f32(2.0) * eps).astype(f32)).astype(f32) - marg).astype(f32)


@pytest.mark.parametrize("e", [-20, -6, 0, 9, 20, 30, 38])
def test_hits_below_stop_are_blocked(e):
    rng = np.random.default_rng(1000 + e)
    n = 200000
    s = 2.0 ** e
    off = rng.choice([0.0, 1.0], n)[:, None] * rng.uniform(-1, 1, (n, 3)) * s * 2.0 ** 10
    p = (rng.uniform(-1, 1, (n, 3)) * s + off).astype(f32)
    X = (p.astype(np.float64) + rng.uniform(-1, 1, (n, 3)) * s * rng.uniform(1e-3, 1, (n, 1))).astype(f32)
    dv = (X - p).astype(f32)
    dist = np.sqrt(_dot(dv, dv)).astype(f32)
    ok = dist > 0
    ws = (dv / dist[:, None]).astype(f32)
    eps = np.where(rng.random(n) < 0.5, f32(1e-3), (f32(1e-3) * f32(s)).astype(f32)).astype(f32)
    stop = _stop(eps, p, dist)
    a_o = (p + (ws * eps[:, None]).astype(f32)).astype(f32)
    for t in (stop, (stop * rng.random(n).astype(f32)).astype(f32)):
        sel = ok & (t >= 0)
        hp = (a_o + (ws * t[:, None]).astype(f32)).astype(f32)
        diff = (hp - p).astype(f32)
        db = np.sqrt(_dot(diff, diff)).astype(f32)
        visible = np.abs((dist - db).astype(f32)) < eps
        assert not np.any(visible & sel), f"scale 2^{e}: {int(np.sum(visible & sel))} visible"
        assert np.sum(sel) > n // 4
