"""pyref -- a second, independent restatement of ray_tracer_games101_branch.comp in pure
Python with numpy float32 scalars (TEST INFRASTRUCTURE ONLY).

It exists to cross-check the C oracle (oracle/rvcp_oracle.c) bit for bit on small cases,
so that a slip in one restatement of the GLSL cannot hide behind the other.  It shares no
code with the oracle: only the numeric contract of DESIGN.md §3.  fma is computed exactly
with fractions (Python 3.10 has no math.fma).
"""
from __future__ import annotations

import ctypes
import ctypes.util
from fractions import Fraction

import numpy as np

# sample_ray's tan() is evaluated on the host once per frame by both the oracle and librvcp
# (C tanf); use the same libm function here.
_libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
_libm.tanf.argtypes = [ctypes.c_float]
_libm.tanf.restype = ctypes.c_float

F = np.float32
PI = F(3.1415926)


def f32_round(q: Fraction) -> np.float32:
    """Round an exact rational to the nearest float32 (ties to even)."""
    if q == 0:
        return F(0.0)
    neg = q < 0
    q = -q if neg else q
    e = q.numerator.bit_length() - q.denominator.bit_length()
    if Fraction(2) ** e > q:
        e -= 1
    ulp_e = max(e, -126) - 23
    m = q / (Fraction(2) ** ulp_e)
    fl = m.numerator // m.denominator
    rem = m - fl
    if rem > Fraction(1, 2) or (rem == Fraction(1, 2) and fl % 2 == 1):
        fl += 1
    val = float(fl) * 2.0 ** ulp_e          # exact in double
    r = F(val)
    return F(-r) if neg else r


def fma(a, b, c) -> np.float32:
    """float32 fma, one rounding.  a*b is exact in float64; the float64 sum's rounding error is
    recovered exactly (TwoSum), which settles the one case double rounding can get wrong: a
    float64 sum lying exactly on a float32 rounding midpoint."""
    a, b, c = float(a), float(b), float(c)
    p = a * b
    s = p + c
    r = F(s)
    if not np.isfinite(s) or float(r) == s:
        return r
    bp = s - p
    err = (p - (s - bp)) + (c - bp)
    if err == 0.0:
        return r
    other = np.nextafter(r, F(np.inf) if s > float(r) else F(-np.inf))
    if (float(r) + float(other)) * 0.5 == s:          # a midpoint: the lost error decides
        return other if (err > 0.0) == (float(other) > float(r)) else r
    return r


def fma_exact(a, b, c) -> np.float32:
    """fma by rational arithmetic (cross-check of fma above)."""
    return f32_round(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c)))


def sinf(x) -> np.float32:
    """DESIGN.md §3.2 software sin."""
    x = F(x)
    q = F(np.rint(F(x * F(float.fromhex("0x1.45f306p-2")))))
    r = fma(q, F(-float.fromhex("0x1.921fb6p+1")), x)
    r = fma(q, F(float.fromhex("0x1.777a5cp-24")), r)
    z = F(r * r)
    p = fma(fma(fma(F(float.fromhex("0x1.5dbdfep-19")), z, F(-float.fromhex("0x1.9f7p-13"))), z,
                F(float.fromhex("0x1.110ed4p-7"))), z, F(-float.fromhex("0x1.55554cp-3")))
    s = fma(p, F(z * r), r)
    odd = F(q - F(F(2.0) * F(np.floor(F(q * F(0.5))))))
    return F(-s) if odd != 0 else s


def fract(x):
    x = F(x)
    return F(x - F(np.floor(x)))


class Rng:
    def __init__(self, time, u, v):
        a = fract(F(sinf(time) * F(43758.5453)))
        b = fract(F(sinf(u) * F(22578.5453)))
        c = fract(F(sinf(v) * F(114514.1919)))
        self.seed = fract(F(F(a + b) + c))
        self.index = F(0.0)

    def __call__(self):
        self.index = F(self.index + F(1.0))
        return fract(F(sinf(F(self.seed + self.index)) * F(43758.5453)))


# ---- vec3 as tuples of float32 ----
def v(x, y, z):
    return (F(x), F(y), F(z))


def add(a, b): return (F(a[0] + b[0]), F(a[1] + b[1]), F(a[2] + b[2]))
def sub(a, b): return (F(a[0] - b[0]), F(a[1] - b[1]), F(a[2] - b[2]))
def mul(a, b): return (F(a[0] * b[0]), F(a[1] * b[1]), F(a[2] * b[2]))
def scale(a, s): return (F(a[0] * s), F(a[1] * s), F(a[2] * s))
def div(a, s): return (F(a[0] / s), F(a[1] / s), F(a[2] / s))
def neg(a): return (F(-a[0]), F(-a[1]), F(-a[2]))
# the builtins dot / cross as fused chains
def dot(a, b): return fma(a[2], b[2], fma(a[1], b[1], F(a[0] * b[0])))


def cross(a, b):
    return (fma(a[1], b[2], F(-F(a[2] * b[1]))), fma(a[2], b[0], F(-F(a[0] * b[2]))),
            fma(a[0], b[1], F(-F(a[1] * b[0]))))


def length(a): return F(np.sqrt(dot(a, a)))
def normalize(a): return scale(a, F(F(1.0) / F(np.sqrt(dot(a, a)))))


INF = (F(np.inf), F(np.inf), F(np.inf))


class Scene:
    def __init__(self, materials, vertices, faces, lum_ids, quirk=True, spheres=()):
        self.mat = [(tuple(F(x) for x in m["albedo"]), int(m["ty"])) for m in materials]
        names = getattr(getattr(materials, "dtype", None), "names", None) or ()
        self.fuzz = [F(m["fuzz"]) if "fuzz" in names else F(0) for m in materials]
        self.ior = [F(m["refraction_ratio"]) if "refraction_ratio" in names else F(1)
                    for m in materials]
        self.sph = [(tuple(F(x) for x in s_["center"]), F(s_["radius"]), int(s_["material_id"]))
                    for s_ in spheres]
        self.pos = [tuple(F(x) for x in vv["position"][:3]) for vv in vertices]
        self.nrm = [tuple(F(x) for x in vv["normal"][:3]) for vv in vertices]
        self.faces = [(tuple(int(i) for i in f["vertices"]), int(f["material_id"])) for f in faces]
        self.lum = [int(i) for i in lum_ids]
        self.quirk = quirk

    def lum_id(self, i):
        if not self.quirk:
            return self.lum[i]
        return self.lum[4 * i] if 4 * i < len(self.lum) else 0


def intersect(sc, o, d, tmin, tmax, face):
    (i0, i1, i2), mid = face
    v0, v1, v2 = sc.pos[i0], sc.pos[i1], sc.pos[i2]
    e1, e2, s = sub(v1, v0), sub(v2, v0), sub(o, v0)
    s1, s2 = cross(d, e2), cross(s, e1)
    with np.errstate(all="ignore"):
        f = F(F(1.0) / dot(s1, e1))
        t = F(f * dot(s2, e2))
        b1 = F(f * dot(s1, s))
        b2 = F(f * dot(s2, d))
    if b1 < 0 or 1 < b1 or b2 < 0 or 1 < b2 or 1 < F(b1 + b2):
        return None
    if t < tmin or tmax < t:
        return None
    w0 = F(F(F(1.0) - b1) - b2)
    n = normalize(add(add(scale(sc.nrm[i0], w0), scale(sc.nrm[i1], b1)), scale(sc.nrm[i2], b2)))
    pos = add(o, scale(d, t))
    if dot(n, d) > 0:
        return t, pos, neg(n), mid, False
    return t, pos, n, mid, True


def scene_hit(sc, o, d, tmin, tmax, counter):
    counter[0] += 1
    best = (F(tmax + F(1.0)), INF, (F(0), F(0), F(0)), 0, True)
    for f in sc.faces:
        h = intersect(sc, o, d, tmin, tmax, f)
        if h is not None and h[0] <= tmax:
            tmax = h[0]
            best = h
    return best


def face_area(sc, fid):
    (i0, i1, i2), _ = sc.faces[fid]
    v0, v1, v2 = sc.pos[i0], sc.pos[i1], sc.pos[i2]
    return F(F(0.5) * length(cross(sub(v1, v0), sub(v2, v0))))


def trace(sc, P, g, o, d, tmin, tmax, counter):
    color = v(0, 0, 0)
    att = v(1, 1, 1)
    for depth in range(P["max_bounces"]):
        if att[0] < P["att_stop"] and att[1] < P["att_stop"] and att[2] < P["att_stop"]:
            break
        t, p, n, mid, _ = scene_hit(sc, o, d, tmin, tmax, counter)
        if t > tmax:
            color = add(color, v(0.1, 0.1, 0.1))
            break
        alb, ty = sc.mat[mid]
        if ty == 3:
            if depth == 0:
                color = add(color, mul(att, alb))
            break
        nl = len(sc.lum)
        if nl:
            S = F(0.0)
            for i in range(nl):
                S = F(S + face_area(sc, sc.lum_id(i)))
            pl = F(g() * S)
            pdf = F(F(1.0) / S)
            acc = F(0.0)
            chosen = None
            for i in range(nl):
                fid = sc.lum_id(i)
                acc = F(acc + face_area(sc, fid))
                if pl <= acc:
                    chosen = fid
                    break
            if chosen is not None:
                (j0, j1, j2), lmid = sc.faces[chosen]
                x = F(np.sqrt(g()))
                y = g()
                X = add(add(scale(sc.pos[j0], F(F(1.0) - x)), scale(sc.pos[j1], F(x * F(F(1.0) - y)))),
                        scale(sc.pos[j2], F(x * y)))
                Xn = normalize(sc.nrm[j0])
                dist = length(sub(X, p))
                ws = div(sub(X, p), dist)
                _, bp, _, _, _ = scene_hit(sc, add(p, scale(ws, P["eps"])), ws, P["t_min"], P["t_max"],
                                        counter)
                db = length(sub(bp, p))
                if abs(F(dist - db)) < P["eps"]:
                    fb = div(alb, PI) if dot(n, ws) > 0 else v(0, 0, 0)
                    c = mul(mul(att, sc.mat[lmid][0]), fb)
                    c = scale(c, dot(n, ws))
                    c = scale(c, dot(Xn, neg(ws)))
                    c = div(c, F(F(dist * dist) * pdf))
                    color = add(color, c)
        if g() > P["rr"]:
            break
        while True:
            q = (F(F(F(2.0) * g()) - F(1.0)), F(F(F(2.0) * g()) - F(1.0)),
                 F(F(F(2.0) * g()) - F(1.0)))
            if not dot(q, q) >= 1.0:
                break
        h = q if dot(q, n) > 0 else neg(q)
        wi = normalize(h)
        fb = div(alb, PI) if dot(n, wi) > 0 else v(0, 0, 0)
        pdf_b = F(F(0.5) / PI) if dot(wi, n) > 0 else F(0.0)
        a = div(scale(fb, dot(n, wi)), F(max(F(0.1), pdf_b) * P["rr"]))
        att = mul(att, a)
        o, d, tmin, tmax = add(p, scale(wi, P["eps"])), wi, P["t_min"], P["t_max"]
    return color


# ---- integrator mode 2: ray_tracer.comp ----
def sphere_hit(o, d, tmin, tmax, sph):
    """is_intersect_with_sphere + is_intersect_with_quadratic_equation (ray_tracer.comp:260-321)."""
    ce, r, mid = sph
    co = sub(o, ce)
    a = dot(d, d)
    b = F(F(2.0) * dot(d, co))
    c = F(dot(co, co) - F(r * r))
    with np.errstate(all="ignore"):
        delta = F(F(b * b) - F(F(F(4.0) * a) * c))
        if delta < 0:
            return None
        sq = F(np.sqrt(delta))
        t0 = F(F(F(-b) + sq) / F(F(2.0) * a))
        t1 = F(F(F(-b) - sq) / F(F(2.0) * a))
    if t0 > t1:
        t0, t1 = t1, t0
    if tmin <= t0 <= tmax:
        t = t0
    elif tmin <= t1 <= tmax:
        t = t1
    else:
        return None
    pos = add(o, scale(d, t))
    n = normalize(sub(pos, ce))
    if dot(co, co) < F(r * r):
        return t, pos, neg(n), mid, False
    return t, pos, n, mid, True


def scene_hit_legacy(sc, o, d, tmin, tmax, counter):
    """get_intersection_with_scene, ray_tracer.comp:369-393 (spheres, then faces)."""
    counter[0] += 1
    best = (F(tmax + F(1.0)), INF, (F(0), F(0), F(0)), 0, True)
    for s_ in sc.sph:
        h = sphere_hit(o, d, tmin, tmax, s_)
        if h is not None and h[0] <= tmax:
            tmax, best = h[0], h
    for f in sc.faces:
        h = intersect(sc, o, d, tmin, tmax, f)
        if h is not None and h[0] <= tmax:
            tmax, best = h[0], h
    return best


def unit_sphere(g):
    while True:
        q = (F(F(F(2.0) * g()) - F(1.0)), F(F(F(2.0) * g()) - F(1.0)), F(F(F(2.0) * g()) - F(1.0)))
        if not dot(q, q) >= 1.0:
            return q


def reflect(i, n):
    return sub(i, scale(n, F(F(2.0) * dot(n, i))))


def refract(i, n, eta):
    d = dot(n, i)
    k = F(F(1.0) - F(F(eta * eta) * F(F(1.0) - F(d * d))))
    if k < 0:
        return v(0, 0, 0)
    return sub(scale(i, eta), scale(n, F(F(eta * d) + F(np.sqrt(k)))))


def trace_legacy(sc, P, g, o, d, tmin, tmax, counter):
    """ray_trace, ray_tracer.comp:618-694, with material_scatter :491-602."""
    color = v(0, 0, 0)
    att = v(1, 1, 1)
    for _ in range(P["max_bounces"]):
        t, p, n, mid, outward = scene_hit_legacy(sc, o, d, tmin, tmax, counter)
        if t > tmax:
            color = add(color, mul(att, v(0, 0, 0)))
            break
        alb, ty = sc.mat[mid]
        if ty == 3:
            color = add(color, mul(att, alb))
            break
        na, nd = v(0, 0, 0), v(0, 0, 0)
        if ty == 0:
            nd = normalize(add(n, normalize(unit_sphere(g))))
            if all(abs(c) < P["eps"] for c in nd):
                nd = n
            na = alb
        elif ty == 1:
            r = reflect(d, n)
            if dot(r, n) < 0:
                r = neg(r)
            while True:
                nd = normalize(add(r, scale(normalize(unit_sphere(g)), sc.fuzz[mid])))
                if not dot(nd, n) < 0:
                    break
            na = alb
        elif ty == 2:
            ratio = F(F(1.0) / sc.ior[mid]) if outward else sc.ior[mid]
            ct = dot(neg(d), n)
            with np.errstate(all="ignore"):
                st = F(np.sqrt(F(F(1.0) - F(ct * ct))))
            refr = F(ratio * st) <= 1.0
            if refr:
                r0 = F(F(F(1.0) - ratio) / F(F(1.0) + ratio))
                r0 = F(r0 * r0)
                x = F(F(1.0) - ct)
                fr = F(r0 + F(F(F(1.0) - r0) * F(F(F(x * x) * F(x * x)) * x)))
                refr = g() >= fr
            nd = refract(d, n, ratio) if refr else reflect(d, n)
            na = v(1, 1, 1)
        att = mul(att, na)
        o, d, tmin, tmax = add(p, scale(nd, P["t_min"])), nd, P["t_min"], P["t_max"]
        if all(c < P["eps"] for c in att):
            break
        if g() >= P["rr"]:
            break
        att = div(att, P["rr"])
    return color


def render_pixel(sc, P, push, W, H, x, y):
    """Linear RGB of pixel (x, y) and the traversal count."""
    cam = push["camera"]
    cpos = tuple(F(c) for c in cam["position"][:3])
    up = tuple(F(c) for c in cam["up"][:3])
    fwd = tuple(F(c) for c in cam["forward"])
    tn, tf, fov = F(cam["t_near"]), F(cam["t_far"]), F(cam["vertical_fov"])
    u_ = F(F(F(x) + F(0.5)) / F(W))
    v_ = F(F(F(y) + F(0.5)) / F(H))
    g = Rng(F(push["time"]), u_, v_)
    rad = F(F(F(fov / F(2.0)) * PI) / F(180.0))
    h = F(F(F(2.0) * tn) * F(_libm.tanf(float(rad))))
    w = F(F(h * F(W)) / F(H))
    uu = scale(normalize(cross(fwd, up)), w)
    vv = scale(normalize(cross(fwd, uu)), h)
    pos = add(cpos, scale(fwd, tn))
    uvp = add(add(pos, scale(uu, F(u_ - F(0.5)))), scale(vv, F(v_ - F(0.5))))
    tc = F(length(sub(uvp, cpos)) / length(sub(pos, cpos)))
    d = normalize(sub(uvp, cpos))
    counter = [0]
    color = v(0, 0, 0)
    if P.get("integrator", 0) == 1:
        for _ in range(P["spp"]):
            color = add(color, trace_legacy(sc, P, g, cpos, d, F(tn * tc), F(tf * tc), counter))
        return div(color, F(P["spp"])), counter[0]
    for _ in range(P["spp"]):
        L = trace(sc, P, g, cpos, d, F(tn * tc), F(tf * tc), counter)
        color = add(color, div(L, F(P["spp"])))
    return color, counter[0]


def params(cfg):
    return dict(spp=int(cfg["spp"]), max_bounces=int(cfg["max_bounces"]),
                att_stop=F(cfg["attenuation_stop_eps"]), t_min=F(cfg["ray_t_min"]),
                t_max=F(cfg["ray_t_max"]), rr=F(cfg["rr_probability"]), eps=F(cfg["eps"]),
                integrator=int(cfg["integrator"]))
