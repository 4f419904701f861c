"""The render's exact contribution culling (csrc/render.hip cull_setup / cull_box_may_hit, ABI v9) restated in
numpy float32 and checked for conservativeness on CPU: whenever the predicate drops a (Gaussian, pixel box) pair,
the per-pixel test of the rasterizer (gsplat v0.1.11 rasterize_forward: sigma = 0.5 (a dx^2 + c dy^2) + b dx dy,
alpha = min(0.999, o exp(-sigma)), skipped when sigma < 0 or alpha < 1/255) fails at every pixel centre of the box.
The device code itself is checked on the GPU by bit-identity of culled and full renders (tests/test_gpu_render.py,
tests/test_gpu_full.py); this pins the geometry of the bound, including adversarial draws near its thresholds."""
import numpy as np

f32 = np.float32


def cull_setup(x, y, a, b, c, o):
    ac = f32(a) * f32(c)
    if not (a > 0 and c > 0 and b * b < f32(0.9801) * ac and np.isfinite(x) and np.isfinite(y) and np.isfinite(ac)):
        return ("always",)
    if not (f32(o) * f32(255) >= f32(0.999)):
        return ("never",) if f32(o) * f32(255) < f32(0.999) else ("always",)
    rho = np.sqrt(f32(b * b / ac))
    lim = (np.log(f32(o) * f32(255)) + f32(2e-4)) / (f32(1) - f32(1e-4) / (f32(1) - rho))
    return ("box", f32(x), f32(y), f32(a), f32(b), f32(c), f32(1) / f32(a), f32(1) / f32(c), f32(lim))


def may_hit(g, px0, px1, py0, py1):
    if g[0] == "always":
        return True
    if g[0] == "never" or px0 > px1 or py0 > py1:
        return False
    _, gx, gy, a, b, c, ia, ic, lim = g
    u0, u1 = gx - (f32(px1) + f32(0.5)), gx - (f32(px0) + f32(0.5))
    v0, v1 = gy - (f32(py1) + f32(0.5)), gy - (f32(py0) + f32(0.5))
    if u0 <= 0 and u1 >= 0 and v0 <= 0 and v1 >= 0:
        return True
    m = f32(3e38)
    for dx in (u0, u1):
        dy = min(max(-b * dx * ic, v0), v1)
        m = min(m, f32(0.5) * (a * dx * dx + c * dy * dy) + b * dx * dy)
    for ey in (v0, v1):
        ex = min(max(-b * ey * ia, u0), u1)
        m = min(m, f32(0.5) * (a * ex * ex + c * ey * ey) + b * ex * ey)
    return bool(m <= lim)


def any_pixel_contributes(x, y, a, b, c, o, px0, px1, py0, py1):
    px = np.arange(px0, px1 + 1, dtype=f32) + f32(0.5)
    py = np.arange(py0, py1 + 1, dtype=f32) + f32(0.5)
    dx = (f32(x) - px)[None, :]
    dy = (f32(y) - py)[:, None]
    sigma = f32(0.5) * (f32(a) * dx * dx + f32(c) * dy * dy) + f32(b) * dx * dy
    alpha = np.minimum(f32(0.999), f32(o) * np.exp(-sigma, dtype=f32))
    return bool(((sigma >= 0) & (alpha >= f32(1.0 / 255.0))).any())


def test_cull_bound_is_conservative():
    rng = np.random.default_rng(7)
    dropped = 0
    for it in range(6000):
        # conic from a random 2x2 covariance: radii 0.3 .. 60 px, any orientation, some near-degenerate
        s1, s2 = np.exp(rng.uniform(np.log(0.3), np.log(60.0), 2))
        if it % 5 == 0:
            s2 = s1 * rng.uniform(1e-3, 3e-2)  # needles
        th = rng.uniform(0, np.pi)
        R = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
        cov = R @ np.diag([s1 * s1, s2 * s2]) @ R.T + 0.3 * np.eye(2)
        inv = np.linalg.inv(cov)
        a, b, c = f32(inv[0, 0]), f32(inv[0, 1]), f32(inv[1, 1])
        o = f32(np.exp(rng.uniform(np.log(1 / 255.0 * 0.98), 0.0)))
        if it % 7 == 0:
            o = f32(1 / 255.0 * (1 + rng.uniform(-2e-4, 2e-4)))  # at the threshold
        px0, py0 = int(rng.integers(0, 64)) * 8, int(rng.integers(0, 64)) * 8
        w = 8 if it % 2 else 16
        x = f32(px0 + rng.uniform(-3 * s1, w + 3 * s1))
        y = f32(py0 + rng.uniform(-3 * s1, w + 3 * s1))
        g = cull_setup(x, y, a, b, c, o)
        if not may_hit(g, px0, px0 + w - 1, py0, py0 + w - 1):
            dropped += 1
            assert not any_pixel_contributes(x, y, a, b, c, o, px0, px0 + w - 1, py0, py0 + w - 1), (
                it, x, y, a, b, c, o, px0, py0, w)
    assert dropped > 1000  # the bound does cull


def test_cull_bound_degenerate_inputs_kept():
    assert cull_setup(1.0, 2.0, 1.0, 1.0, 1.0, 0.5) == ("always",)        # rho = 1
    assert cull_setup(1.0, 2.0, -1.0, 0.0, 1.0, 0.5) == ("always",)       # not PD
    assert cull_setup(np.nan, 2.0, 1.0, 0.0, 1.0, 0.5) == ("always",)     # non-finite position
    assert cull_setup(1.0, 2.0, 1.0, 0.0, 1.0, np.nan) == ("always",)     # NaN opacity
    assert cull_setup(1.0, 2.0, 1.0, 0.0, 1.0, 0.5 / 255) == ("never",)   # below 1/255 everywhere
