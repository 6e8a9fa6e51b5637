"""The CPU oracle (oracle/libptoracle.so) against known answers.

The reference's radiance cannot be produced in this container (GLSL needs a WebGL context; none
exists here) and the reference ships no tests, so radiance parity vs the GLSL render is
"parity unpinned" (DESIGN.md §Parity). What is pinned here:
  * integer / exact pieces: rng() (js/PathTracingCommon.js:500-508) against an independent Python
    evaluation of the same uint32 recurrence; blue-noise texel addressing;
  * the pinned transcendental built-ins against float64 truth within a few ulp;
  * structural facts of the restated program (row-range independence, frame-1 history clear,
    moving-camera blend, alpha/sharpness flags, screenOutput on constant images).
"""
import math

import numpy as np
import pytest

import helpers as H
import ptoracle as po


def rng_reference(s0, s1, n):
    """uvec2 seed; seed += 1; q = K*((seed>>1)^seed.yx); n = K*(q.x^(q.y>>3)); float(n)/2^32."""
    K, M = 1103515245, 0xFFFFFFFF
    out = []
    for _ in range(n):
        s0, s1 = (s0 + 1) & M, (s1 + 1) & M
        qx = (K * ((s0 >> 1) ^ s1)) & M
        qy = (K * ((s1 >> 1) ^ s0)) & M
        v = (K * (qx ^ (qy >> 3))) & M
        out.append(np.float32(v) * np.float32(2.0 ** -32))
    return np.array(out, np.float32)


def test_rng_known_answers():
    seeds = [(0, 0), (1, 2), (1919, 2158), (7 * 1000, 8 * 999), (0xFFFFFFF0 & 0xFFFFFF, 12345)]
    for s0, s1 in seeds:
        ref = rng_reference(s0, s1, 1)
        got = po.math_probe(11, np.array([s0], np.float32), np.array([s1], np.float32))
        assert got.view(np.uint32)[0] == ref.view(np.uint32)[0]


def _ulp_err(got, ref):
    got = got.astype(np.float64)
    ulp = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    return np.abs(got - ref) / ulp


@pytest.mark.parametrize("op,fn,lo,hi,tol", [
    (0, lambda x: np.exp2(x), -20, 20, 4),
    (1, lambda x: np.log2(x), 1e-3, 1e3, 4),
    (2, np.sin, 0.0, 2 * math.pi, 4),
    (3, np.cos, 0.0, 2 * math.pi, 4),
    (4, np.arctan, -20, 20, 4),
    (8, np.exp, -20, 20, 24),   # exp2(x*log2e): the rounded product costs |x|*2^-24 relative
    (9, np.log, 1e-3, 1e3, 8),
])
def test_pinned_math_accuracy(op, fn, lo, hi, tol):
    x = np.random.default_rng(op).uniform(lo, hi, 200000).astype(np.float32)
    got = po.math_probe(op, x)
    ref = fn(x.astype(np.float64))
    err = _ulp_err(got, ref)
    # absolute error floor near zero crossings of sin/cos/log
    ok = (err <= tol) | (np.abs(got - ref) < 2e-7)
    assert ok.all(), "max ulp %g" % err[~ok].max()


def test_pinned_math_edges():
    inf, nan = np.float32(np.inf), np.float32(np.nan)
    assert po.math_probe(0, np.array([200.0, -200.0, 0.0], np.float32)).tolist() == [np.inf, 0.0, 1.0]
    r = po.math_probe(1, np.array([0.0, -1.0, 1.0, np.inf], np.float32))
    assert r[0] == -np.inf and np.isnan(r[1]) and r[2] == 0.0 and r[3] == np.inf
    p = po.math_probe(7, np.array([0.0, 1.0, 4.0], np.float32), np.array([2.2, 0.4545, 0.5], np.float32))
    assert p[0] == 0.0 and p[1] == 1.0 and abs(p[2] - 2.0) < 1e-6
    a = po.math_probe(6, np.array([1.0, -1.0, 0.0, 1.5], np.float32))
    assert a[0] == 0.0 and abs(a[1] - math.pi) < 1e-6 and abs(a[2] - math.pi / 2) < 1e-6 and np.isnan(a[3])
    t = po.math_probe(5, np.array([1.0, -1.0, 0.0], np.float32), np.array([0.0, -1.0, -1.0], np.float32))
    assert abs(t[0] - math.pi / 2) < 1e-6 and abs(t[1] + 3 * math.pi / 4) < 1e-6 and abs(t[2] - math.pi) < 1e-6


def test_row_ranges_compose():
    """Rendering row bands separately (the multi-GPU split) equals one full-frame pass."""
    meta = H.stream("gltf_teapot_320x180")
    sc = H.oracle_scene(meta)
    u = H.path_call(meta["frames"][0])["uniforms"]
    prev = np.zeros((180, 320, 4), np.float32)
    full, _ = sc.path_trace(u, prev)
    parts = np.zeros_like(full)
    for r0 in range(0, 180, 16):
        out, _ = sc.path_trace(u, prev, r0, min(180, r0 + 16))
        parts[r0:r0 + 16] = out[r0:r0 + 16]
    assert np.array_equal(full.view(np.uint32), parts.view(np.uint32))


def test_history_semantics():
    """uFrameCounter == 1 clears history; uCameraIsMoving halves both; otherwise sum
    (js/PathTracingCommon.js:1326-1357)."""
    meta = H.stream("cornell_256")
    sc = H.oracle_scene(meta)
    u = dict(H.path_call(meta["frames"][1])["uniforms"])   # frame 2, not moving
    junk = np.random.default_rng(0).uniform(0, 5, (256, 256, 4)).astype(np.float32)
    junk[..., 3] = 0.0
    zero = np.zeros_like(junk)
    cur, _ = sc.path_trace(u, zero)
    summed, _ = sc.path_trace(u, junk)
    assert np.allclose(summed[..., :3], junk[..., :3] + cur[..., :3], rtol=0, atol=0)
    u1 = dict(u, uFrameCounter=["f", [1.0]])
    cleared, _ = sc.path_trace(u1, junk)
    fresh, _ = sc.path_trace(u1, zero)
    assert np.array_equal(cleared, fresh)
    um = dict(u, uCameraIsMoving=["i", [1]])
    moving, _ = sc.path_trace(um, junk)
    assert np.array_equal(moving[..., :3], np.float32(0.5) * junk[..., :3] + np.float32(0.5) * cur[..., :3])


def test_sharpness_flags_reach_alpha():
    meta = H.stream("cornell_256")
    accs, _, _ = H.oracle_replay(meta, 2)
    a = accs[-1][..., 3]
    vals = set(np.unique(a).tolist())
    assert vals <= {0.0, np.float32(1.01).item(), -1.0}
    assert (a == np.float32(1.01)).mean() > 0.01     # edges + directly seen light


def test_screen_output_constant_image():
    """Uniform image, alpha 0: every filter tap is taken, result = Reinhard(x/N)^0.4545."""
    acc = np.zeros((16, 16, 4), np.float32)
    acc[..., :3] = 3.0
    out = po.screen_output(acc, 0.5, 1.0)
    v = 1.5 / 2.5
    expect = int(math.floor((v ** 0.4545) * 255 + 0.5))
    # the interior sees 25 equal taps; the 2-pixel border sees zero-valued out-of-range taps
    assert abs(int(out[8, 8, 0]) - expect) <= 1
    assert out[8, 8, 3] == 255
    assert out[0, 0, 0] < out[8, 8, 0]


def test_bunny_counts_plausible():
    """Primary+secondary rays at the default bunny camera: the model is small in frame, so most
    segments test only the root box (SURVEY.md §8a12 probe: ~2% of primary rays hit it)."""
    meta = H.stream("gltf_bunny_1080p")
    sc = H.oracle_scene(meta)
    u = H.path_call(meta["frames"][0])["uniforms"]
    _, cnt = sc.path_trace(u, np.zeros((1080, 1920, 4), np.float32), 500, 600)
    assert cnt["stack_overflow"] == 0
    assert cnt["paths"] == 100 * 1920
    assert 1.5 < cnt["segments"] / cnt["paths"] < 4.0
    assert cnt["node_fetches"] >= cnt["segments"]


def _sky_f64(sun, d):
    """Get_Sky_Color (js/PathTracingCommon.js:373-475) transcribed in float64 numpy: an independent
    check of the oracle's f32 restatement (formula and constants), not of its rounding."""
    sun = np.asarray(sun, np.float64)
    d = np.asarray(d, np.float64)
    d = d / np.linalg.norm(d, axis=1, keepdims=True)
    up = np.array([0.0, 1.0, 0.0])
    cos_vs = d @ sun
    cos_su = up @ sun
    z = np.clip(cos_su, -1.0, 1.0)
    sunE = 200.0 * max(0.0, 1.0 - np.e ** (-((1.6110731556870734 - np.arccos(z)) / 1.5)))
    rayleigh = np.array([5.804542996261093E-6, 1.3562911419845635E-5, 3.0265902468824876E-5]) * 2.0
    mie = 0.434 * (0.2 * 0.5) * 10E-18 * np.array([1.8399918514433978E14, 2.7798023919660528E14, 4.0790479543861094E14]) * 0.03
    zen = np.arccos(np.maximum(0.0, d[:, 1]))
    inv = 1.0 / (np.cos(zen) + 0.15 * (93.885 - zen * 180.0 / np.pi) ** -1.253)
    fex = np.exp(-(rayleigh[None] * (8400.0 * inv)[:, None] + mie[None] * (1250.0 * inv)[:, None]))
    br = rayleigh[None] * (0.05968310365946075 * (1.0 + (cos_vs * 0.5 + 0.5) ** 2))[:, None]
    g = 0.76
    hg = 0.07957747154594767 * (1 - g * g) / np.maximum(0.0, 1 - 2 * g * cos_vs + g * g) ** 1.5
    bm = mie[None] * hg[:, None]
    q = sunE * (br + bm) / (rayleigh + mie)[None]
    lin = (q * (1 - fex)) ** 1.5
    t = np.clip((1.0 - cos_su) ** 5, 0, 1)
    lin = lin * ((1 - t) + (q * fex) ** 0.5 * t)
    x = np.clip((cos_vs - 0.9998) / 0.00002, 0, 1)
    sundisk = x * x * (3 - 2 * x)
    l0 = 0.1 * fex + sunE * 19000.0 * fex * sundisk[:, None]
    tex = (lin + l0) * 0.04 + np.array([0.0, 0.0003, 0.00075])
    sunfade = 1.0 - np.clip(1.0 - np.exp(sun[1] / 450000.0), 0, 1)
    return tex ** (1.0 / (1.2 + 1.2 * sunfade))


def test_sky_color_matches_float64_transcription():
    sun = np.array(H.path_call(H.stream("sky_256")["frames"][0])["uniforms"]["uSunDirection"][1], np.float32)
    rng = np.random.default_rng(7)
    d = rng.normal(size=(4096, 3)).astype(np.float32)
    d[:64] = sun + rng.normal(scale=0.004, size=(64, 3)).astype(np.float32)   # around the sun disk
    got = po.sky_color(sun, d).astype(np.float64)
    want = _sky_f64(sun.astype(np.float64), d.astype(np.float64))
    assert np.all(np.isfinite(got))
    np.testing.assert_allclose(got, want, rtol=2e-4, atol=1e-6)


def test_sky_scene_properties():
    """Physical-sky scene (js/PhysicalSkyModel_FragmentShader.js): rays that see the sky directly are
    sharp (alpha 1.01) and every pixel is lit (no quad light: the sun lobe and the sky light it)."""
    meta = H.stream("sky_256")
    accs, cans, cnts = H.oracle_replay(meta, 1, with_output=True)
    a = accs[0]
    assert np.all(np.isfinite(a))
    assert (a[..., 3] == np.float32(1.01)).mean() > 0.05
    assert a[..., :3].min() >= 0.0 and a[..., :3].mean() > 0.1
    assert cnts[0]["node_fetches"] == 0 and cnts[0]["segments"] > cnts[0]["paths"]


def _implicit(shape, k, p):
    """Residual of each unit shape's surface at p (js/PathTracingCommon.js:690-1163), float64."""
    x, y, z = p[:, 0], p[:, 1], p[:, 2]
    r2 = x * x + z * z
    if shape == 0:
        return np.abs(x * x + y * y + z * z - 1)
    if shape == 1:
        return np.abs(r2 - 1)
    if shape in (2, 8):
        kk = min(max(k, 0.01), 1.0)
        j, h = 1 / kk, 2 / kk - 1
        if shape == 2:
            return np.abs(j * r2 - kk * 0.25 * (y - h) ** 2)
        fx = np.abs(j * x * x - kk * 0.25 * (y - h) ** 2)
        fz = np.abs(j * z * z - kk * 0.25 * (y - h) ** 2)
        return np.minimum(fx, fz)
    if shape == 3:
        return np.abs(r2 + 0.5 * (y - 1))
    if shape == 4:
        K = (k ** 4 + 0.0012) * 1000
        return np.abs(K * r2 - (K - 1) * y * y - 1) / K
    if shape == 5:
        kk = k + 0.25
        cyl = np.abs(r2 - 1)
        cap = np.minimum(np.abs(r2 + (y - kk) ** 2 - 1), np.abs(r2 + (y + kk) ** 2 - 1))
        return np.where(np.abs(y) <= kk, cyl, cap)
    if shape == 6:
        kk = k - 0.01
        return np.minimum.reduce([np.abs(r2 - 1), np.abs(r2 - kk), np.abs(np.abs(y) - 1)])
    if shape == 7:
        return np.abs(np.maximum.reduce([np.abs(x), np.abs(y), np.abs(z)]) - 1)
    if shape in (9, 10):
        return np.abs(y)
    kk = 1 - min(max(k, 0.01), 0.99)
    return np.abs(np.hypot(np.sqrt(r2) - (1 - kk), y) - kk)


@pytest.mark.parametrize("shape", range(12))
def test_quadric_intersectors_hit_their_surfaces(shape):
    """Each restated intersector returns points on its shape's implicit surface (a transcription
    check independent of rounding: sign or term errors would move the hits off the surface)."""
    rng = np.random.default_rng(shape)
    n = 4000
    target = rng.uniform(-0.9, 0.9, (n, 3))
    ro = target + rng.normal(size=(n, 3)) * 4.0
    rd = target - ro
    k = 0.6
    t, _ = po.quadric_probe(shape, k, ro, rd)
    hit = t < 1e6
    assert hit.mean() > 0.05
    p = ro[hit].astype(np.float64) + rd[hit].astype(np.float64) * t[hit, None].astype(np.float64)
    tol = 0.02 if shape == 11 else 2e-3   # the torus is ray-marched to |d| < 0.01
    assert np.quantile(_implicit(shape, k, p), 0.99) < tol


def test_screen_output_bypass_thresholds():
    """The two bypasses of js/PathTracingCommon.js:293-296 switch on where the GPU test
    (test_screen_output_sample_count_branches) places N: from N = 201 (1/N < 0.005) a sharp pixel
    (a = 1.01) no longer sees its neighbours, from N = 5001 (1/N < 0.0002) no pixel does."""
    rs = np.random.RandomState(3)
    acc = np.zeros((24, 24, 4), np.float32)
    acc[..., :3] = rs.uniform(0, 50, (24, 24, 3)).astype(np.float32)
    acc[..., 3] = rs.choice(np.array([0.0, 1.01, -1.0], np.float32), (24, 24))
    acc[12, 12, 3] = np.float32(1.01)    # a sharp pixel
    acc[12, 6, 3] = 0.0                  # a filtered one
    other = acc.copy()
    other[10:15, 10:15, :3] += 7.0       # its neighbourhoods change, the pixels themselves do not
    other[12, 12, :3] = acc[12, 12, :3]
    other[10:15, 4:9, :3] += 7.0
    other[12, 6, :3] = acc[12, 6, :3]

    def px(a, n, y, x):
        return po.screen_output(a, float(np.float32(1.0 / n)), 1.0)[y, x].tolist()

    assert px(acc, 200, 12, 12) != px(other, 200, 12, 12)     # filtered
    assert px(acc, 201, 12, 12) == px(other, 201, 12, 12)     # sharp-pixel bypass
    assert px(acc, 4999, 12, 6) != px(other, 4999, 12, 6)
    assert px(acc, 5001, 12, 6) == px(other, 5001, 12, 6)     # full bypass


def test_sky_mesh_composite_is_the_sky_scene_plus_the_model():
    """PTO_SCENE_SKYMESH (BASELINE configs[4]) = the physical-sky program with the glTF model block
    appended to SceneIntersect: with the model moved out of every ray's reach the image is the sky
    scene's, bit for bit (same SetupScene, same radiance, same rng draws); with the model in view the
    model's pixels change and the walk is counted."""
    meta_sky = H.stream("sky_256")
    tiny = H.synthetic_dragon(32, 32)
    far = list(H.SKY_MESH_MODEL_INV)
    far[13] = -1.0e5                                         # model space = world shifted by 1e5 in y
    meta_far = H.sky_mesh_stream(model_inv=far)
    sky, _, _ = H.oracle_replay(meta_sky, 2, width=96, height=64)
    comp, _, cnt = H.oracle_replay(meta_far, 2, width=96, height=64, mesh=tiny)
    for a, b in zip(sky, comp):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert cnt[0]["hit_lookups"] == 0
    near, _, cnt = H.oracle_replay(H.sky_mesh_stream(), 2, width=96, height=64, mesh=tiny)
    assert cnt[0]["hit_lookups"] > 0 and cnt[0]["node_fetches"] > 0
    assert (near[-1] != sky[-1]).any(-1).mean() > 0.01
