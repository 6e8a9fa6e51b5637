"""GPU parity: libpt.so (HIP, gfx950) against the CPU oracle on the reference's recorded uniform
streams. The bar is bit-exact: both sides implement the pinned GLSL semantics,
so every RGBA32F accumulation texel and every RGBA8 canvas byte must agree exactly.

Run on an MI355X: python -m pytest tests -m gpu
"""
import numpy as np
import pytest

import helpers as H

pytestmark = pytest.mark.gpu


def _bits_equal(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    if a.dtype == np.float32:
        return np.array_equal(a.view(np.uint32), b.view(np.uint32))
    return np.array_equal(a, b)


def _diff_report(a, b):
    if a.dtype == np.float32:
        bad = a.view(np.uint32) != b.view(np.uint32)
    else:
        bad = a != b
    pix = bad.reshape(bad.shape[0], bad.shape[1], -1).any(-1)
    d = np.abs(a.astype(np.float64) - b.astype(np.float64))
    ys, xs = np.nonzero(pix)
    first = (int(xs[0]), int(ys[0])) if len(xs) else None
    return "mismatching pixels %d / %d (%.4f%%), max |diff| %.3g, first (x,y)=%s" % (
        pix.sum(), pix.size, 100.0 * pix.mean(), np.nanmax(d), first)


def test_library_identity(engine):
    import babylon_pt as bp
    assert bp.lib().pt_version().decode().endswith("gfx950")


@pytest.mark.parametrize("op", list(range(15)))
def test_pinned_math_bitexact(engine, op):
    """Device built-ins == oracle built-ins, bit for bit, over ranges the shaders use and edges."""
    import ptoracle as po
    rng = np.random.default_rng(100 + op)
    n = 1 << 16
    if op in (0, 8):        # exp2 / exp
        x = np.concatenate([rng.uniform(-160, 130, n), rng.uniform(-2, 2, n), [0.0, -0.0, np.inf, -np.inf, np.nan]])
    elif op in (1, 9):      # log2 / log
        x = np.concatenate([10.0 ** rng.uniform(-40, 38, n), rng.uniform(0, 2, n), [0.0, -1.0, np.inf, np.nan, 1e-45]])
    elif op in (2, 3):      # sin / cos
        x = np.concatenate([rng.uniform(0, 6.2831855, n), rng.uniform(-100, 100, n), [0.0, -0.0, np.inf, np.nan]])
    elif op in (4, 6):      # atan / acos
        x = np.concatenate([rng.uniform(-1.2, 1.2, n), rng.uniform(-50, 50, n), [1.0, -1.0, 0.0, np.nan]])
    elif op == 5:           # atan2(x, y)
        x = rng.uniform(-10, 10, n)
    elif op == 7:           # pow
        x = np.concatenate([rng.uniform(0, 1, n), rng.uniform(0, 50, n), [0.0, 1.0]])
    elif op == 10:          # sqrt
        x = np.concatenate([rng.uniform(0, 4, n), 10.0 ** rng.uniform(-40, 38, n), [0.0, -1.0, np.inf]])
    elif op in (12, 13, 14):  # a / b, 1 / sqrt(a), 1 / a: every exponent, denormals, edges
        x = np.concatenate([rng.integers(0, 2 ** 32, 2 * n, dtype=np.uint64).astype(np.uint32).view(np.float32),
                            rng.uniform(-4, 4, n).astype(np.float32),
                            np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 1.2e-38, 8.5e37, 8.6e37,
                                      2.0 ** 126, -2.0 ** 126, 2.0 ** -126, 2.0 ** 127], np.float32)])
        x = x.astype(np.float64)
    else:                   # rng stream from seeds
        x = rng.integers(0, 2 ** 24, 2 * n).astype(np.float64)
    x = x.astype(np.float32)
    y = None
    if op == 5:
        y = rng.uniform(-10, 10, x.size).astype(np.float32)
        y[:8] = 0.0
    elif op == 7:
        y = np.concatenate([rng.uniform(0.01, 3.0, x.size - 2), [2.2, 0.4545]]).astype(np.float32)
    elif op == 11:
        y = rng.integers(0, 2 ** 24, x.size).astype(np.float32)
    elif op == 12:
        y = rng.integers(0, 2 ** 32, x.size, dtype=np.uint64).astype(np.uint32).view(np.float32).copy()
    ref = po.math_probe(op, x, y)
    got = engine.math_probe(op, x, y)
    same = (ref.view(np.uint32) == got.view(np.uint32)) | (np.isnan(ref) & np.isnan(got))
    assert same.all(), "op %d: %d mismatches, e.g. x=%r ref=%r got=%r" % (
        op, (~same).sum(), x[~same][:3], ref[~same][:3], got[~same][:3])


def test_fast_reciprocal_is_ieee_on_every_input(engine):
    """grcp (v_rcp_f32 + one FMA Newton step, IEEE division outside [2^-126, 2^126)) equals the
    correctly rounded 1.0f / x for all 2^32 binary32 inputs (NaN == NaN)."""
    assert engine.math_exhaustive(0) == 0


def test_fast_sqrt_is_ieee_on_every_input(engine):
    """gsqrt (v_sqrt_f32 + residual-sign correction on [2^-96, 2^126], sqrtf elsewhere) equals
    the correctly rounded sqrtf for all 2^32 binary32 inputs (NaN == NaN)."""
    assert engine.math_exhaustive(1) == 0


@pytest.mark.parametrize("seed", [0, 1])
def test_screen_output_adversarial_accumulation(engine, seed):
    """screenOutput of an accumulation buffer with values across the binary32 range (denormals,
    +-0, huge, inf, NaN, negative) and every edge flag value in alpha, drawn through the effect
    API as the render loop does: bit-exact with the oracle's RGBA8 canvas (and the fused copy)."""
    import babylon_pt as bp
    rng = np.random.default_rng(seed)
    h, w = 67, 93
    mag = rng.choice(np.array([0.0, 1e-40, 1e-38, 3e-37, 1e-20, 1e-3, 0.5, 1.0, 3.0, 1e3, 1e30, 3e38], np.float32), size=(h, w, 3))
    acc = (mag * rng.uniform(0.5, 2.0, size=(h, w, 3))).astype(np.float32)
    acc *= np.where(rng.random((h, w, 3)) < 0.1, -1.0, 1.0).astype(np.float32)
    special = rng.random((h, w, 3))
    acc[special < 0.02] = np.inf
    acc[(special >= 0.02) & (special < 0.03)] = np.nan
    acc[(special >= 0.03) & (special < 0.05)] = -0.0
    alpha = rng.choice(np.array([0.0, -1.0, 1.01, 0.5, 1.0, 2.0, np.nan], np.float32), size=(h, w))
    frame = np.concatenate([acc, alpha[..., None]], axis=-1).astype(np.float32)
    src = bp.RenderTargetTexture("acc", (w, h), engine)
    dst = bp.RenderTargetTexture("copy", (w, h), engine)
    tgt = bp.RenderTargetTexture("out", (w, h), engine)
    src.write(frame)
    copy = bp.EffectWrapper(engine, "screenCopy", [], ["pathTracedImageBuffer"], name="copy")
    out = bp.EffectWrapper(engine, "screenOutput", ["uOneOverSampleCounter", "uToneMappingExposure"],
                           ["accumulationBuffer"], name="out")
    ren = bp.EffectRenderer(engine)
    engine.resize_canvas(w, h)
    for inv, exp in [(1.0, 1.0), (float(np.float32(1.0 / 7.0)), 1.7), (0.003, 1.0), (0.0001, 0.25)]:
        copy.effect.setTexture("pathTracedImageBuffer", src)
        out.effect.setFloat("uOneOverSampleCounter", inv)
        out.effect.setFloat("uToneMappingExposure", exp)
        out.effect.setTexture("accumulationBuffer", src)
        ren.render(copy, dst)
        ren.render(out)
        engine.sync()
        got = engine.read_canvas(w, h)
        want = H.po_screen_output(frame, inv, exp)
        assert _bits_equal(want, got), "1/N %r exposure %r: %s" % (inv, exp, _diff_report(want, got))
        assert _bits_equal(frame, dst.read())
        # into an RGBA32F target: the tone-mapped floats themselves
        out.effect.setTexture("accumulationBuffer", src)
        ren.render(out, tgt)
        engine.sync()
        import ptoracle as po
        want_f = po.screen_output_f32(frame, inv, exp)
        got_f = tgt.read()
        assert _bits_equal(want_f, got_f), "float target, 1/N %r exposure %r: %s" % (inv, exp, _diff_report(want_f, got_f))


def _replay_gpu(engine, meta, frames=None, width=None, height=None, parts=1, split_output=False, mesh=None):
    import babylon_pt as bp
    m = None
    if meta["scene"] in ("gltf", "hdri", "skymesh"):
        m = H.texture_payloads(meta, mesh if mesh is not None else H.mesh(meta))
    player = bp.StreamPlayer(engine, meta, H.bluenoise(), m, width, height)
    accs, canvases = [], []
    w, h = player.width, player.height
    engine.resize_canvas(w, h)
    for i in range(len(meta["frames"][:frames])):
        if parts == 1:
            engine.set_row_partition(1, 0)
            player.play_frame(i)
        else:
            # every part renders its bands into the same targets, then copy + output full-frame
            calls = meta["frames"][i]
            for p in range(parts):
                engine.set_row_partition(parts, p)
                player.play_call(calls[0])
            engine.set_row_partition(1, 0)
            if split_output:   # copy full-frame, then screenOutput band by band (output partition)
                player.play_call(calls[1])
                engine.set_output_partition(True)
                for p in range(parts):
                    engine.set_row_partition(parts, p)
                    player.play_call(calls[2])
                engine.set_output_partition(False)
                engine.set_row_partition(1, 0)
            else:
                for c in calls[1:]:
                    player.play_call(c)
        engine.sync()
        accs.append(player.textures["pathTracingRenderTarget"].read())
        canvases.append(engine.read_canvas(w, h))
    return accs, canvases, player


# (schedule, BVH layout): every combination must give the same bits
BACKENDS = [(b, l) for b in ("megakernel", "persistent", "wavefront") for l in ("pairs", "trail", "reference")]


@pytest.fixture(params=BACKENDS, ids=["-".join(b) for b in BACKENDS])
def backend(request, engine):
    engine.set_backend(request.param[0])
    engine.set_bvh_layout(request.param[1])
    yield request.param
    engine.set_backend("megakernel")
    engine.set_bvh_layout("pairs")


@pytest.mark.parametrize("name,frames", [
    ("cornell_256", None),
    ("sky_256", None),
    ("gltf_teapot_320x180", None),
    ("gltf_duck_320x180", None),
    ("gltf_helmet_320x180", None),
    ("hdri_teapot_320x180", None),
    ("hdri_helmet_320x180", None),
    ("quadric_256", None),
])
def test_stream_bitexact(engine, backend, name, frames):
    """Whole recorded streams (path trace -> copy -> output per frame) match the oracle exactly."""
    meta = H.stream(name)
    ref_acc, ref_can, _ = H.oracle_replay(meta, frames, with_output=True)
    got_acc, got_can, _ = _replay_gpu(engine, meta, frames)
    if meta["scene"] in ("gltf", "hdri"):
        assert engine.bvh_layout_used() == backend[1]
    for i, (ra, ga, rc, gc) in enumerate(zip(ref_acc, got_acc, ref_can, got_can)):
        assert _bits_equal(ra, ga), "%s frame %d accumulation: %s" % (name, i, _diff_report(ra, ga))
        assert _bits_equal(rc, gc), "%s frame %d canvas: %s" % (name, i, _diff_report(rc, gc))


def _quadric_variant(mat, k, rotate):
    """The recorded quadric stream with every shape switched to material `mat`, uShapeK = k and,
    optionally, each shape's inverse matrix rotated (what the GUI controls change)."""
    import copy
    meta = copy.deepcopy(H.stream("quadric_256"))
    th = 0.7
    rx = np.array([[1, 0, 0, 0], [0, np.cos(th), -np.sin(th), 0], [0, np.sin(th), np.cos(th), 0], [0, 0, 0, 1]])
    rz = np.array([[np.cos(th), -np.sin(th), 0, 0], [np.sin(th), np.cos(th), 0, 0], [0, 0, 1, 0], [0, 0, 0, 1]])
    for f in meta["frames"]:
        u = H.path_call(f)["uniforms"]
        u["uAllShapesMatType"] = ["i", [mat]]
        u["uShapeK"] = ["f", [k]]
        if rotate:
            for name in list(u):
                if name.endswith("InvMatrix") and name != "uCameraMatrix":
                    m = np.array(u[name][1], np.float64).reshape(4, 4)
                    u[name] = ["f", [float(v) for v in np.float32(m @ rx @ rz).reshape(-1)]]
    return meta


@pytest.mark.parametrize("mat,k,rotate", [(1, 0.5, False), (2, 0.8, True), (3, 0.3, True), (4, 1.0, True)])
def test_quadric_materials_and_transforms_bitexact(engine, backend, mat, k, rotate):
    """All twelve unit shapes under each material, a non-default uShapeK and rotated transforms."""
    meta = _quadric_variant(mat, k, rotate)
    ref_acc, ref_can, _ = H.oracle_replay(meta, 2, with_output=True)
    got_acc, got_can, _ = _replay_gpu(engine, meta, 2)
    for ra, ga, rc, gc in zip(ref_acc, got_acc, ref_can, got_can):
        assert _bits_equal(ra, ga), _diff_report(ra, ga)
        assert _bits_equal(rc, gc), _diff_report(rc, gc)


def test_bunny_1080p_bitexact_and_counters(engine, backend):
    """BASELINE config 2 at full size (1920x1080, StanfordBunny via BVH_Fast_Builder layout)."""
    meta = H.stream("gltf_bunny_1080p")
    ref_acc, ref_can, ref_cnt = H.oracle_replay(meta, 2, with_output=True)
    engine.set_counting(True)
    engine.reset_counters()
    try:
        got_acc, got_can, _ = _replay_gpu(engine, meta, 2)
        cnt = engine.counters()
    finally:
        engine.set_counting(False)
    for i in range(2):
        assert _bits_equal(ref_acc[i], got_acc[i]), "frame %d: %s" % (i, _diff_report(ref_acc[i], got_acc[i]))
        assert _bits_equal(ref_can[i], got_can[i]), "frame %d canvas: %s" % (i, _diff_report(ref_can[i], got_can[i]))
    ref_total = {k: sum(c[k] for c in ref_cnt) for k in ref_cnt[0]}
    assert cnt == ref_total


def test_dragon_standin_1080p_bitexact_and_counters(engine, backend):
    """A 524,288-triangle mesh (the texture's capacity; helpers.synthetic_dragon, BVH by the native
    builder) under the bunny stream's camera at 1920x1080: BASELINE config 4's geometry scale."""
    meta = H.stream("gltf_bunny_1080p")
    mesh = H.synthetic_dragon()
    ref_acc, ref_can, ref_cnt = H.oracle_replay(meta, 2, with_output=True, mesh=mesh)
    import babylon_pt as bp
    engine.set_counting(True)
    engine.reset_counters()
    try:
        player = bp.StreamPlayer(engine, meta, H.bluenoise(), H.texture_payloads(meta, mesh))
        engine.resize_canvas(meta["width"], meta["height"])
        got_acc, got_can = [], []
        for i in range(2):
            player.play_frame(i)
            engine.sync()
            got_acc.append(player.textures["pathTracingRenderTarget"].read())
            got_can.append(engine.read_canvas(meta["width"], meta["height"]))
        cnt = engine.counters()
    finally:
        engine.set_counting(False)
    assert engine.bvh_layout_used() == backend[1]
    for ra, ga, rc, gc in zip(ref_acc, got_acc, ref_can, got_can):
        assert _bits_equal(ra, ga), _diff_report(ra, ga)
        assert _bits_equal(rc, gc), _diff_report(rc, gc)
    assert cnt == {k: sum(c[k] for c in ref_cnt) for k in ref_cnt[0]}


@pytest.mark.parametrize("size", [(480, 272), (203, 117)])
def test_overlapped_frames_observed_between_draws(engine, size):
    """Frame overlap: the path tracing of draw k + 1 runs beside draw k's, gated only by
    the main stream's state two draws back, and the history blend follows on the main stream. Sixteen
    frames of the dragon stand-in (the recording, then still-camera frames) are issued with no sync
    between them, except that the accumulation is read right after the path-tracing draw of frames 3
    and 9 (before their copy / output), the screenCopy target right after frame 5's copy draw (a deferred
    copy) and the canvas after frame 7's output. Every read, and the last frame's accumulation and
    canvas, equal the oracle's bits."""
    import copy
    import babylon_pt as bp
    W, Hh = size
    meta = copy.deepcopy(H.stream("gltf_bunny_1080p"))
    mesh = H.synthetic_dragon()
    player = bp.StreamPlayer(engine, meta, H.bluenoise(), H.texture_payloads(meta, mesh), W, Hh)
    meta["frames"] = meta["frames"] + [player.synth_frame(k) for k in range(12)]
    ref_acc, ref_can, _ = H.oracle_replay(meta, None, W, Hh, with_output=True, mesh=mesh)
    engine.resize_canvas(W, Hh)
    seen = []
    for i, calls in enumerate(meta["frames"]):
        for call in calls:
            player.play_call(call)
            if call["shader"] == "pathTracingFragmentShader" and i in (3, 9):
                seen.append(("acc after path tracing", i, player.textures["pathTracingRenderTarget"].read(), ref_acc[i]))
            if call["shader"] == "screenCopyFragmentShader" and i == 5:
                seen.append(("screenCopy target", i, player.textures["screenCopyRenderTarget"].read(), ref_acc[i]))
            if call["shader"] == "screenOutputFragmentShader" and i == 7:
                seen.append(("canvas", i, engine.read_canvas(W, Hh), ref_can[i]))
    engine.sync()
    seen.append(("final acc", len(meta["frames"]) - 1, player.textures["pathTracingRenderTarget"].read(), ref_acc[-1]))
    seen.append(("final canvas", len(meta["frames"]) - 1, engine.read_canvas(W, Hh), ref_can[-1]))
    for what, i, got, want in seen:
        assert _bits_equal(want, got), "%s, frame %d: %s" % (what, i, _diff_report(want, got))


@pytest.mark.parametrize("layout,order", [("pairs", "keys"), ("trail", "keys"), ("pairs", "stored"),
                                          ("pairs", "octant-major 8x8x8")])
def test_late_bounce_compaction_1080p_bitexact(monkeypatch, layout, order):
    """Late-bounce compaction forced on (PT_CONT=1, from bounce 2 for waves with <= 48 live paths, the
    default PT_CONT_LANES: the
    pt_trace<P,false,true> variant stores them, pt_cont runs them packed on the draw's side stream):
    the dragon stand-in's four recorded 1920x1080 frames, accumulation and canvas bit-exact - with pt_cont
    taking the records in ray-key order (the default: 4x4x4 cells, light flag first), in store order
    (PT_CONT_SORT=0), and in the 8192-key octant-major order (PT_CONT_SORT_GRID=3, PT_CONT_SORT_KEY=1)."""
    import babylon_pt as bp
    monkeypatch.setenv("PT_CONT", "1")
    if order == "stored":
        monkeypatch.setenv("PT_CONT_SORT", "0")
    elif order != "keys":
        monkeypatch.setenv("PT_CONT_SORT_GRID", "3")
        monkeypatch.setenv("PT_CONT_SORT_KEY", "1")
    e = bp.Engine(0)
    try:
        e.set_bvh_layout(layout)
        meta = H.stream("gltf_bunny_1080p")
        mesh = H.synthetic_dragon()
        ref_acc, ref_can, _ = H.oracle_replay(meta, None, with_output=True, mesh=mesh)
        got_acc, got_can, _ = _replay_gpu(e, meta, None, mesh=mesh)
        assert e.queue_stats()["late_bounce_compaction"] == "on"
    finally:
        e.dispose()
    for i, (ra, ga, rc, gc) in enumerate(zip(ref_acc, got_acc, ref_can, got_can)):
        assert _bits_equal(ra, ga), "frame %d: %s" % (i, _diff_report(ra, ga))
        assert _bits_equal(rc, gc), "frame %d canvas: %s" % (i, _diff_report(rc, gc))


def test_late_bounce_compaction_auto_mode_bitexact(monkeypatch):
    """The default auto mode (PT_CONT=2): a target's first 32 draws use the default (on from
    PT_CONT_AUTO_PIXELS, here 0, so on; the last two before the trial compact either way, warming the
    variant up on the side streams), then blocks of 10 draws with compaction on, off, off with two frames
    in flight (twice), off, on, draws 3-7 of each timed by events on the main stream; at the 93rd draw
    the host waits for the trial once and keeps the faster mode (and, without compaction, the faster
    depth). 96 frames of the dragon stand-in at 480x272 accumulate the oracle's bits whatever the draws
    chose - across the switches between buffer-set cycles too - and the decision is reported."""
    import copy
    import babylon_pt as bp
    monkeypatch.delenv("PT_CONT", raising=False)
    monkeypatch.setenv("PT_CONT_AUTO_PIXELS", "0")
    W, Hh = 480, 272
    e = bp.Engine(0)
    try:
        meta = copy.deepcopy(H.stream("gltf_bunny_1080p"))
        mesh = H.synthetic_dragon()
        player = bp.StreamPlayer(e, meta, H.bluenoise(), H.texture_payloads(meta, mesh), W, Hh)
        meta["frames"] = meta["frames"] + [player.synth_frame(k) for k in range(92)]
        e.resize_canvas(W, Hh)
        states = []
        for i in range(len(meta["frames"])):
            player.play_frame(i)
            if i in (10, 40, 55):
                q = e.queue_stats()
                states.append((q["late_bounce_compaction"], q["frames_in_flight"]))
        e.sync()
        got_acc = player.textures["pathTracingRenderTarget"].read()
        got_can = e.read_canvas(W, Hh)
        qs = e.queue_stats()
    finally:
        e.dispose()
    ref_acc, ref_can, _ = H.oracle_replay(meta, None, W, Hh, with_output=True, mesh=mesh)
    assert _bits_equal(ref_acc[-1], got_acc), _diff_report(ref_acc[-1], got_acc)
    assert _bits_equal(ref_can[-1], got_can), _diff_report(ref_can[-1], got_can)
    assert states == [("auto: default on", 3), ("auto: trial", 3), ("auto: trial", 2)], states
    assert qs["late_bounce_compaction"] in ("auto: on", "auto: off"), qs
    assert qs["frames_in_flight"] == 3 if qs["late_bounce_compaction"] == "auto: on" else qs["frames_in_flight"] in (2, 3)
    assert qs["compaction_trial_ratio"] and 0.2 < qs["compaction_trial_ratio"] < 5.0, qs


def _oracle_at(meta, frames, W, Hh, mesh, keep_acc, keep_can):
    """The oracle over `frames` (lists of calls) at W x H, keeping the accumulation after the frames in
    keep_acc and the canvas after those in keep_can (a 4K run keeps a few frames, not all of them)."""
    import ptoracle as po
    sc = H.oracle_scene(meta, W, Hh, mesh)
    acc = np.zeros((Hh, W, 4), np.float32)
    accs, cans = {}, {}
    for i, f in enumerate(frames):
        acc, _ = sc.path_trace(H.with_resolution(H.path_call(f)["uniforms"], W, Hh), acc)
        if i in keep_acc:
            accs[i] = acc.copy()
        if i in keep_can:
            ou = H.output_call(f)["uniforms"]
            cans[i] = po.screen_output(acc, ou["uOneOverSampleCounter"][1][0],
                                       ou.get("uToneMappingExposure", ["f", [0.0]])[1][0])
    return accs, cans


@pytest.mark.parametrize("case", ["dragon_1080p", "dragon_4k_whole", "sky_dragon_4k_from_frame1"])
def test_bench_schedule_bitexact(monkeypatch, case):
    """The draws exactly as bench.py's step loop issues them, at the bench's sizes and default knobs (no
    PT_* environment: three frames in flight, no overlap lag, late-bounce compaction in the auto mode's
    default, which is on from 2 MP traced), with no sync or read between frames except one mid-stream read:
      dragon_1080p              - the headline: the dragon stand-in's 4 recorded 1920x1080 frames + 12 of
                                  the render loop's still-camera frames;
      dragon_4k_whole           - dragon_4k_1gpu: the same at 3840x2160 as ONE partition (the compacting
                                  whole-frame 4K path), 4 recorded + 4 frames;
      sky_dragon_4k_from_frame1 - converge_1024spp: sky + dragon stand-in at 3840x2160 from frame 1 (history
                                  cleared), 3 recorded + 5 frames.
    The accumulation read right after one mid-stream path-tracing draw (before its copy / output), the
    canvas after one mid-stream output, and the last frame's accumulation and canvas equal the oracle's
    bits; queue_stats shows that every still-camera draw launched pt_cont with three frames in flight, so
    the test cannot pass on a serial fallback (js/PathTracingCommon.js:1304-1357,
    js/GLTFModelPathTracing_FragmentShader.js:387-609)."""
    import copy
    import os
    import babylon_pt as bp
    for k in list(os.environ):
        if k.startswith("PT_"):
            monkeypatch.delenv(k)
    if case == "sky_dragon_4k_from_frame1":
        meta, W, Hh, extra, read_acc, read_can = H.sky_mesh_stream(), 3840, 2160, 5, 3, 5
    else:
        meta = copy.deepcopy(H.stream("gltf_bunny_1080p"))
        W, Hh = (1920, 1080) if case == "dragon_1080p" else (3840, 2160)
        extra, read_acc, read_can = (12, 9, 7) if case == "dragon_1080p" else (4, 4, 5)
    mesh = _dragon()
    e = bp.Engine(0)
    try:
        player = bp.StreamPlayer(e, meta, H.bluenoise(), H.texture_payloads(meta, mesh), W, Hh)
        frames = meta["frames"] + [player.synth_frame(k) for k in range(extra)]
        e.resize_canvas(W, Hh)
        seen = []
        for i, calls in enumerate(frames):
            for call in calls:
                player.play_call(call)
                if call["shader"] == "pathTracingFragmentShader" and i == read_acc:
                    seen.append(("acc after path tracing", i, player.textures["pathTracingRenderTarget"].read()))
                if call["shader"] == "screenOutputFragmentShader" and i == read_can:
                    seen.append(("canvas", i, e.read_canvas(W, Hh)))
        e.sync()
        last = len(frames) - 1
        seen.append(("final acc", last, player.textures["pathTracingRenderTarget"].read()))
        seen.append(("final canvas", last, e.read_canvas(W, Hh)))
        qs = e.queue_stats()
    finally:
        e.dispose()
    assert qs["late_bounce_compaction"] == "auto: default on", qs
    assert qs["frames_in_flight"] == 3, qs
    # (a moving-camera draw runs alone and does not compact: the recorded stream's first frame)
    still = sum(1 for f in frames if f[0]["uniforms"]["uCameraIsMoving"][1][0] == 0)
    assert still > 0 and qs["compacting_draws"] == still, qs
    accs, cans = _oracle_at(meta, frames, W, Hh, mesh, {read_acc, last}, {read_can, last})
    for what, i, got in seen:
        want = cans[i] if "canvas" in what else accs[i]
        assert got.shape == want.shape
        assert _bits_equal(want, got), "%s %s, frame %d: %s" % (case, what, i, _diff_report(want, got))


@pytest.mark.parametrize("layout", ["pairs", "trail"])
@pytest.mark.parametrize("workload", ["bunny", "dragon"])
def test_timed_kernel_1080p_bitexact(engine, workload, layout):
    """The kernels the bench times, at the configurations it times them on: the production
    (non-counting) megakernel - any-hit shadow rays and last segments, longest-first order and split
    tiles from the second frame on - over whole 1920x1080 frames of StanfordBunny (BASELINE
    configs[1]) and the dragon stand-in (the headline), all four recorded frames (the first clears
    the history, the rest blend), accumulation and canvas bit-exact with the oracle."""
    meta = H.stream("gltf_bunny_1080p")
    mesh = H.synthetic_dragon() if workload == "dragon" else H.mesh(meta)
    ref_acc, ref_can, _ = H.oracle_replay(meta, None, with_output=True, mesh=mesh)
    engine.set_backend("megakernel")
    engine.set_bvh_layout(layout)
    engine.set_counting(False)
    try:
        got_acc, got_can, _ = _replay_gpu(engine, meta, None, mesh=mesh)
        assert engine.bvh_layout_used() == layout
    finally:
        engine.set_bvh_layout("pairs")
    assert len(got_acc) == len(meta["frames"]) == 4
    for i, (ra, ga, rc, gc) in enumerate(zip(ref_acc, got_acc, ref_can, got_can)):
        assert _bits_equal(ra, ga), "%s frame %d: %s" % (workload, i, _diff_report(ra, ga))
        assert _bits_equal(rc, gc), "%s frame %d canvas: %s" % (workload, i, _diff_report(rc, gc))


@pytest.mark.parametrize("key", ["bookcase", "twoparts"])
def test_reference_multimesh_models_bitexact(engine, backend, key):
    """The reference's two other models (150 / 5 merged meshes, mixed vertex-attribute sets, so
    NaN UVs in the triangle texture; the bookcase's BVH is 41 levels deep), as its own pipeline
    builds them (tests/golden/mesh_<key>.npz), under the teapot stream: bit-exact, counters equal."""
    meta = H.stream("gltf_teapot_320x180")
    mesh = H.mesh(key)
    ref_acc, ref_can, ref_cnt = H.oracle_replay(meta, 2, with_output=True, mesh=mesh)
    import babylon_pt as bp
    engine.set_counting(True)
    engine.reset_counters()
    try:
        player = bp.StreamPlayer(engine, meta, H.bluenoise(), H.texture_payloads(meta, mesh))
        engine.resize_canvas(meta["width"], meta["height"])
        got_acc, got_can = [], []
        for i in range(2):
            player.play_frame(i)
            engine.sync()
            got_acc.append(player.textures["pathTracingRenderTarget"].read())
            got_can.append(engine.read_canvas(meta["width"], meta["height"]))
        cnt = engine.counters()
    finally:
        engine.set_counting(False)
    for ra, ga, rc, gc in zip(ref_acc, got_acc, ref_can, got_can):
        assert _bits_equal(ra, ga), _diff_report(ra, ga)
        assert _bits_equal(rc, gc), _diff_report(rc, gc)
    assert cnt == {k: sum(c[k] for c in ref_cnt) for k in ref_cnt[0]}
    assert sum(c["node_fetches"] for c in ref_cnt) > 0


def test_stack_overflow_is_defined_and_reported(engine, backend):
    """A tree whose walks nest deeper than stackLevels[28] (out of bounds in the GLSL): pushes past
    level 27 are dropped and such pops are culled, identically to the oracle, nothing is read out
    of bounds, and the draw reports PT_ERR_DATA."""
    import babylon_pt as bp
    meta = H.stream("gltf_bunny_1080p")
    mesh = H.synthetic_dragon(128, 128, knot=(2, 3), tube=3.2)
    ref_acc, _, ref_cnt = H.oracle_replay(meta, 1, width=480, height=270, mesh=mesh)
    assert ref_cnt[0]["stack_overflow"] > 0
    player = bp.StreamPlayer(engine, meta, H.bluenoise(), H.texture_payloads(meta, mesh), 480, 270)
    engine.resize_canvas(480, 270)
    player.play_call(meta["frames"][0][0])
    with pytest.raises(bp.PtError, match="PT_ERR_DATA"):
        engine.sync()
    engine.sync()   # the error is reported once
    assert _bits_equal(ref_acc[0], player.textures["pathTracingRenderTarget"].read())
    # the restart trail takes trees of depth <= 28 only (then stackLevels[28] cannot overflow): this
    # one keeps the child-pair walk with its stack
    assert engine.bvh_layout_used() == ("pairs" if backend[1] == "trail" else backend[1])


@pytest.mark.parametrize("parts", [2, 3, 8])
def test_row_partition_is_exact(engine, backend, parts):
    """Band sharding (the multi-GPU split) reproduces the full-frame result bit for bit."""
    meta = H.stream("gltf_teapot_320x180")
    full, _, _ = _replay_gpu(engine, meta, 2)
    split, _, _ = _replay_gpu(engine, meta, 2, parts=parts)
    for a, b in zip(full, split):
        assert _bits_equal(a, b), _diff_report(a, b)


@pytest.mark.parametrize("parts", [2, 3, 8])
def test_partitioned_screen_output_is_exact(engine, parts):
    """screenOutput under the output partition, band by band, gives the full-frame canvas (the
    halo rows are all present here: every part writes the same accumulation target)."""
    meta = H.stream("gltf_teapot_320x180")
    _, full, _ = _replay_gpu(engine, meta, 2)
    _, split, _ = _replay_gpu(engine, meta, 2, parts=parts, split_output=True)
    for a, b in zip(full, split):
        assert np.array_equal(a, b)


_MAPS = {}


def _maps(kind):
    if kind not in _MAPS:
        _MAPS[kind] = H.helmet_maps() if kind == "real" else H.synthetic_pbr_maps()
    return _MAPS[kind]


@pytest.mark.parametrize("maps_kind", ["real", "seeded"])
@pytest.mark.parametrize("name", ["gltf_helmet_320x180", "hdri_helmet_320x180"])
def test_pbr_maps_bitexact(engine, backend, name, maps_kind):
    """DamagedHelmet with all four PBR samplers bound - its real maps (the reference's JPEGs,
    tests/golden/helmet_maps, 2048x2048) and seeded stand-ins that reach every material branch
    (helpers.synthetic_pbr_maps): albedo pow 2.2, normal-map perturbation, metallic-roughness
    material switches and emission, bit for bit against the oracle on every schedule."""
    import babylon_pt as bp
    meta = H.stream(name)
    maps = _maps(maps_kind)
    player = bp.StreamPlayer(engine, meta, H.bluenoise(), H.texture_payloads(meta, H.mesh(meta)))
    for kind, sampler in H.PBR_SAMPLERS.items():
        player.textures[sampler] = bp.Texture(engine, maps[kind], name=kind)
    got = []
    for i in range(3):
        player.play_frame(i)
        engine.sync()
        got.append(player.textures["pathTracingRenderTarget"].read())
    ref, _, _ = H.oracle_replay(meta, 3, maps=maps)
    for i, (ra, ga) in enumerate(zip(ref, got)):
        assert _bits_equal(ra, ga), "%s frame %d: %s" % (name, i, _diff_report(ra, ga))


def test_deferred_screen_copy_is_observed_exactly(engine):
    """screenCopy is deferred to ride along with the next screenOutput of the same source; reading
    its target first, or drawing anything else first, must still see the copy."""
    import babylon_pt as bp
    meta = H.stream("gltf_teapot_320x180")
    player = bp.StreamPlayer(engine, meta, H.bluenoise(), H.texture_payloads(meta, H.mesh(meta)))
    pt_call, cp_call, out_call = meta["frames"][0]
    player.play_call(pt_call)
    player.play_call(cp_call)
    acc = player.textures["pathTracingRenderTarget"].read()          # flushes nothing it needs
    copied = player.textures["screenCopyRenderTarget"].read()        # must flush the copy
    assert _bits_equal(acc, copied)
    # copy deferred, then the next frame's path tracing reads it as previousBuffer
    f1 = meta["frames"][1]
    player.play_call(f1[0])
    player.play_call(f1[1])
    player.play_call(meta["frames"][2][0])                            # flush before this draw
    engine.sync()
    ref, _, _ = H.oracle_replay(meta, 3)
    # frame 2's path tracing used frame 1's copy as history
    assert _bits_equal(ref[2], player.textures["pathTracingRenderTarget"].read())


def test_odd_sizes_bitexact(engine, backend):
    """Odd target sizes: quad helpers beyond the edge, partial 16x16 tiles, partial bands."""
    meta = H.stream("gltf_teapot_320x180")
    ref_acc, ref_can, _ = H.oracle_replay(meta, 2, width=203, height=117, with_output=True)
    got_acc, got_can, _ = _replay_gpu(engine, meta, 2, width=203, height=117)
    for ra, ga, rc, gc in zip(ref_acc, got_acc, ref_can, got_can):
        assert _bits_equal(ra, ga), _diff_report(ra, ga)
        assert _bits_equal(rc, gc), _diff_report(rc, gc)


def test_in_place_history(engine, backend):
    """previousBuffer bound to the target itself (legal: each pixel reads only its own texel)."""
    import babylon_pt as bp
    meta = H.stream("cornell_256")
    ref_acc, _, _ = H.oracle_replay(meta, 3)
    player = bp.StreamPlayer(engine, meta, H.bluenoise())
    rt = player.textures["pathTracingRenderTarget"]
    for i in range(3):
        call = dict(H.path_call(meta["frames"][i]))
        call["samplers"] = dict(call["samplers"], previousBuffer="pathTracingRenderTarget")
        player.play_call(call)
    engine.sync()
    assert _bits_equal(ref_acc[2], rt.read())


@pytest.mark.parametrize("backend_name", ["megakernel", "persistent", "wavefront"])
def test_malformed_bvh_links_fall_back_exactly(engine, backend_name):
    """A tree whose right-child links are not exact integers (legal input: the GLSL just fetches
    whatever texel the float index lands on) cannot be re-packed; the draw must fall back to the
    reference-layout walk and still match the oracle bit for bit."""
    import babylon_pt as bp
    meta = H.stream("gltf_teapot_320x180")
    mesh = H.mesh(meta)
    bvh = mesh["bvh"].copy()                    # (nodes, 8): texel pair per node
    inner = np.nonzero(bvh[:, 0] < 0)[0]
    bvh[inner[3], 4] += 0.5                     # node's right-child link -> between two texels
    bvh[inner[7], 4] = -3.0                     # ... and one pointing before the texture
    bad = dict(mesh, bvh=bvh)
    engine.set_backend(backend_name)
    try:
        ref_acc, _, _ = H.oracle_replay(meta, 2, mesh=bad)
        player = bp.StreamPlayer(engine, meta, H.bluenoise(), H.texture_payloads(meta, bad))
        got = []
        for i in range(2):
            player.play_frame(i)
            engine.sync()
            got.append(player.textures["pathTracingRenderTarget"].read())
        assert engine.bvh_layout_used() == "reference"
    finally:
        engine.set_backend("megakernel")
    for ra, ga in zip(ref_acc, got):
        assert _bits_equal(ra, ga), _diff_report(ra, ga)


def test_errors_are_codes_not_crashes(engine):
    import babylon_pt as bp
    with pytest.raises(bp.PtError, match="PT_ERR_SHADER"):
        bp.EffectWrapper(engine, "void main() {}", [], [], "bogus")
    rt = bp.RenderTargetTexture("rt", (16, 16), engine)
    pt = bp.EffectWrapper(engine, "cornell", ["uResolution"], ["previousBuffer", "blueNoiseTexture"], "pt")
    with pytest.raises(bp.PtError, match="PT_ERR_STATE"):
        bp.EffectRenderer(engine).render(pt, rt)      # samplers unbound
    engine.sync()


def test_interactive_loop_bitexact(engine):
    """The Python host's render loop (pt_controls.RenderLoop) driving the boundary live - its
    uniforms over the first frame's call template - renders what the oracle renders from the
    reference's own recorded stream with the same inputs (tests/golden/controls_cornell.json:
    flight, rotation, FOV, focus, aperture, then accumulation)."""
    import babylon_pt as bp
    import pt_controls as pc
    meta = H.stream("controls_cornell")
    nf = 24
    ref_acc, ref_can, _ = H.oracle_replay(meta, nf, with_output=True)
    rng = iter(bp.splitmix64_uniforms(meta["seed"], 2 * nf))
    loop = pc.RenderLoop(meta["width"], meta["height"], random=lambda: next(rng))
    player = bp.StreamPlayer(engine, meta, H.bluenoise())
    engine.resize_canvas(player.width, player.height)
    template = meta["frames"][0]
    for i in range(nf):
        c = meta["controls"][i]
        for k in c.get("down", []):
            loop.key_down(k)
        for k in c.get("up", []):
            loop.key_up(k)
        if c.get("wheel"):
            loop.wheel(c["wheel"])
        if c.get("rot"):
            loop.camera.rotation = [float(c["rot"][0]), float(c["rot"][1]), 0.0]
        u = loop.step()
        for call in template:
            player.play_call(call, uniform_override=u)
        engine.sync()
        ga = player.textures["pathTracingRenderTarget"].read()
        gc = engine.read_canvas(player.width, player.height)
        assert _bits_equal(ref_acc[i], ga), "frame %d accumulation: %s" % (i, _diff_report(ref_acc[i], ga))
        assert _bits_equal(ref_can[i], gc), "frame %d canvas: %s" % (i, _diff_report(ref_can[i], gc))


def test_dragon_4k_eight_bands_bitexact(engine):
    """BASELINE configs[3] on one GPU: the 524,288-triangle dragon stand-in at 3840x2160 under the
    bunny stream's camera, rendered as 8 band partitions (the rows each of 8 ranks owns), copied
    full-frame and output band by band (pt_set_output_partition) - bit-exact with the oracle's
    whole-frame render, accumulation and canvas, over 2 frames (history blend included)."""
    meta = H.stream("gltf_bunny_1080p")
    mesh = H.synthetic_dragon()
    W, Hh = 3840, 2160
    ref_acc, ref_can, _ = H.oracle_replay(meta, 2, width=W, height=Hh, with_output=True, mesh=mesh)
    got_acc, got_can, _ = _replay_gpu(engine, meta, 2, W, Hh, parts=8, split_output=True, mesh=mesh)
    for i, (ra, ga, rc, gc) in enumerate(zip(ref_acc, got_acc, ref_can, got_can)):
        assert ra.shape == (Hh, W, 4)
        assert _bits_equal(ra, ga), "frame %d accumulation: %s" % (i, _diff_report(ra, ga))
        assert _bits_equal(rc, gc), "frame %d canvas: %s" % (i, _diff_report(rc, gc))


@pytest.mark.parametrize("n", [4, 200, 201, 4999, 5001, 1024 * 64])
def test_screen_output_sample_count_branches(engine, n):
    """screenOutput at the sample counts a converged run reaches (BASELINE configs[4]: 1024 spp and
    beyond): the edge-aware filter, the sharp-pixel bypass once 1/N < 0.005 and the full bypass
    once 1/N < 0.0002 (js/PathTracingCommon.js:293-296), on a real accumulation buffer whose
    alpha carries the path tracer's edge flags (1.01 / -1 / 0) - bit-exact with the oracle."""
    import babylon_pt as bp
    meta = H.stream("cornell_256")
    player = bp.StreamPlayer(engine, meta, H.bluenoise())
    engine.resize_canvas(player.width, player.height)
    for i in range(len(meta["frames"])):
        player.play_frame(i)
    engine.sync()
    acc = player.textures["pathTracingRenderTarget"].read()
    flags = set(np.unique(acc[..., 3]).tolist())
    assert flags <= {0.0, -1.0, np.float32(1.01).item()} and len(flags) >= 2, flags
    inv = float(np.float32(1.0 / n))
    out_call = next(c for c in meta["frames"][-1] if c["shader"] == "screenOutputFragmentShader")
    player.play_call(out_call, uniform_override={"uOneOverSampleCounter": ["f", [inv]]})
    engine.sync()
    got = engine.read_canvas(player.width, player.height)
    exp = out_call["uniforms"].get("uToneMappingExposure", ["f", [1.0]])[1][0]
    want = H.po_screen_output(acc, inv, exp)
    assert _bits_equal(want, got), _diff_report(want, got)


@pytest.mark.parametrize("name", ["sky_256", "cornell_256"])
def test_long_accumulation_bitexact(engine, name):
    """64 progressive frames past the recording (the render loop's still-camera frames:
    uSampleCounter / uFrameCounter counting up, fresh uRandomVec2 each frame): the running
    accumulation and the canvas stay bit-exact with the oracle - no drift in the history blend."""
    import copy
    import babylon_pt as bp
    meta = copy.deepcopy(H.stream(name))
    player = bp.StreamPlayer(engine, meta, H.bluenoise())
    meta["frames"] = meta["frames"] + [player.synth_frame(k) for k in range(64)]
    ref_acc, ref_can, _ = H.oracle_replay(meta, with_output=True)
    engine.resize_canvas(player.width, player.height)
    for i in range(len(meta["frames"])):
        player.play_frame(i)
    engine.sync()
    ga = player.textures["pathTracingRenderTarget"].read()
    gc = engine.read_canvas(player.width, player.height)
    assert _bits_equal(ref_acc[-1], ga), _diff_report(ref_acc[-1], ga)
    assert _bits_equal(ref_can[-1], gc), _diff_report(ref_can[-1], gc)


# ------------------------------------------------------------------------- BASELINE configs[4]
# The physical-sky scene with the glTF model block in its SceneIntersect (PT_PROG_SKY_MESH,
# DESIGN.md §1), on the 524,288-triangle dragon stand-in.

_DRAGON = {}


def _dragon():
    if "m" not in _DRAGON:
        _DRAGON["m"] = H.synthetic_dragon()
    return _DRAGON["m"]


@pytest.mark.parametrize("material", [3, 4, 2, 1])
def test_sky_mesh_bitexact_and_counters(engine, backend, material):
    """Sky + dragon composite under each model material (Metal = the page default, ClearCoat_Diffuse,
    Transparent, Diffuse): the sky's CalculateRadiance with mesh hits, shadow rays toward the sun
    lobe through the BVH, double-sided leaves for Transparent; accumulation, canvas and the
    algorithmic-byte counters equal the oracle's on every schedule and BVH layout."""
    meta = H.sky_mesh_stream(material)
    mesh = _dragon()
    ref_acc, ref_can, ref_cnt = H.oracle_replay(meta, None, width=320, height=180, with_output=True, mesh=mesh)
    engine.set_counting(True)
    engine.reset_counters()
    try:
        got_acc, got_can, _ = _replay_gpu(engine, meta, None, 320, 180, mesh=mesh)
        cnt = engine.counters()
    finally:
        engine.set_counting(False)
    assert engine.bvh_layout_used() == backend[1]
    for i, (ra, ga, rc, gc) in enumerate(zip(ref_acc, got_acc, ref_can, got_can)):
        assert _bits_equal(ra, ga), "frame %d accumulation: %s" % (i, _diff_report(ra, ga))
        assert _bits_equal(rc, gc), "frame %d canvas: %s" % (i, _diff_report(rc, gc))
    assert cnt == {k: sum(c[k] for c in ref_cnt) for k in ref_cnt[0]}
    assert sum(c["hit_lookups"] for c in ref_cnt) > 0


def _with_material(meta, material):
    """A recorded glTF stream with the model's material switched (uModelMaterialType)."""
    frames = []
    for f in meta["frames"]:
        fr = []
        for c in f:
            if c["shader"] == "pathTracingFragmentShader":
                c = dict(c, uniforms=dict(c["uniforms"], uModelMaterialType=["i", [material]]))
            fr.append(c)
        frames.append(fr)
    return dict(meta, frames=frames)


@pytest.mark.parametrize("scene", ["gltf_teapot", "sky_dragon"])
@pytest.mark.parametrize("material", [1, 2, 4])
def test_mesh_materials_any_hit_bitexact(engine, backend, scene, material):
    """The production kernels (no counting) under the mesh materials the recorded streams do not
    carry - Diffuse, Transparent (double-sided leaves), ClearCoat_Diffuse: shadow rays and the sixth
    segment of Diffuse / glass paths end their walk at the first occluder and skip the hit lookup
    (pt_trace.h bounceStep), which must leave every accumulation and canvas bit as the oracle's
    full closest-hit walk has it (the counting variant, used by the tests that compare counters,
    keeps the full walk)."""
    if scene == "gltf_teapot":
        meta, mesh, W, Hh = _with_material(H.stream("gltf_teapot_320x180"), material), None, 320, 180
    else:
        meta, mesh, W, Hh = H.sky_mesh_stream(material), _dragon(), 160, 90
    ref_acc, ref_can, _ = H.oracle_replay(meta, None, width=W, height=Hh, with_output=True, mesh=mesh)
    got_acc, got_can, _ = _replay_gpu(engine, meta, None, W, Hh, mesh=mesh)
    for i, (ra, ga, rc, gc) in enumerate(zip(ref_acc, got_acc, ref_can, got_can)):
        assert _bits_equal(ra, ga), "frame %d accumulation: %s" % (i, _diff_report(ra, ga))
        assert _bits_equal(rc, gc), "frame %d canvas: %s" % (i, _diff_report(rc, gc))


def test_sky_mesh_effect_from_shader_text(engine):
    """The composite is recognised from its fragment source: the sky shader text with the glTF
    model's samplers declared -> PT_PROG_SKY_MESH; the sky shader alone stays PT_PROG_SKY."""
    import babylon_pt as bp
    sky = "#include<pathtracing_physical_sky_functions>\nvoid main(){}\n#include<pathtracing_default_main>"
    comp = "uniform sampler2D tAABBTexture;\nuniform sampler2D tTriangleTexture;\n" + sky
    assert bp.EffectWrapper(engine, sky, [], [], "sky").program() == bp.PROG["sky"]
    assert bp.EffectWrapper(engine, comp, [], [], "comp").program() == bp.PROG["skymesh"]


def test_sky_mesh_4k_eight_bands_bitexact(engine):
    """BASELINE configs[4] at its size: 3840x2160, rendered as the 8 band partitions of an 8-GPU
    node, copied full-frame and output band by band - bit-exact with the oracle's whole-frame
    render over the recorded frames (history clear, moving-camera blend, still camera)."""
    meta = H.sky_mesh_stream()
    mesh = _dragon()
    W, Hh = 3840, 2160
    ref_acc, ref_can, _ = H.oracle_replay(meta, None, width=W, height=Hh, with_output=True, mesh=mesh)
    got_acc, got_can, _ = _replay_gpu(engine, meta, None, W, Hh, parts=8, split_output=True, mesh=mesh)
    for i, (ra, ga, rc, gc) in enumerate(zip(ref_acc, got_acc, ref_can, got_can)):
        assert ra.shape == (Hh, W, 4)
        assert _bits_equal(ra, ga), "frame %d accumulation: %s" % (i, _diff_report(ra, ga))
        assert _bits_equal(rc, gc), "frame %d canvas: %s" % (i, _diff_report(rc, gc))


@pytest.mark.parametrize("lag", ["0", "2"])
def test_sky_mesh_bands_compaction_lag_bitexact(monkeypatch, lag):
    """Band partitions of small frames with late-bounce compaction forced on (PT_CONT=1) and the
    overlap lag (PT_OVERLAP_LAG: buffer sets beyond the three side streams, so a stream runs its next
    draw before the main stream blended its previous one): 4 parts of 960x544 sky + dragon stand-in,
    copied full-frame and output band by band, bit-exact with the oracle's whole-frame render."""
    import babylon_pt as bp
    monkeypatch.setenv("PT_CONT", "1")
    monkeypatch.setenv("PT_OVERLAP_LAG", lag)
    meta = H.sky_mesh_stream()
    mesh = _dragon()
    W, Hh = 960, 544
    e = bp.Engine(0)
    try:
        got_acc, got_can, _ = _replay_gpu(e, meta, None, W, Hh, parts=4, split_output=True, mesh=mesh)
        assert e.queue_stats()["late_bounce_compaction"] == "on"
    finally:
        e.dispose()
    ref_acc, ref_can, _ = H.oracle_replay(meta, None, width=W, height=Hh, with_output=True, mesh=mesh)
    for i, (ra, ga, rc, gc) in enumerate(zip(ref_acc, got_acc, ref_can, got_can)):
        assert _bits_equal(ra, ga), "frame %d accumulation: %s" % (i, _diff_report(ra, ga))
        assert _bits_equal(rc, gc), "frame %d canvas: %s" % (i, _diff_report(rc, gc))


def test_sky_mesh_converges_1024_frames_bitexact(engine):
    """configs[4]'s converged run at a reduced size: 1024 progressive frames (the 3 recorded ones,
    then the render loop's still-camera frames) through pathTracing -> screenCopy -> screenOutput;
    the accumulation after frame 1024 and the 5x5-filtered canvas at uSampleCounter = 1024 are
    bit-exact with the oracle's."""
    import ptoracle as po
    import babylon_pt as bp
    meta = H.sky_mesh_stream()
    mesh = _dragon()
    W, Hh, N = 128, 72, 1024
    player = bp.StreamPlayer(engine, meta, H.bluenoise(), H.texture_payloads(meta, mesh), W, Hh)
    engine.resize_canvas(W, Hh)
    frames = meta["frames"] + [player.synth_frame(k) for k in range(N - len(meta["frames"]))]
    sc = H.oracle_scene(meta, W, Hh, mesh)
    acc = np.zeros((Hh, W, 4), np.float32)
    for f in frames:
        acc, _ = sc.path_trace(H.with_resolution(H.path_call(f)["uniforms"], W, Hh), acc)
        for c in f:
            player.play_call(c)
    engine.sync()
    ou = H.output_call(frames[-1])["uniforms"]
    assert ou["uOneOverSampleCounter"][1][0] == np.float32(1.0 / N)
    want = po.screen_output(acc, ou["uOneOverSampleCounter"][1][0], ou.get("uToneMappingExposure", ["f", [1.0]])[1][0])
    ga = player.textures["pathTracingRenderTarget"].read()
    gc = engine.read_canvas(W, Hh)
    assert _bits_equal(acc, ga), _diff_report(acc, ga)
    assert _bits_equal(want, gc), _diff_report(want, gc)


def test_helmet_real_maps_1080p_bitexact(engine):
    """BASELINE configs[2] at its size: DamagedHelmet in the HDRI scene at 1920x1080 with the four
    real PBR maps bound, 3 recorded frames, accumulation and canvas bit-exact."""
    import babylon_pt as bp
    meta = H.stream("hdri_helmet_320x180")
    maps = _maps("real")
    W, Hh = 1920, 1080
    player = bp.StreamPlayer(engine, meta, H.bluenoise(), H.texture_payloads(meta, H.mesh(meta)), W, Hh)
    for kind, sampler in H.PBR_SAMPLERS.items():
        player.textures[sampler] = bp.Texture(engine, maps[kind], name=kind)
    engine.resize_canvas(W, Hh)
    got_acc, got_can = [], []
    for i in range(3):
        player.play_frame(i)
        engine.sync()
        got_acc.append(player.textures["pathTracingRenderTarget"].read())
        got_can.append(engine.read_canvas(W, Hh))
    ref_acc, ref_can, _ = H.oracle_replay(meta, 3, width=W, height=Hh, with_output=True, maps=maps)
    for i in range(3):
        assert _bits_equal(ref_acc[i], got_acc[i]), "frame %d: %s" % (i, _diff_report(ref_acc[i], got_acc[i]))
        assert _bits_equal(ref_can[i], got_can[i]), "frame %d canvas: %s" % (i, _diff_report(ref_can[i], got_can[i]))


@pytest.mark.parametrize("name", ["gltf_helmet_320x180", "hdri_helmet_320x180", "gltf_teapot_320x180"])
def test_split_tiles_bitexact(name, monkeypatch):
    """Tile splitting (the slowest tiles of the longest-first order shaded by 16 waves of 16 lanes,
    pt_trace / pt_order_build) forced on every frame after the first: the recorded stream's
    accumulation and canvas stay bit-exact with the oracle, and the draws did split tiles. (No overlap
    lag: with it a small frame's buffer set comes round again only after the three recorded frames.)"""
    import babylon_pt as bp
    monkeypatch.setenv("PT_SPLIT_ALWAYS", "1")
    monkeypatch.setenv("PT_SPLIT_TILES", "64")
    monkeypatch.setenv("PT_OVERLAP_LAG", "0")
    e = bp.Engine(0)
    try:
        meta = H.stream(name)
        maps = _maps("seeded") if "helmet" in name else None
        m = H.texture_payloads(meta, H.mesh(meta))
        player = bp.StreamPlayer(e, meta, H.bluenoise(), m)
        if maps:
            for kind, sampler in H.PBR_SAMPLERS.items():
                player.textures[sampler] = bp.Texture(e, maps[kind], name=kind)
        w, h = player.width, player.height
        e.resize_canvas(w, h)
        n = len(meta["frames"])
        got_acc, got_can, split = [], [], []
        for i in range(n):
            player.play_frame(i)
            e.sync()
            got_acc.append(player.textures["pathTracingRenderTarget"].read())
            got_can.append(e.read_canvas(w, h))
            split.append(e.queue_stats()["split_tiles"])
        ref_acc, ref_can, _ = H.oracle_replay(meta, n, with_output=True, maps=maps)
        for i in range(n):
            assert _bits_equal(ref_acc[i], got_acc[i]), "frame %d: %s" % (i, _diff_report(ref_acc[i], got_acc[i]))
            assert _bits_equal(ref_can[i], got_can[i]), "frame %d canvas: %s" % (i, _diff_report(ref_can[i], got_can[i]))
        assert max(split) >= 8, split
    finally:
        e.dispose()


@pytest.mark.gpu
def test_order_build_beyond_register_tiles_is_a_permutation(monkeypatch):
    """pt_order_build holds up to 32 tiles per thread (32768 16x16 tiles) in registers and loops
    over memory beyond that. A 3840x2400 frame has 36000 tiles: four frames of the bunny workload
    with longest-first order and forced tile splitting accumulate the same bits as without the
    order (a duplicated or missing tile in the permutation would show)."""
    import babylon_pt as bp
    meta, mesh_arrays, _, _ = H.workload("bunny")
    W, Hh = 3840, 2400
    assert (W // 16) * (Hh // 16) > 32768
    out = {}
    for lpt in ("1", "0"):
        monkeypatch.setenv("PT_LPT", lpt)
        monkeypatch.setenv("PT_SPLIT_ALWAYS", lpt)
        e = bp.Engine(0)
        try:
            p = bp.StreamPlayer(e, meta, H.bluenoise(), H.texture_payloads(meta, mesh_arrays), W, Hh)
            e.resize_canvas(p.width, p.height)
            split = []
            for k in range(4):
                for call in p.synth_frame(k):
                    p.play_call(call)
                e.sync()
                split.append(e.queue_stats()["split_tiles"])
            out[lpt] = (p.textures["pathTracingRenderTarget"].read(), e.read_canvas(W, Hh), split)
        finally:
            e.dispose()
    assert _bits_equal(out["1"][0], out["0"][0]), _diff_report(out["0"][0], out["1"][0])
    assert _bits_equal(out["1"][1], out["0"][1])
    assert max(out["1"][2]) >= 8, out["1"][2]


def test_draw_events_opt_in_and_sampled_timing_window(engine, monkeypatch):
    """Per-draw events cost stream time, so pt_last_render_ms turns them on at its first call (which
    reports PT_ERR_ARG); the timing window brackets every PT_TIMING_EVERY-th draw of each kind."""
    import babylon_pt as bp
    meta = H.stream("gltf_teapot_320x180")
    player = bp.StreamPlayer(engine, meta, H.bluenoise(), H.texture_payloads(meta, H.mesh(meta)), 96, 64)
    engine.resize_canvas(96, 64)

    def play(k):
        for call in player.synth_frame(k):
            player.play_call(call)

    play(0)
    engine.sync()
    with pytest.raises(bp.PtError):
        engine.last_render_ms("gltf")       # no draw was bracketed yet: this call turns events on
    play(1)
    engine.sync()
    assert engine.last_render_ms("gltf") > 0.0
    monkeypatch.setenv("PT_TIMING_EVERY", "3")
    engine.timing_begin()
    for k in range(2, 9):                   # 7 frames: draws 0, 3, 6 of each kind are bracketed
        play(k)
    ms, n = engine.timing_end("gltf")
    assert n == 3 and ms > 0.0
    out_ms, out_n = engine.timing_end("screenOutput")
    assert out_n == 3 and out_ms > 0.0
    monkeypatch.setenv("PT_TIMING_EVERY", "1")
    engine.timing_begin()
    for k in range(9, 11):
        play(k)
    assert engine.timing_end("gltf")[1] == 2
