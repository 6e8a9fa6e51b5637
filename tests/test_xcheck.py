"""The reference's shader text, transcribed mechanically, against the oracle and the HIP path.

oracle/xcheck/transcribe.py turns the GLSL of js/PathTracingCommon.js and each scene's
js/*_FragmentShader.js into C++ by syntax-only rewrites (literal suffixes, swizzle proxies,
braced constructors, out-parameter copies) over a GLSL stand-in (oracle/xcheck/glsl_shim.h) that
shares only the pinned transcendental sequences with the oracle; oracle/xcheck/run_xcheck.py ran
it in the build container on every recorded stream and stored its accumulation after each frame
under tests/golden/xcheck/. Neither the reference nor its transcription (the git-ignored
oracle/_ref/, also listed in .gpurunignore; tests/conftest.py refuses a GPU session that finds
it) travels to the GPU box: there only those committed frames are read. These tests pin the oracle and
the HIP kernels to those frames bit for bit: a misreading of the GLSL (an expression, a branch, a
constant, the order of rng() calls) in the hand-written oracle or kernels would show here, which
the oracle-vs-HIP tests alone cannot see. Radiance parity against a GL driver stays unpinned: the
built-ins' rounding is the pinned one on all three sides.
"""
import json
import os

import numpy as np
import pytest

import helpers as H

XDIR = os.path.join(H.GOLD, "xcheck")
REPORT = json.load(open(os.path.join(XDIR, "report.json")))
CASES = sorted(n for n in REPORT if not n.startswith("_"))
OUT_CASES = [(name, n) for name in sorted(REPORT["_screen_output"]) for n in (1, 2, 200, 201, 4999, 5001)]


def _fixture(name):
    r = REPORT[name]
    d = np.load(os.path.join(XDIR, "%s_%dx%d.npz" % (name, r["width"], r["height"])))
    return r, [d["acc%d" % k] for k in range(r["frames"])]


def _maps(r):
    return H.helmet_maps() if r["maps"] == "helmet" else None


def _same_bits(want, got, what):
    bad = (want.view(np.uint32) != got.view(np.uint32)).any(-1)
    assert not bad.any(), "%s: %d of %d pixels differ from the transcribed reference" % (what, bad.sum(), bad.size)


def test_report_covers_every_reference_shader():
    """Every scene shader of the reference is transcribed (the sky+model composite has no
    reference shader to transcribe), screenCopy and screenOutput too, and the build-time
    comparison found no differing pixel."""
    assert {REPORT[n]["scene"] for n in CASES} == {"cornell", "gltf", "hdri", "sky", "quadric"}
    for n in CASES:
        for f in REPORT[n]["per_frame"]:
            assert f["pixels_differing"] == 0 and f["max_abs"] == 0.0, n
    for n, r in REPORT["_screen_output"].items():
        assert all(v == 0 for v in r["pixels_differing_by_N"].values()), (n, r)


def _quantize(c):
    """the canvas store of a [0,1] colour: u8 = floor(255 c + 0.5) in binary32"""
    c = np.asarray(c, np.float32)
    return np.floor(c * np.float32(255.0) + np.float32(0.5)).astype(np.uint8)


def _output_fixture(name, n):
    r = REPORT["_screen_output"][name]
    d = np.load(os.path.join(XDIR, "screen_output_%s_%dx%d.npz" % (name, r["width"], r["height"])))
    return r, d["acc"], _quantize(d["out_%d" % n])


@pytest.mark.parametrize("name,n", OUT_CASES)
def test_oracle_screen_output_matches_transcribed_reference(name, n):
    """screenOutput at N either side of its bypass thresholds, on an accumulation whose alpha
    carries the path tracer's edge flags; includes the frame border, where the GLSL's
    ivec2(gl_FragCoord.xy + vec2(-1, .)) truncates -0.5 to texel 0."""
    r, acc, want = _output_fixture(name, n)
    got = H.po_screen_output(acc, float(np.float32(1.0 / n)), r["exposure"])
    assert np.array_equal(want, got), "%d px differ" % (want != got).any(-1).sum()


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_transcribed_reference(name):
    r, want = _fixture(name)
    meta = H.stream(name)
    got, _, _ = H.oracle_replay(meta, r["frames"], width=r["width"], height=r["height"], maps=_maps(r))
    for k in range(r["frames"]):
        _same_bits(want[k], got[k], "%s frame %d (oracle)" % (name, k))


@pytest.mark.gpu
@pytest.mark.parametrize("name,n", OUT_CASES)
def test_hip_screen_output_matches_transcribed_reference(engine, name, n):
    import babylon_pt as bp
    r, acc, want = _output_fixture(name, n)
    meta = H.stream(name)
    payload = H.texture_payloads(meta, H.mesh(meta)) if meta["scene"] in ("gltf", "hdri") else None
    player = bp.StreamPlayer(engine, meta, H.bluenoise(), payload, r["width"], r["height"])
    engine.resize_canvas(player.width, player.height)
    player.textures["pathTracingRenderTarget"].write(acc)
    out_call = H.output_call(meta["frames"][0])
    player.play_call(out_call, uniform_override={"uOneOverSampleCounter": ["f", [float(np.float32(1.0 / n))]],
                                                 "uToneMappingExposure": ["f", [r["exposure"]]]})
    got = engine.read_canvas(player.width, player.height)
    assert np.array_equal(want, got), "%d px differ" % (want != got).any(-1).sum()


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_hip_matches_transcribed_reference(engine, name):
    import babylon_pt as bp
    r, want = _fixture(name)
    meta = H.stream(name)
    payload = H.texture_payloads(meta, H.mesh(meta)) if meta["scene"] in ("gltf", "hdri") else None
    player = bp.StreamPlayer(engine, meta, H.bluenoise(), payload, r["width"], r["height"])
    maps = _maps(r)
    if maps:
        for kind, sampler in H.PBR_SAMPLERS.items():
            player.textures[sampler] = bp.Texture(engine, maps[kind], name=kind)
    engine.resize_canvas(player.width, player.height)
    for k in range(r["frames"]):
        player.play_frame(k)
        _same_bits(want[k], player.textures["pathTracingRenderTarget"].read(), "%s frame %d (HIP)" % (name, k))
