"""The reference's shader text, transcribed mechanically, against the oracle and the HIP path.

oracle/xcheck/transcribe.py turns the GLSL of js/PathTracingCommon.js and each scene's
js/*_FragmentShader.js into C++ by syntax-only rewrites (literal suffixes, swizzle proxies,
braced constructors, out-parameter copies) over a GLSL stand-in (oracle/xcheck/glsl_shim.h) that
shares only the pinned transcendental sequences with the oracle; oracle/xcheck/run_xcheck.py ran
it in the build container on every recorded stream and stored its accumulation after each frame
under tests/golden/xcheck/ (the reference is not on the GPU box). These tests pin the oracle and
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
CASES = sorted(REPORT)


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
    reference shader to transcribe) and the build-time comparison found no differing pixel."""
    assert {REPORT[n]["scene"] for n in CASES} == {"cornell", "gltf", "hdri", "sky", "quadric"}
    for n in CASES:
        for f in REPORT[n]["per_frame"]:
            assert f["pixels_differing"] == 0 and f["max_abs"] == 0.0, n


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_transcribed_reference(name):
    r, want = _fixture(name)
    meta = H.stream(name)
    got, _, _ = H.oracle_replay(meta, r["frames"], width=r["width"], height=r["height"], maps=_maps(r))
    for k in range(r["frames"]):
        _same_bits(want[k], got[k], "%s frame %d (oracle)" % (name, k))


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
