"""The Python host's render loop (python/pt_controls.py) against the reference's own loop:
tests/golden/controls_cornell.json is js/Babylon_Path_Tracing.js run under Node with vendored
babylon.js, its KeyboardState / FOV flags / camera.rotation driven frame by frame
(tests/golden/gen/make_fixtures.py CONTROL_STREAMS). Every uniform the loop sets must match
bit for bit, uCameraMatrix included (Babylon's float32 LookAtLH + invert restated)."""
import json
import math
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "babylon.js-pathtracing-renderer_amd", "python"))

import babylon_pt as bp   # noqa: E402
import pt_controls as pc  # noqa: E402

GOLD = os.path.join(HERE, "golden", "controls_cornell.json")


def _drive(meta):
    rng = iter(bp.splitmix64_uniforms(meta["seed"], 2 * len(meta["frames"])))
    loop = pc.RenderLoop(meta["width"], meta["height"], random=lambda: next(rng))
    out = []
    for c in meta["controls"][:len(meta["frames"])]:
        for k in c.get("down", []):
            loop.key_down(k)
        for k in c.get("up", []):
            loop.key_up(k)
        if c.get("wheel"):
            loop.wheel(c["wheel"])
        if c.get("rot"):
            loop.camera.rotation = [float(c["rot"][0]), float(c["rot"][1]), 0.0]
        out.append(loop.step())
    return out


def test_render_loop_matches_reference_stream():
    meta = json.load(open(GOLD))
    got = _drive(meta)
    checked = 0
    for i, (frame, u) in enumerate(zip(meta["frames"], got)):
        for call in frame:
            for name, val in call["uniforms"].items():
                if name in u:
                    assert u[name][0] == val[0], (i, name)
                    assert [float(x) for x in u[name][1]] == [float(x) for x in val[1]], (i, name, u[name], val)
                    checked += 1
    # every frame: 11 pathTracing uniforms + uOneOverSampleCounter
    assert checked == 12 * len(meta["frames"])


def test_stream_exercises_the_controls():
    """The fixture covers what the test claims: flight on all three axes, a rotated basis, FOV
    both ways, focus up and down, the aperture clamp at 0, and still frames accumulating."""
    meta = json.load(open(GOLD))
    pt = [f[0]["uniforms"] for f in meta["frames"]]
    pos = [tuple(u["uCameraMatrix"][1][12:15]) for u in pt]
    assert len(set(pos)) >= 8
    assert len({tuple(u["uCameraMatrix"][1][8:11]) for u in pt}) == 3
    assert len({u["uVLen"][1][0] for u in pt}) == 3
    assert {u["uFocusDistance"][1][0] for u in pt} == {113, 114, 115}
    ap = [u["uApertureSize"][1][0] for u in pt]
    assert max(ap) == 2 and ap[-1] == 0
    assert [u["uSampleCounter"][1][0] for u in pt[-6:]] == [2, 3, 4, 5, 6, 7]


def test_clamps_and_counters():
    loop = pc.RenderLoop(64, 32, random=lambda: 0.5)
    loop.step()
    for _ in range(200):                      # FOV clamps at 150 degrees
        loop.wheel(1)
        u = loop.step()
    assert loop.camera.fov == 150 * (math.pi / 180)
    assert u["uULen"][1][0] == u["uVLen"][1][0] * 2
    for _ in range(200):                      # and at 1 degree
        loop.wheel(-1)
        loop.step()
    assert loop.camera.fov == 1 * (math.pi / 180)
    loop.key_down("dash")
    for _ in range(200):                      # focus distance floors at 1
        u = loop.step()
    assert u["uFocusDistance"][1][0] == 1
    loop.key_up("dash")
    loop.aperture = 99999.5
    loop.key_down("rightbracket")
    u = loop.step()
    assert u["uApertureSize"][1][0] == 100000.0
    loop.key_up("rightbracket")
    u = loop.step()                           # still: progressive refinement
    assert u["uCameraIsMoving"][1] == [0] and u["uSampleCounter"][1] == [2.0]
    assert u["uOneOverSampleCounter"][1] == [0.5]
    loop.invalidate()                         # a GUI change restarts accumulation
    u = loop.step()
    assert u["uCameraIsMoving"][1] == [1] and u["uSampleCounter"][1] == [1.0] and u["uFrameCounter"][1] == [1.0]
    loop.resize(128, 32)
    u = loop.step()
    assert u["uCameraIsMoving"][1] == [1] and u["uResolution"][1] == [128.0, 32.0]
    with pytest.raises(ValueError):
        loop.key_down("x")


def test_dynamic_scene_resets_samples():
    loop = pc.RenderLoop(8, 8, scene_is_dynamic=True, random=lambda: 0.0)
    for _ in range(4):
        u = loop.step()
    assert u["uSampleCounter"][1] == [1.0] and u["uFrameCounter"][1] == [4.0]


def test_camera_matrix_is_rigid_inverse_of_view():
    cam = pc.UniversalCamera((3.0, -7.0, -50.0), rotation=(0.3, -1.1, 0.0))
    m = cam.world_matrix()
    r = [m[0:3], m[4:7], m[8:11]]
    for i in range(3):
        for j in range(3):
            d = sum(r[i][k] * r[j][k] for k in range(3))
            assert abs(d - (1.0 if i == j else 0.0)) < 1e-6
    assert max(abs(a - b) for a, b in zip(m[12:15], cam.position)) < 1e-4
    with pytest.raises(ValueError):
        pc.UniversalCamera((0, 0, 0), rotation=(0, 0, 0.1)).world_matrix()
