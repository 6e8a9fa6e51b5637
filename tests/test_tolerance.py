"""The fp32 tolerance study (tools/tolerance.py -> tests/golden/tolerance.json), on CPU.

The HIP path is bit-exact against the pinned oracle. This pins what "matches the reference GLSL render
within a stated fp32 tolerance" means for a GL driver with another legal built-in set (FMA contraction,
the C library's transcendentals, an approximate reciprocal square root in normalize): measured over the
nine recorded streams and the dragon stand-in, 1024 progressive frames each."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "golden", "tolerance.json")


@pytest.fixture(scope="module")
def report():
    with open(FIX) as f:
        return json.load(f)


def test_fixture_covers_every_stream_and_build(report):
    assert report["frames"] == 1024 and report["checkpoints"] == [1, 64, 1024]
    assert set(report["variants"]) == {"fma", "libm", "gpu"}
    assert set(report["cases"]) == {"cornell_256", "sky_256", "quadric_256", "gltf_teapot", "gltf_duck", "gltf_helmet",
                                    "gltf_bunny", "hdri_teapot", "hdri_helmet", "dragon_standin"}


def test_stated_tolerance_holds(report):
    """DESIGN.md §2's statement: against any of the other built-in sets, per frame at most 0.5 % of the
    paths are re-routed (mean <= 0.2 %), and the progressive estimate after 1024 frames is within an
    RMSE of 5e-4 of the pinned one - at least 20x below the pinned render's own Monte Carlo standard
    error at 1024 spp - while most pixels differ in some bit every frame (the built-ins do change
    the rounding: bit-exactness is a property of the pinned semantics, not of GLSL)."""
    worst_ratio = 1e9
    for name, c in report["cases"].items():
        mc = c["mc_standard_error_rms"]["1024"]
        for v, x in c["variants"].items():
            assert x["rerouted_frac_max"] <= 5e-3, (name, v)
            assert x["rerouted_frac_mean"] <= 2e-3, (name, v)
            assert x["bit_divergent_frac_mean"] >= 0.2, (name, v)
            e = x["estimate"]["1024"]["rmse"]
            assert e <= 5e-4, (name, v, e)
            worst_ratio = min(worst_ratio, mc / e)
    assert worst_ratio >= 20.0, worst_ratio


@pytest.mark.parametrize("name", ["cornell_256", "gltf_teapot", "hdri_helmet"])
def test_first_frame_reproduces(name, report):
    """The study's generator reproduces its committed first-frame numbers exactly, with the toolchain
    that generated them (tolerance.json "toolchain"). The fma / libm / gpu builds' bits depend on how
    gcc fuses under -ffp-contract=fast and on the C library's transcendentals, so under another gcc or
    libc (or without x86 FMA, -mfma) the committed numbers are not a prediction and the case is skipped
    with the reason, rather than compared within a bound loose enough to pass a regression."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import tolerance
    tc = tolerance.toolchain()
    if tc["machine"] not in ("x86_64", "AMD64"):
        pytest.skip("the fma / libm / gpu oracle builds use x86 FMA (-mfma)")
    if tc != report.get("toolchain"):
        pytest.skip("toolchain %r differs from the study's %r: its fma / libm / gpu builds round differently"
                    % (tc, report.get("toolchain")))
    got = tolerance.run_case(name, 1, report["variants"])
    want = report["cases"][name]
    for v in report["variants"]:
        g, w = got["variants"][v], want["variants"][v]
        assert g["bit_divergent_frac_frame1"] == w["bit_divergent_frac_frame1"], (name, v)
        assert g["estimate"]["1"]["rmse"] == pytest.approx(w["estimate"]["1"]["rmse"], rel=1e-12), (name, v)


def test_toolchain_recorded(report):
    assert set(report["toolchain"]) == {"gcc", "libc", "machine"}
