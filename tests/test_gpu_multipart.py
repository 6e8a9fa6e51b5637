"""Multi-part contexts (pt_ctx_create_devices / _mask): the frame fanned out over several parts
inside pt_render - 16-row bands per part, halo rows pulled from the band neighbours before
screenOutput, RGBA8 bands gathered into part 0's canvas, all ordered by HIP events (pt_group.cpp).
On a one-GPU box the parts share device 0, which runs the same split / halo / gather code (the
copies are then device-local instead of over xGMI). Bit-exact against the oracle's whole frame."""
import os
import shutil
import subprocess

import numpy as np
import pytest

import helpers as H

pytestmark = pytest.mark.gpu


def _replay(engine, meta, frames=None, width=None, height=None, mesh=None, maps=None):
    import babylon_pt as bp
    payload = H.texture_payloads(meta, mesh if mesh is not None else H.mesh(meta)) \
        if meta["scene"] in ("gltf", "hdri", "skymesh") else None
    player = bp.StreamPlayer(engine, meta, H.bluenoise(), payload, width, height)
    if maps:
        for kind, sampler in H.PBR_SAMPLERS.items():
            player.textures[sampler] = bp.Texture(engine, maps[kind], name=kind)
    engine.resize_canvas(player.width, player.height)
    accs, cans = [], []
    for i in range(len(meta["frames"][:frames])):
        player.play_frame(i)
        accs.append(player.textures["pathTracingRenderTarget"].read())
        cans.append(engine.read_canvas(player.width, player.height))
    return accs, cans


def _check(ref_acc, ref_can, got_acc, got_can):
    for i, (ra, ga, rc, gc) in enumerate(zip(ref_acc, got_acc, ref_can, got_can)):
        assert np.array_equal(ra.view(np.uint32), ga.view(np.uint32)), "frame %d accumulation: %d px differ" % (
            i, (ra.view(np.uint32) != ga.view(np.uint32)).any(-1).sum())
        assert np.array_equal(rc, gc), "frame %d canvas: %d px differ" % (i, (rc != gc).any(-1).sum())


@pytest.mark.parametrize("parts", [2, 3, 8])
def test_multipart_context_bitexact(parts):
    import babylon_pt as bp
    meta = H.stream("gltf_teapot_320x180")
    e = bp.Engine(devices=[0] * parts)
    try:
        assert e.parts == parts
        got = _replay(e, meta)
    finally:
        e.dispose()
    ref_acc, ref_can, _ = H.oracle_replay(meta, with_output=True)
    _check(ref_acc, ref_can, *got)


@pytest.mark.parametrize("parts,size", [(2, (320, 180)), (3, (203, 117))])
def test_multipart_without_peer_access_bitexact(monkeypatch, parts, size):
    """The route a node without peer access between its GPUs takes (hipDeviceCanAccessPeer false or
    hipDeviceEnablePeerAccess failing: the context still opens, pt_group.cpp): halo pulls and the canvas
    gather band by band through hipMemcpyPeerAsync, forced here by PT_PEER=0 - the reference's unchanged
    render loop over it (js/GLTF_Model_Path_Tracing.js:1228-1235), accumulation and canvas bit-exact,
    a partial last band and clipped halo rows included at 203x117."""
    import babylon_pt as bp
    monkeypatch.setenv("PT_PEER", "0")
    meta = H.stream("gltf_teapot_320x180")
    W, Hh = size
    e = bp.Engine(devices=[0] * parts)
    try:
        assert e.parts == parts and e.peer_copies is False
        got = _replay(e, meta, width=W, height=Hh)
    finally:
        e.dispose()
    ref_acc, ref_can, _ = H.oracle_replay(meta, width=W, height=Hh, with_output=True)
    _check(ref_acc, ref_can, *got)


@pytest.mark.parametrize("parts", [2, 5])
def test_multipart_odd_size_bitexact(parts):
    """203x117: a partial last band (5 rows), a halo row pair clipped at the top edge."""
    import babylon_pt as bp
    meta = H.stream("cornell_256")
    e = bp.Engine(devices=[0] * parts)
    try:
        got = _replay(e, meta, width=203, height=117)
    finally:
        e.dispose()
    ref_acc, ref_can, _ = H.oracle_replay(meta, width=203, height=117, with_output=True)
    _check(ref_acc, ref_can, *got)


def test_multipart_sky_dragon_4k_bitexact():
    """BASELINE configs[4] through an 8-part context (the 8-GPU split inside libpt)."""
    import babylon_pt as bp
    meta = H.sky_mesh_stream()
    mesh = H.synthetic_dragon()
    e = bp.Engine(devices=[0] * 8)
    try:
        got = _replay(e, meta, width=3840, height=2160, mesh=mesh)
    finally:
        e.dispose()
    ref_acc, ref_can, _ = H.oracle_replay(meta, width=3840, height=2160, with_output=True, mesh=mesh)
    _check(ref_acc, ref_can, *got)


def test_multipart_long_run_and_mask():
    """pt_ctx_create_mask(1) is the one-part context; a 4-part context over 40 progressive frames
    (every frame's canvas gathered while the next frame traces) ends bit-exact."""
    import copy
    import ctypes
    import babylon_pt as bp
    err = ctypes.c_int(0)
    c = bp.lib().pt_ctx_create_mask(1, ctypes.byref(err))
    assert c and bp.lib().pt_ctx_parts(c) == 1
    bp.lib().pt_ctx_destroy(c)
    assert not bp.lib().pt_ctx_create_mask(0, ctypes.byref(err)) and err.value == -1
    meta = copy.deepcopy(H.stream("sky_256"))
    e = bp.Engine(devices=[0] * 4)
    try:
        player = bp.StreamPlayer(e, meta, H.bluenoise())
        meta["frames"] = meta["frames"] + [player.synth_frame(k) for k in range(37)]
        e.resize_canvas(player.width, player.height)
        for i in range(len(meta["frames"])):
            player.play_frame(i)
        ga = player.textures["pathTracingRenderTarget"].read()
        gc = e.read_canvas(player.width, player.height)
    finally:
        e.dispose()
    ref_acc, ref_can, _ = H.oracle_replay(meta, with_output=True)
    _check(ref_acc[-1:], ref_can[-1:], [ga], [gc])


def test_multipart_refuses_per_process_knobs():
    import babylon_pt as bp
    e = bp.Engine(devices=[0, 0])
    try:
        with pytest.raises(bp.PtError, match="PT_ERR_ARG"):
            e.set_row_partition(2, 0)
        with pytest.raises(bp.PtError, match="PT_ERR_ARG"):
            e.set_output_partition(True)
    finally:
        e.dispose()


REPLAY = os.path.join(H.ROOT, "babylon.js-pathtracing-renderer_amd", "js", "replay_stream.js")


@pytest.mark.skipif(not shutil.which("node"), reason="node not installed")
@pytest.mark.parametrize("devices", ["0,0", "0,0,0"])
def test_node_multipart_replay_bitexact(tmp_path, devices):
    """The JavaScript host (the reference's drop-in path: shim -> N-API -> libpt) with a multi-part
    context from PT_DEVICES: the unchanged render calls fan out inside libpt, bit-exact."""
    meta = H.stream("gltf_teapot_320x180")
    H.bluenoise().tofile(tmp_path / "bluenoise.u8")
    for k, v in H.texture_payloads(meta, H.mesh(meta)).items():
        v.tofile(tmp_path / (k + ".f32"))
    out = str(tmp_path / "out")
    subprocess.run(["node", REPLAY, os.path.join(H.GOLD, "gltf_teapot_320x180.json"), str(tmp_path), out],
                   check=True, timeout=300, env=dict(os.environ, PT_DEVICES=devices))
    w, h = meta["width"], meta["height"]
    acc = np.fromfile(out + ".acc.f32", np.float32).reshape(h, w, 4)
    can = np.fromfile(out + ".canvas.u8", np.uint8).reshape(h, w, 4)
    ref_acc, ref_can, _ = H.oracle_replay(meta, with_output=True)
    _check(ref_acc[-1:], ref_can[-1:], [acc], [can])


@pytest.mark.parametrize("parts", [2, 3])
def test_destroy_right_after_output_without_sync(parts):
    """pt_ctx_destroy, pt_texture_destroy and pt_render_target_resize sync every part first: a part's
    queued halo pull or the gather may still read another part's buffers (over the peer link when
    the devices differ; hipFree waits only for its own device). Destroyed / resized straight after a
    screenOutput with no sync, then a fresh context renders the stream bit-exactly."""
    import babylon_pt as bp
    meta = H.stream("gltf_teapot_320x180")
    for resize in (False, True):
        e = bp.Engine(devices=[0] * parts)
        player = bp.StreamPlayer(e, meta, H.bluenoise(), H.texture_payloads(meta, H.mesh(meta)))
        e.resize_canvas(player.width, player.height)
        player.play_frame(0)
        if resize:
            player.textures["pathTracingRenderTarget"].resize((160, 90))
            player.textures["screenCopyRenderTarget"].dispose()
        e.dispose()
    e = bp.Engine(devices=[0] * parts)
    try:
        got = _replay(e, meta)
    finally:
        e.dispose()
    ref_acc, ref_can, _ = H.oracle_replay(meta, with_output=True)
    _check(ref_acc, ref_can, *got)


def test_multipart_draw_events_opt_in_every_part():
    """pt_last_render_ms over several parts: its first call turns per-draw events on for every part
    at once (one failing call, with a message), the next reports the slowest part's draw."""
    import babylon_pt as bp
    meta = H.stream("gltf_teapot_320x180")
    e = bp.Engine(devices=[0, 0, 0])
    try:
        player = bp.StreamPlayer(e, meta, H.bluenoise(), H.texture_payloads(meta, H.mesh(meta)), 96, 64)
        e.resize_canvas(96, 64)
        player.play_frame(0)
        e.sync()
        with pytest.raises(bp.PtError, match="per-draw timing"):
            e.last_render_ms("gltf")
        player.play_frame(1)
        e.sync()
        assert e.last_render_ms("gltf") > 0.0
        assert e.last_render_ms("screenOutput") > 0.0
    finally:
        e.dispose()
