"""The bench's N > 1 route (bench.py: one process per GPU, torch.distributed over RCCL) rehearsed on
one GPU in one process: N contexts on device 0 stand for the N ranks, and everything rides one torch
stream exactly as in bench.py - libpt enqueues on it through pt_set_stream, the accumulation and
screenCopy targets are torch tensors wrapped by pt_render_target_wrap, screenOutput writes a torch
uint8 canvas through pt_canvas_wrap. Each context shades its row partition (pt_set_row_partition,
pt_set_output_partition); the halo rows and the RGBA8 bands move by plain torch copies on the same
stream where the bench uses RCCL P2P and gather. No engine.sync anywhere: only the stream orders
libpt's kernels against torch's copies (one torch synchronize per frame, to read the result). The
assembled accumulation and canvas must equal the oracle's whole frame bit for bit.
(RCCL itself refuses two ranks on one device, so its calls run first in the driver's multi-GPU runs;
exchange_halos / PipelinedBandGather are covered over gloo by tests/test_distributed.py.)"""
import numpy as np
import pytest

import helpers as H

pytestmark = pytest.mark.gpu


def _band_copy(dst, src, world, rank, rows=slice(0, 16)):
    """dst's rows `rows` of rank `rank`'s bands from src (both band-padded (bands*16, W, C))."""
    import babylon_pt as bp
    bp.band_view(dst, world)[:, rank, rows].copy_(bp.band_view(src, world)[:, rank, rows])


@pytest.mark.parametrize("name,world,size", [
    ("gltf_teapot_320x180", 2, None),
    ("gltf_teapot_320x180", 3, (203, 117)),   # a partial last band, halos clipped at the frame's edges
    ("cornell_256", 2, None),
])
def test_torch_stream_ranks_bitexact(name, world, size):
    import torch
    import babylon_pt as bp
    meta = H.stream(name)
    W, Hh = size or (meta["width"], meta["height"])
    pad = bp.padded_bands(Hh, world)
    stream = torch.cuda.Stream(device=0)
    torch.cuda.set_stream(stream)
    payload = H.texture_payloads(meta, H.mesh(meta)) if meta["scene"] in ("gltf", "hdri") else None
    ranks = []
    try:
        for r in range(world):
            e = bp.Engine(0)
            e.set_stream(stream.cuda_stream)
            acc = torch.zeros((pad * 16, W, 4), dtype=torch.float32, device="cuda")
            cpy = torch.zeros((Hh, W, 4), dtype=torch.float32, device="cuda")
            canvas = torch.zeros((pad * 16, W, 4), dtype=torch.uint8, device="cuda")
            player = bp.StreamPlayer(e, meta, H.bluenoise(), payload, W, Hh,
                                     {"pathTracingRenderTarget": acc.data_ptr(), "screenCopyRenderTarget": cpy.data_ptr()})
            e.resize_canvas(W, Hh)
            e.set_row_partition(world, r)
            e.set_output_partition(True)
            ranks.append((e, player, acc, canvas, cpy))   # the tensors stay alive: libpt holds their pointers
        full_acc = torch.zeros((pad * 16, W, 4), dtype=torch.float32, device="cuda")
        full_can = torch.zeros((pad * 16, W, 4), dtype=torch.uint8, device="cuda")
        ref_acc, ref_can, _ = H.oracle_replay(meta, width=W, height=Hh, with_output=True)
        for i, frame in enumerate(meta["frames"]):
            pt_call, cp_call, out_call = frame
            for e, player, acc, canvas, _ in ranks:        # path tracing + screenCopy of each rank's bands
                player.play_call(pt_call)
                player.play_call(cp_call)
            for r, (e, player, acc, canvas, _) in enumerate(ranks):   # halo rows from the band neighbours
                lo, hi = (r - 1) % world, (r + 1) % world
                _band_copy(acc, ranks[lo][2], world, lo, slice(14, 16))
                _band_copy(acc, ranks[hi][2], world, hi, slice(0, 2))
            for e, player, acc, canvas, _ in ranks:        # screenOutput of each rank's bands into its canvas
                e.canvas_wrap(W, Hh, canvas.data_ptr())
                player.play_call(out_call)
            for r, (e, player, acc, canvas, _) in enumerate(ranks):   # the gather (and the bands' accumulation)
                _band_copy(full_can, canvas, world, r)
                _band_copy(full_acc, acc, world, r)
            torch.cuda.current_stream().synchronize()
            got_acc = full_acc[:Hh].cpu().numpy()
            got_can = full_can[:Hh].cpu().numpy()
            bad = (got_acc.view(np.uint32) != ref_acc[i].view(np.uint32)).any(-1)
            assert not bad.any(), "frame %d accumulation: %d of %d pixels differ (rows %s, columns %d..%d)" % (
                i, bad.sum(), bad.size, sorted(set(np.nonzero(bad)[0].tolist()))[:40], np.nonzero(bad)[1].min(),
                np.nonzero(bad)[1].max())
            badc = (got_can != ref_can[i]).any(-1)
            assert not badc.any(), "frame %d canvas: %d of %d pixels differ" % (i, badc.sum(), badc.size)
    finally:
        for e, *_ in ranks:
            e.set_stream(None)
            e.dispose()
        torch.cuda.set_stream(torch.cuda.default_stream(0))
