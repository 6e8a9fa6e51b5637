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


class _Ranks:
    """N contexts on device 0 standing for the bench's N ranks on one torch stream (module docstring):
    frame(calls) runs one frame's three draws through the partitioned route with torch copies in place
    of the RCCL halo exchange and gather; full_acc / full_can hold the assembled frame."""

    def __init__(self, world, W, Hh, make):
        import torch
        import babylon_pt as bp
        self.world, self.W, self.Hh = world, W, Hh
        pad = bp.padded_bands(Hh, world)
        self.stream = torch.cuda.Stream(device=0)
        torch.cuda.set_stream(self.stream)
        self.ranks = []
        for r in range(world):
            e = bp.Engine(0)
            e.set_stream(self.stream.cuda_stream)
            acc = torch.zeros((pad * 16, W, 4), dtype=torch.float32, device="cuda")
            cpy = torch.zeros((Hh, W, 4), dtype=torch.float32, device="cuda")
            canvas = torch.zeros((pad * 16, W, 4), dtype=torch.uint8, device="cuda")
            player = make(e, {"pathTracingRenderTarget": acc.data_ptr(), "screenCopyRenderTarget": cpy.data_ptr()})
            e.resize_canvas(W, Hh)
            e.set_row_partition(world, r)
            e.set_output_partition(True)
            self.ranks.append((e, player, acc, canvas, cpy))   # the tensors stay alive: libpt holds their pointers
        self.full_acc = torch.zeros((pad * 16, W, 4), dtype=torch.float32, device="cuda")
        self.full_can = torch.zeros((pad * 16, W, 4), dtype=torch.uint8, device="cuda")

    def frame(self, calls):
        import torch
        world, W, Hh = self.world, self.W, self.Hh
        pt_call, cp_call, out_call = calls
        for e, player, acc, canvas, _ in self.ranks:        # path tracing + screenCopy of each rank's bands
            player.play_call(pt_call)
            player.play_call(cp_call)
        for r, (e, player, acc, canvas, _) in enumerate(self.ranks):   # halo rows from the band neighbours
            lo, hi = (r - 1) % world, (r + 1) % world
            _band_copy(acc, self.ranks[lo][2], world, lo, slice(14, 16))
            _band_copy(acc, self.ranks[hi][2], world, hi, slice(0, 2))
        for e, player, acc, canvas, _ in self.ranks:        # screenOutput of each rank's bands into its canvas
            e.canvas_wrap(W, Hh, canvas.data_ptr())
            player.play_call(out_call)
        for r, (e, player, acc, canvas, _) in enumerate(self.ranks):   # the gather (and the bands' accumulation)
            _band_copy(self.full_can, canvas, world, r)
            _band_copy(self.full_acc, acc, world, r)
        torch.cuda.current_stream().synchronize()
        return self.full_acc[:Hh].cpu().numpy(), self.full_can[:Hh].cpu().numpy()

    def close(self):
        import torch
        for e, *_ in self.ranks:
            e.set_stream(None)
            e.dispose()
        torch.cuda.set_stream(torch.cuda.default_stream(0))


@pytest.mark.parametrize("name,world,size", [
    ("gltf_teapot_320x180", 2, None),
    ("gltf_teapot_320x180", 3, (203, 117)),   # a partial last band, halos clipped at the frame's edges
    ("cornell_256", 2, None),
])
def test_torch_stream_ranks_bitexact(name, world, size):
    import babylon_pt as bp
    meta = H.stream(name)
    W, Hh = size or (meta["width"], meta["height"])
    payload = H.texture_payloads(meta, H.mesh(meta)) if meta["scene"] in ("gltf", "hdri") else None
    rk = _Ranks(world, W, Hh, lambda e, rt: bp.StreamPlayer(e, meta, H.bluenoise(), payload, W, Hh, rt))
    try:
        ref_acc, ref_can, _ = H.oracle_replay(meta, width=W, height=Hh, with_output=True)
        for i, frame in enumerate(meta["frames"]):
            got_acc, got_can = rk.frame(frame)
            bad = (got_acc.view(np.uint32) != ref_acc[i].view(np.uint32)).any(-1)
            assert not bad.any(), "frame %d accumulation: %d of %d pixels differ (rows %s, columns %d..%d)" % (
                i, bad.sum(), bad.size, sorted(set(np.nonzero(bad)[0].tolist()))[:40], np.nonzero(bad)[1].min(),
                np.nonzero(bad)[1].max())
            badc = (got_can != ref_can[i]).any(-1)
            assert not badc.any(), "frame %d canvas: %d of %d pixels differ" % (i, badc.sum(), badc.size)
    finally:
        rk.close()


@pytest.mark.parametrize("workload,world,size", [("bunny", 3, (203, 117)), ("helmet", 2, (256, 144))])
def test_bench_n_gpu_check_with_torch_copies(workload, world, size):
    """bench.py's n_gpu_bitexact check (nrank_check) on the one-GPU lease: the first PARITY_FRAMES
    recorded frames through the N-rank route (torch copies in place of RCCL), compared by
    bench.compare_frames with bench.one_gpu_reference's whole-frame render in a fresh context: equal;
    and one flipped accumulation bit or canvas byte is reported."""
    import bench
    W, Hh = size
    rk = _Ranks(world, W, Hh, lambda e, rt: bench.make_player(e, workload, W, Hh, rt)[0])
    try:
        player = rk.ranks[0][1]
        for i in range(bench.PARITY_FRAMES):
            acc, can = rk.frame(player.meta["frames"][i])
    finally:
        rk.close()
    ref = bench.one_gpu_reference(workload, W, Hh, 0, range(bench.PARITY_FRAMES))
    res = bench.compare_frames(can, acc, *ref)
    assert res["n_gpu_bitexact"] is True, res
    acc2 = acc.copy()
    acc2.view(np.uint32)[Hh // 2, W // 3, 0] ^= 1
    assert bench.compare_frames(can, acc2, *ref)["accumulation_pixels_differing"] == 1
    can2 = can.copy()
    can2[Hh - 1, W - 1, 0] ^= 4
    assert bench.compare_frames(can2, acc, *ref)["n_gpu_bitexact"] is False


def test_rank_detail_filled_on_the_rehearsal():
    """bench.py's N > 1 rank_detail filled on the one-GPU lease: each rehearsed rank's path-tracing
    kernel ms from its own timing window, the halo exchange and the RGBA8 band gather (torch copies in
    place of RCCL) timed with CUDA events on the shared stream, the bands each rank owns: the fields
    bench.rank_fields assembles are all present and positive, and the bands add up to the frame."""
    import torch
    import bench
    import babylon_pt as bp
    world, W, Hh = 3, 480, 270
    rk = _Ranks(world, W, Hh, lambda e, rt: bench.make_player(e, "bunny", W, Hh, rt)[0])
    try:
        player = rk.ranks[0][1]
        for e, *_ in rk.ranks:
            e.timing_begin()
        for k in range(4):
            rk.frame(player.synth_frame(k))
        kernel = []
        for e, *_ in rk.ranks:
            ms, n = e.timing_end("gltf")
            assert n == 4
            kernel.append(ms / n)

        def timed(fn):
            s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            t.record()
            torch.cuda.synchronize()
            return s.elapsed_time(t)

        rows = []
        for r, (e, _, acc, canvas, _) in enumerate(rk.ranks):
            lo, hi = (r - 1) % world, (r + 1) % world
            halo = timed(lambda: (_band_copy(acc, rk.ranks[lo][2], world, lo, slice(14, 16)),
                                  _band_copy(acc, rk.ranks[hi][2], world, hi, slice(0, 2))))
            gather = timed(lambda: _band_copy(rk.full_can, canvas, world, r))
            rows.append([kernel[r], halo, gather, bp.bands_owned(Hh, world, r)])
    finally:
        rk.close()
    d = bench.rank_fields(rows)
    for k in ("pathtrace_kernel_ms", "halo_ms", "gather_ms"):
        assert 0.0 < d[k]["min"] <= d[k]["max"], (k, d)
    assert sum(d["bands_per_rank"]) == (Hh + 15) // 16 and d["slowest_rank"] in range(world)
