"""Multi-GPU path on CPU: world_size 2 over gloo. Each rank shades its 16-row bands (the split
pt_set_row_partition makes on the GPU; here the CPU oracle renders the owned rows), the bands are
gathered to rank 0 with the same helpers bench.py uses over RCCL, and the assembled frame must equal
the single-process full-frame render bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import helpers as H


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, name, w, h, out_path):
    import babylon_pt as bp
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        meta = H.stream(name)
        sc = H.oracle_scene(meta, w, h)
        u = H.with_resolution(H.path_call(meta["frames"][0])["uniforms"], w, h)
        pad = bp.padded_bands(h, world)
        acc = torch.zeros((pad * 16, w, 4), dtype=torch.float32)
        prev = np.zeros((h, w, 4), np.float32)
        for b in range(rank, (h + 15) // 16, world):        # this rank's bands only
            r0, r1 = b * 16, min(h, (b + 1) * 16)
            out, _ = sc.path_trace(u, prev, r0, r1, nthreads=2)
            acc[r0:r1] = torch.from_numpy(out[r0:r1])
        assert sorted(bp.owned_rows(h, world, rank)) == [r for b in range(rank, (h + 15) // 16, world)
                                                        for r in range(b * 16, min(h, b * 16 + 16))]
        send = torch.zeros((pad // world, 16, w, 4), dtype=torch.float32)
        glist = [torch.empty_like(send) for _ in range(world)] if rank == 0 else None
        full = torch.zeros((pad * 16, w, 4), dtype=torch.float32) if rank == 0 else None
        bp.gather_bands(dist, acc, world, rank, send, glist, full)
        if rank == 0:
            np.save(out_path, full[:h].numpy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_band_gather_assembles_the_frame(tmp_path, world):
    name, w, h = "gltf_teapot_320x180", 96, 72
    out = str(tmp_path / "full.npy")
    mp.spawn(_worker, args=(world, _free_port(), name, w, h, out), nprocs=world, join=True)
    got = np.load(out)
    meta = H.stream(name)
    ref, _, _ = H.oracle_replay(meta, 1, width=w, height=h)
    assert np.array_equal(got.view(np.uint32), ref[0].view(np.uint32))


def _worker_output(rank, world, port, name, w, h, out_path):
    """Distributed screenOutput: each rank shades its bands, exchanges 2-row halos with its band
    neighbours (babylon_pt.exchange_halos), runs screenOutput on its own bands only and the RGBA8
    bands are gathered to rank 0 - the path bench.py takes at N > 1."""
    import babylon_pt as bp
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        meta = H.stream(name)
        sc = H.oracle_scene(meta, w, h)
        u = H.with_resolution(H.path_call(meta["frames"][0])["uniforms"], w, h)
        pad = bp.padded_bands(h, world)
        acc = torch.zeros((pad * 16, w, 4), dtype=torch.float32)
        prev = np.zeros((h, w, 4), np.float32)
        mine = bp.owned_rows(h, world, rank)
        for b in range(rank, (h + 15) // 16, world):
            r0, r1 = b * 16, min(h, (b + 1) * 16)
            out, _ = sc.path_trace(u, prev, r0, r1, nthreads=2)
            acc[r0:r1] = torch.from_numpy(out[r0:r1])
        bp.exchange_halos(dist, acc, world, rank, bp.halo_buffers(acc, world))
        # the halo rows now hold the neighbours' values; everything else not owned stays zero
        local = acc[:h].numpy()
        out8 = torch.zeros((pad * 16, w, 4), dtype=torch.uint8)
        shaded = H.po_screen_output(local, 1.0)
        out8[mine] = torch.from_numpy(shaded[mine])
        send = torch.zeros((pad // world, 16, w, 4), dtype=torch.uint8)
        glist = [torch.empty_like(send) for _ in range(world)] if rank == 0 else None
        full = torch.zeros((pad * 16, w, 4), dtype=torch.uint8) if rank == 0 else None
        bp.gather_bands(dist, out8, world, rank, send, glist, full)
        if rank == 0:
            np.save(out_path, full[:h].numpy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_output_with_halo_exchange(tmp_path, world):
    name, w, h = "gltf_teapot_320x180", 96, 72
    out = str(tmp_path / "canvas.npy")
    mp.spawn(_worker_output, args=(world, _free_port(), name, w, h, out), nprocs=world, join=True)
    got = np.load(out)
    meta = H.stream(name)
    ref, _, _ = H.oracle_replay(meta, 1, width=w, height=h)
    want = H.po_screen_output(ref[0], 1.0)
    assert np.array_equal(got, want)


def _worker_pipeline(rank, world, port, w, h, frames, out_path):
    """PipelinedBandGather over gloo: each rank writes frame-dependent values into its own bands
    of the canvas it is handed; rank 0 must assemble every frame, in order, exactly."""
    import babylon_pt as bp
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pad = bp.padded_bands(h, world)
        pipe = bp.PipelinedBandGather(dist, world, rank, pad * 16, w, "cpu", keep=True)
        mine = bp.owned_rows(h, world, rank)
        for k in range(frames):
            canvas = pipe.target()
            canvas.zero_()
            canvas[mine] = torch.tensor([k % 251, rank, 7, 255], dtype=torch.uint8)
            pipe.submit()
        pipe.drain()
        if rank == 0:
            np.save(out_path, np.stack([f[:h].numpy() for _, f in pipe.frames]))
            assert [i for i, _ in pipe.frames] == list(range(frames))
            # bench.py --dump-canvas: the newest frame
            assert torch.equal(pipe.last_frame(), pipe.frames[-1][1])
        else:
            assert pipe.last_frame() is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_pipelined_band_gather(tmp_path, world):
    import babylon_pt as bp
    w, h, frames = 40, 72, 5
    out = str(tmp_path / "frames.npy")
    mp.spawn(_worker_pipeline, args=(world, _free_port(), w, h, frames, out), nprocs=world, join=True)
    got = np.load(out)
    for k in range(frames):
        want = np.zeros((h, w, 4), np.uint8)
        for r in range(world):
            want[bp.owned_rows(h, world, r)] = [k % 251, r, 7, 255]
        assert np.array_equal(got[k], want), k


def _worker_rank_detail(rank, world, port, out_path):
    """bench.rank_detail over gloo: every rank hands in its own row, rank 0 gets the line's field."""
    import json
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    import babylon_pt as bp
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        row = [0.5 + 0.25 * rank, 0.01 * (rank + 1), float("nan") if rank == 1 else 0.02, bp.bands_owned(2160, world, rank)]
        d = bench.rank_detail(dist, torch, "cpu", row)
        if rank == 0:
            with open(out_path, "w") as f:
                json.dump(d, f)
        else:
            assert d is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_rank_detail_fields(tmp_path, world):
    """The N > 1 line's rank_detail (bench.py): min / max over ranks of the path-tracing kernel ms, the
    halo and gather ms (unmeasured ranks left out), the bands each rank owns and the slowest rank."""
    import json
    out = str(tmp_path / "detail.json")
    mp.spawn(_worker_rank_detail, args=(world, _free_port(), out), nprocs=world, join=True)
    with open(out) as f:
        d = json.load(f)
    assert set(d) == {"pathtrace_kernel_ms", "halo_ms", "gather_ms", "bands_per_rank", "slowest_rank", "method"}
    assert d["pathtrace_kernel_ms"] == {"min": 0.5, "max": 0.5 + 0.25 * (world - 1)}
    assert d["slowest_rank"] == world - 1
    assert d["halo_ms"] == {"min": 0.01, "max": round(0.01 * world, 4)}
    assert d["gather_ms"] == {"min": 0.02, "max": 0.02}   # rank 1's NaN: not measured
    nb = (2160 + 15) // 16
    assert d["bands_per_rank"] == [len(range(r, nb, world)) for r in range(world)] and sum(d["bands_per_rank"]) == nb
    assert all(isinstance(x, int) for x in d["bands_per_rank"]) and isinstance(d["method"], str)
