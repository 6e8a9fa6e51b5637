"""One rank's share of an N-GPU frame, on one GPU (tools/README.md): rank R's 16-row bands of the
N-way round-robin partition (pt_set_row_partition), pathTracing + screenCopy of those bands and
screenOutput of those bands (pt_set_output_partition), as bench.py's ranks draw them - without the
RCCL halo exchange and gather, which the one-GPU box cannot run. Prints the rank's paths per second
(the pixels its bands hold) and ms per frame, the per-rank half of a strong-scaling point.

usage: python tools/rank_proxy.py [--workload dragon] [--size 3840x2160] [--world 8] [--rank 0]
                                  [--steps 200] [--warmup 100]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="dragon")
    ap.add_argument("--size", default="3840x2160")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    args = ap.parse_args()
    import babylon_pt as bp
    W, Hh = (int(v) for v in args.size.lower().split("x"))
    engine = bp.Engine(0)
    try:
        v, ms, rows, _, _, lat = bench.rank_share_run(engine, args.workload, W, Hh, args.world, args.rank, args.warmup,
                                                      args.steps)
        q = engine.queue_stats()
        bench.end_partition(engine)
        print(json.dumps({"workload": args.workload, "size": [W, Hh], "world": args.world, "rank": args.rank,
                          "rows": rows, "mpaths_per_s": round(v, 2), "ms_per_frame": round(ms, 4),
                          "late_bounce_compaction": q["late_bounce_compaction"],
                          "frames_in_flight": q["frames_in_flight"],
                          "frame_latency_ms": bench.latency_summary(lat, ms), "env": {k: v for k, v in os.environ.items()
                                                                             if k.startswith("PT_")}}))
    finally:
        engine.dispose()


if __name__ == "__main__":
    main()
