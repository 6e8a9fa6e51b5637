"""The moving-camera anchor of bench.py (moving_camera_run: the dragon stand-in at 1920x1080 with
uCameraIsMoving on every draw, one frame in flight) on a fresh engine, for A/B of the knobs that shape a
serial frame (tools/README.md). Prints Mpaths/s, ms per frame, the frame latency and the compaction mode.

usage: python tools/moving_proxy.py [--steps 100]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    args = ap.parse_args()
    import babylon_pt as bp
    engine = bp.Engine(0)
    try:
        r = bench.moving_camera_run(engine, args)
        q = engine.queue_stats()
        r.update({"late_bounce_compaction": q["late_bounce_compaction"], "frames_in_flight": q["frames_in_flight"],
                  "env": {k: v for k, v in os.environ.items() if k.startswith("PT_")}})
        print(json.dumps(r))
    finally:
        engine.dispose()


if __name__ == "__main__":
    main()
