"""Host submission rate of bench.py's step loop (tools/README.md): how long the host takes to enqueue
one step (the frame's calls through the C ABI) against the device time per step, to tell a
host-bound frame rate from a device-bound one.

usage: python tools/host_rate.py [--workload W] [--size WxH] [--steps K] [--warmup W]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="dragon")
    ap.add_argument("--size", default=None)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--cprofile", action="store_true", help="also print the host loop's top functions (cProfile)")
    args = ap.parse_args()
    import babylon_pt as bp
    W, Hh = (1920, 1080) if not args.size else tuple(int(v) for v in args.size.lower().split("x"))
    engine = bp.Engine(0)
    player, _, _ = bench.make_player(engine, args.workload, W, Hh)
    engine.resize_canvas(W, Hh)

    def step(k):
        for call in player.synth_frame(k):
            player.play_call(call)

    for k in range(args.warmup):
        step(k)
    engine.sync()
    calls = 0
    t_synth = 0.0
    per_call = {}
    t0 = time.perf_counter()
    for k in range(args.warmup, args.warmup + args.steps):
        a = time.perf_counter()
        cs = player.synth_frame(k)
        t_synth += time.perf_counter() - a
        for call in cs:
            a = time.perf_counter()
            player.play_call(call)
            per_call[call["effect"]] = per_call.get(call["effect"], 0.0) + time.perf_counter() - a
            calls += 1
    t_host = time.perf_counter() - t0
    engine.sync()
    t_all = time.perf_counter() - t0
    n = args.steps
    if args.cprofile:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for k in range(args.warmup + n, args.warmup + 2 * n):
            step(k)
        pr.disable()
        engine.sync()
        pstats.Stats(pr).strip_dirs().sort_stats("tottime").print_stats(16)
    print("host us/step %.1f (synth_frame %.1f, %.1f calls/step)  device-bound us/step %.1f  host share %.2f"
          % (1e6 * t_host / n, 1e6 * t_synth / n, calls / n, 1e6 * t_all / n, t_host / t_all))
    print("  host us/step per call: " + ", ".join("%s %.1f" % (k, 1e6 * v / n) for k, v in per_call.items()))
    engine.dispose()


if __name__ == "__main__":
    main()
