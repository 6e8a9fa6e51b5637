"""How consecutive frames overlapped, from a rocprofv3 --kernel-trace CSV (tools/README.md).

usage: python tools/ktrace_overlap.py RUN_KERNEL_TRACE.CSV [--last N]

For the last N path-tracing launches (pt_trace): each launch's queue, start relative to the previous
launch's start, duration, and how many launches ran at once; then the span of those launches, the
frame interval (span / N), the mean number of path-tracing launches in flight and the share of the
span with none running (the frame pipeline drained), and per queue the launches it carried."""
import argparse
import csv
import collections


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=40)
    ap.add_argument("--rows", action="store_true", help="print every launch")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.csv)))
    def counting(name):   # pt_trace<PROG, COUNT, CONT>: the counting variant is not a frame's launch
        args = name.split("<", 1)[1].split(">", 1)[0].split(",")
        return len(args) > 1 and args[1].strip() == "true"
    tr = [r for r in rows if "pt_trace<" in r["Kernel_Name"] and not counting(r["Kernel_Name"])]
    other = [r for r in rows if r not in tr]
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    tr = tr[-args.last:]
    if not tr:
        print("no pt_trace launches")
        return
    t0 = int(tr[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in tr)
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in tr]
    ev = sorted([(s, 1) for s, _ in iv] + [(e, -1) for _, e in iv])
    busy = idle = 0
    n = 0
    last = t0
    weighted = 0
    for t, d in ev:
        if t > last:
            weighted += n * (t - last)
            if n == 0:
                idle += t - last
            last = t
        n += d
    span = t1 - t0
    prev = None
    per_q = collections.Counter(r["Queue_Id"] for r in tr)
    if args.rows:
        for r, (s, e) in zip(tr, iv):
            live = sum(1 for s2, e2 in iv if s2 < e and e2 > s) - 1
            print("q%-3s +%8.1f us  dur %8.1f us  overlapping %d" % (r["Queue_Id"], (s - prev) / 1e3 if prev else 0.0,
                                                               (e - s) / 1e3, live))
            prev = s
    durs = sorted((e - s) / 1e3 for s, e in iv)
    others = collections.Counter(r["Kernel_Name"].split("(")[0] for r in other
                                 if t0 <= int(r["Start_Timestamp"]) <= t1)
    print("launches %d  span %.3f ms  interval %.1f us  in flight %.2f  idle %.1f %%  dur median %.1f us max %.1f us"
          % (len(tr), span / 1e6, span / 1e3 / len(tr), weighted / span, 100.0 * idle / span, durs[len(durs) // 2],
             durs[-1]))
    print("queues:", dict(per_q), " other kernels in the span:", dict(others))


if __name__ == "__main__":
    main()
