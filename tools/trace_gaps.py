"""Busy time vs idle gaps of a rocprofv3 kernel trace (--kernel-trace, csv): per kernel class
the calls and summed duration, and the idle time between consecutive kernels of one queue
(end of one to start of the next), over the last `--window-ms` of the trace (the timed steps).

usage: python tools/trace_gaps.py <kernel_trace.csv> [--window-ms W]
"""
import argparse
import collections
import csv


def cls(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("isl::", "").split("<")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window-ms", type=float, default=0.0)
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "0"), cls(r["Kernel_Name"])))
    rows.sort()
    if a.window_ms > 0:
        t_end = max(e for _, e, _, _ in rows)
        rows = [r for r in rows if r[0] >= t_end - a.window_ms * 1e6]
    dur = collections.defaultdict(float)
    calls = collections.defaultdict(int)
    for s, e, _, k in rows:
        dur[k] += e - s
        calls[k] += 1
    span = max(e for _, e, _, _ in rows) - min(s for s, _, _, _ in rows)
    busy = 0
    last_end = None
    for s, e, _, _ in rows:   # union of kernel intervals over all queues
        if last_end is None or s > last_end:
            busy += e - s
            last_end = e
        elif e > last_end:
            busy += e - last_end
            last_end = e
    gaps = collections.defaultdict(list)
    prev = {}
    for s, e, q, k in rows:
        if q in prev:
            gaps[q].append(max(0, s - prev[q]))
        prev[q] = e
    print("kernels %d  span %.3f ms  busy (any queue) %.3f ms  idle %.3f ms" % (
        len(rows), span / 1e6, busy / 1e6, (span - busy) / 1e6))
    for q, g in gaps.items():
        g = sorted(g)
        if not g:
            continue
        print("queue %s: %d gaps, sum %.3f ms, median %.2f us, p90 %.2f us" % (
            q, len(g), sum(g) / 1e6, g[len(g) // 2] / 1e3, g[int(0.9 * (len(g) - 1))] / 1e3))
    print("%-34s %6s %10s %9s" % ("kernel", "calls", "ms", "avg us"))
    for k in sorted(dur, key=lambda k: -dur[k]):
        print("%-34s %6d %10.3f %9.2f" % (k[:34], calls[k], dur[k] / 1e6, dur[k] / calls[k] / 1e3))


if __name__ == "__main__":
    main()
