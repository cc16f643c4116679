"""Per-kernel-class time and MFMA-busy fraction from a rocprofv3 trace pass (--stats) and an
SQ pass (SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE) of the same command.

usage: python tools/trace_summary.py <kernel_stats.csv> <sq_dir> [--clock-ghz G] [--out f.json]
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / cycles, with cycles = GRBM_GUI_ACTIVE / 8 XCDs
(reads high on short dispatches) and, with --clock-ghz, = duration x the in-kernel clock."""
import argparse
import collections
import csv
import glob
import json
import os


def cls(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("isl::", "").split("<")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("sq")
    ap.add_argument("--clock-ghz", type=float, default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dur = collections.defaultdict(float)
    calls = collections.defaultdict(int)
    for r in csv.DictReader(open(a.stats)):
        dur[cls(r["Name"])] += float(r["TotalDurationNs"])
        calls[cls(r["Name"])] += int(r["Calls"])
    sq = collections.defaultdict(lambda: collections.defaultdict(float))
    f = glob.glob(os.path.join(a.sq, "**", "*counter_collection.csv"), recursive=True)[0]
    for r in csv.DictReader(open(f)):
        sq[cls(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    tot = sum(dur.values())
    out = {"total_ms": round(tot / 1e6, 3), "kernels": {}}
    for k in sorted(dur, key=lambda k: -dur[k]):
        e = {"ms": round(dur[k] / 1e6, 3), "share": round(dur[k] / tot, 4), "calls": calls[k]}
        s = sq.get(k)
        if s and s.get("GRBM_GUI_ACTIVE"):
            e["mfma_busy_grbm_clock"] = round(s["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (s["GRBM_GUI_ACTIVE"] / 8), 4)
            if a.clock_ghz:
                e["mfma_busy_stamp_clock"] = round(s["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (dur[k] * a.clock_ghz), 4)
        out["kernels"][k] = e
    txt = json.dumps(out, indent=1)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt)


if __name__ == "__main__":
    main()
