"""Summarise rocprofv3 --pmc passes of bench.py into per-step HBM traffic.

Usage: python tools/pmc_summary.py <fetch_dir> <write_dir> --steps S --out profiles/rNN/pmc_summary.json
           [--traffic-out profiles/conv_traffic.json] [--sq <sq_dir> --stats <kernel_stats.csv>]

FETCH_SIZE / WRITE_SIZE are in KiB.  Per MI355X_MICROARCH.md (§HBM), gfx950's
FETCH_SIZE reports half of the bytes of wide coalesced reads: the read side is
doubled before it is compared with algorithmic bytes; WRITE_SIZE is exact for
16-byte-per-lane stores.  The conv kernels load 16 B per lane and store 16 B per
lane.  Counts are divided by the number of bench steps that ran under the
profiler (warmup + validation-free timed steps).
"""
import argparse
import collections
import csv
import glob
import json
import os


NET_KERNELS = ("conv_mfma", "wino_f23", "maxpool", "conv_x3", "wino_x3", "wino_f16")


def kclass(k):
    """Kernel class of a rocprof kernel name: the function name, except that the blur's exact
    re-run (blur_nms_kernel<T, FUSED, true, ...>) is its own class, blur_nms_exact."""
    # kernels in an anonymous namespace (conv_x3_c12) are named "void (anonymous namespace)::f<...>(...)":
    # drop the qualifier before splitting at the argument list (the "" row)
    k = k.replace("(anonymous namespace)::", "").replace("isl::", "")
    cls = k.split("(")[0].replace("void ", "").split("<")[0].strip()
    if cls == "blur_nms_kernel" and "<" in k:
        args = [a.strip() for a in k.split("<", 1)[1].split(">", 1)[0].split(",")]
        if len(args) >= 3 and args[2] == "true":
            return "blur_nms_exact"
    return cls


def load(d, name):
    """Per kernel class: summed counter value and number of dispatches; the net's
    kernels are also summed into the class "net_run"."""
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    out = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != name:
            continue
        k = r["Kernel_Name"]
        cls = kclass(k)
        v = float(r["Counter_Value"])
        did = r.get("Dispatch_Id", r.get("Correlation_Id", ""))
        out[cls] += v
        disp[cls].add(did)
        if any(t in k for t in NET_KERNELS):
            out["net_run"] += v
            disp["net_run"].add(did)
    return out, {k: len(v) for k, v in disp.items()}


def durations(stats_csv):
    """kernel class -> (calls, average ns) from a rocprofv3 --stats kernel_stats.csv."""
    out = {}
    for r in csv.DictReader(open(stats_csv)):
        k = kclass(r["Name"])
        c, t = out.get(k, (0, 0.0))
        out[k] = (c + int(r["Calls"]), t + float(r["TotalDurationNs"]))
    return {k: (c, t / c) for k, (c, t) in out.items()}


POST_KERNELS = ("blur_nms_kernel", "blur_nms_exact", "limb_kernel", "tile_live_kernel", "band_live_kernel",
                "stage2_need_kernel", "compact_kernel", "assemble_kernel", "resize_sep_kernel")


def post_traffic(res, stats_csv, out_path, src):
    """HBM traffic of the post kernels per launch (PMC) and the rate over their rocprof
    average duration, against the 8 TB/s HBM peak."""
    dur = durations(stats_csv)
    t = {"source": src, "peak_GBps": 8000.0,
         "note": "per launch (one launch = the post of one bench step, 32 frames): hbm_bytes = FETCH_SIZE x2 (gfx950 "
                 "wide-read correction) + WRITE_SIZE; avg_us = rocprofv3 --stats average of the same kernel in the "
                 "trace pass of the same command; GBps = hbm_bytes / avg_us. blur_nms_kernel (the fp32 filter over the "
                 "live tiles) is bound by the latency of its per-tile phases (window loads, the two passes, the NMS; "
                 "tools/tile_prof.py), not by HBM; blur_nms_exact re-runs the few undecided tiles in fp64"}
    for k in POST_KERNELS:
        if k in res and k in dur:
            b = res[k]["hbm_bytes_per_launch"]
            us = dur[k][1] / 1e3
            t[k] = {"hbm_bytes_per_launch": round(b), "avg_us": round(us, 2), "GBps": round(b / us / 1e3, 1),
                    "frac_of_hbm_peak": round(b / us / 1e3 / 8000.0, 4)}
    json.dump(t, open(out_path, "w"), indent=1)


def mfma_busy(sq_dir, stats_csv, sq_out, clock_ghz=None):
    """MFMA pipe busy fraction and effective clock of the x3 conv kernels.
    SQ_VALU_MFMA_BUSY_CYCLES counts 32 cycles per 32x32x16 MFMA summed over the chip's
    1024 SIMDs; GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md)."""
    f = glob.glob(os.path.join(sq_dir, "**", "*counter_collection.csv"), recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        k = n.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("isl::", "").split("<")[0]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", ""))
        if "conv_x3" in n or "wino_f16" in n:   # the whole conv stage: conv_x3_f16 + conv_x3_c12 + wino_f16
            acc["conv_stage"][r["Counter_Name"]] += float(r["Counter_Value"])
            disp["conv_stage"].add(r.get("Dispatch_Id", ""))
    json.dump({"note": "raw SQ/GRBM counter sums per kernel class over the profiled bench run",
               "kernels": {k: dict(v, dispatches=len(disp[k])) for k, v in acc.items()}}, open(sq_out, "w"), indent=1)
    x = acc.get("conv_x3_f16")
    if not x or not x.get("GRBM_GUI_ACTIVE"):
        return {}
    stats = list(csv.DictReader(open(stats_csv)))
    wall_ns = sum(float(r["TotalDurationNs"]) for r in stats if "conv_x3_f16" in r["Name"])
    active = x["GRBM_GUI_ACTIVE"] / 8
    cs = acc["conv_stage"]
    stage_wall = sum(float(r["TotalDurationNs"]) for r in stats if "conv_x3" in r["Name"] or "wino_f16" in r["Name"])
    extra = {"conv_stage_mfma_busy_frac": round(cs["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (cs["GRBM_GUI_ACTIVE"] / 8), 4),
             "conv_stage_note": "all conv kernels of the net (conv_x3_f16 + the conv1_1->conv1_2 pair's conv_x3_c12 (or conv_x3_rgb when unfused)"
                                " + the Winograd wino_f16): MFMA busy / GRBM cycles, as x3_mfma_busy_frac"}
    wf = acc.get("wino_f16")
    if wf and wf.get("GRBM_GUI_ACTIVE"):
        extra["wino_f16_mfma_busy_frac"] = round(wf["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (wf["GRBM_GUI_ACTIVE"] / 8), 4)
    if clock_ghz:
        extra["conv_stage_mfma_busy_frac_at_stamp_clock"] = round(
            cs["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (stage_wall * clock_ghz), 4)
    if clock_ghz:
        # GRBM_GUI_ACTIVE / 8 / wall reads high on sub-10 ms dispatches (MI355X_MICROARCH.md, DVFS item 6):
        # the in-kernel clock of a stamp build (s_memtime / s_memrealtime) is the one to divide by
        extra.update({"x3_mfma_busy_frac_at_stamp_clock": round(x["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (wall_ns * clock_ghz), 4),
                      "x3_stamp_clock_ghz": clock_ghz})
    return dict(extra, **{"x3_mfma_busy_frac": round(x["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / active, 4),
            "x3_effective_clock_ghz": round(active / wall_ns, 3),
            "mfma_note": "SQ_VALU_MFMA_BUSY_CYCLES (32 cycles per 32x32x16 MFMA, summed over 1024 SIMDs) / 1024 / "
                         "(GRBM_GUI_ACTIVE / 8 XCDs): the fraction of conv_x3_f16's cycles the MFMA pipes were "
                         "busy, at the clock the chip actually ran (DVFS); effective clock = GRBM_GUI_ACTIVE / 8 / "
                         "summed conv_x3_f16 duration of the trace pass of the same command. Source: "
                         + os.path.relpath(sq_out)})


def main():
    p = argparse.ArgumentParser()
    p.add_argument("fetch")
    p.add_argument("write")
    p.add_argument("--steps", type=int, required=True)
    p.add_argument("--out", required=True)
    p.add_argument("--traffic-out", default=None)
    p.add_argument("--sq", default=None, help="SQ/GRBM pass dir (SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE)")
    p.add_argument("--stats", default=None, help="kernel_stats.csv of the trace pass of the same command")
    p.add_argument("--clock-ghz", type=float, default=None, help="in-kernel clock from a stamp build (tools/archive/gpu_clock.sh)")
    p.add_argument("--post-out", default=None, help="write the post kernels' traffic here (profiles/post_traffic.json)")
    a = p.parse_args()
    (fe, nfe), (wr, nwr) = load(a.fetch, "FETCH_SIZE"), load(a.write, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fe) | set(wr)):
        rb = fe.get(k, 0.0) * 1024 * 2 / a.steps
        wb = wr.get(k, 0.0) * 1024 / a.steps
        n = max(nfe.get(k, 0), 1)
        res[k] = {"read_bytes_per_step": rb, "write_bytes_per_step": wb, "hbm_bytes_per_step": rb + wb,
                  "dispatches": nfe.get(k, 0),
                  "hbm_bytes_per_launch": (fe.get(k, 0.0) * 2 + wr.get(k, 0.0)) * 1024 / n,
                  "raw_fetch_kib_per_step": fe.get(k, 0.0) / a.steps, "raw_write_kib_per_step": wr.get(k, 0.0) / a.steps}
    json.dump(res, open(a.out, "w"), indent=1)
    if a.traffic_out and "net_run" in res:
        t = {"hbm_bytes_per_net_run": res["net_run"]["hbm_bytes_per_step"],
             "source": os.path.relpath(a.out),
             "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KiB->B; per bench step "
                     "(one net run over the batch) and per launch (averaged over the net's launches) of each conv kernel"}
        for cls, key in (("wino_f23_mfma", "wino"), ("conv_x3_f16", "x3"), ("conv_mfma_f32", "direct"),
                         ("wino_x3_f16", "wino_x3")):
            if cls in res:
                t[key + "_hbm_bytes_per_launch"] = res[cls]["hbm_bytes_per_launch"]
                t[key + "_dispatches"] = res[cls]["dispatches"]
        if a.sq and a.stats:
            t.update(mfma_busy(a.sq, a.stats, os.path.join(os.path.dirname(a.out), "sq_counters.json"), a.clock_ghz))
        json.dump(t, open(a.traffic_out, "w"), indent=1)
    if a.post_out and a.stats:
        post_traffic(res, a.stats, a.post_out, os.path.relpath(a.out))
    for k, v in res.items():
        print("%-40s read %10.1f MB  write %10.1f MB" % (k, v["read_bytes_per_step"] / 1e6, v["write_bytes_per_step"] / 1e6))


if __name__ == "__main__":
    main()
