"""Per-layer durations of the last bench step from a rocprofv3 kernel trace.

Kernel launches map onto the netspec convs in order; a fused Mconv6 -> Mconv7 launch
(conv_x3_f16 with VAR bit 16, csrc/conv_x3.hip) and the conv1_1 -> conv1_2 launch
(conv_x3_c12, csrc/conv_c12.hip) cover two convs each and are counted as both (their rows are
labelled "pair"), so the rows stay aligned after the fusions.  Split-K reduces,
pools and the post kernels are listed by name.  TF is the direct-conv count (fp32-eq) per
second; a row above a third of the FP16 peak (838.9 TF-eq; 36/16 of that for the Winograd kernel's
"W2" rows) cannot be real and is flagged.
"""
import csv
import re
import sys

sys.path.insert(0, "isl-signlanguage-translation_amd")
from islpose import netspec  # noqa: E402


def main(path, h=368, w=656, B=32, kind=0, quiet=False):
    if path.endswith(".db"):
        import sqlite3
        c = sqlite3.connect(path)
        rows = [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e}
                for n, s, e in c.execute("select name, start, end from kernels")]
    else:
        rows = list(csv.DictReader(open(path)))
    rows = sorted(rows, key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "preprocess" in r["Kernel_Name"]]
    seq = rows[idx[-1]:]
    convs = netspec.convs_for(kind)
    ci, tot, groups = 0, 0.0, {}
    for r in seq:
        n = r["Kernel_Name"]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        conv_kernels = ("conv_mfma", "wino_f23", "conv_x3_f16", "conv_x3_rgb", "conv_x3_wr", "conv_x3_c12", "wino_x3",
                        "wino_f16")
        if any(k in n for k in conv_kernels):
            targs = re.search(r"conv_x3_f16<([^>]*)>", n)
            # two convs in one launch: the fused 1x1 pair (VAR 16) or conv1_1 -> conv1_2 (conv_c12.hip)
            fused = (bool(targs) and (int(targs.group(1).split(",")[5]) & 16) != 0) or "conv_x3_c12" in n
            c = convs[ci]
            fl = 2 * c.cout * c.cin * c.k * c.k * h * w * B
            tag = ("W2" if "wino_f16" in n else "WX" if "wino_x3" in n else ("W" if "wino" in n else ("X" if "x3" in n else "D")))
            if "conv_x3_wr" in n:
                tag += " wave-ranges"
            if fused:
                c2 = convs[ci + 1]
                fl += 2 * c2.cout * c2.cin * c2.k * c2.k * h * w * B
                key = "%dx%d c%d->%d->%d k%d pair %s" % (h, w, c.cin, c.cout, c2.cout, c2.k, tag)
            else:
                key = "%dx%d c%d->%d k%d %s" % (h, w, c.cin, c.cout, c.k, tag)
            g = groups.setdefault(key, [0, 0.0, 0.0])
            g[0] += 1; g[1] += d; g[2] += fl
            last = convs[ci + 1] if fused else c
            if last.name in ("conv1_2", "conv2_2", "conv3_4"):
                h //= 2; w //= 2
            ci += 2 if fused else 1
        else:
            g = groups.setdefault(n.replace("(anonymous namespace)::", "").split("(")[0][:40], [0, 0.0, 0.0])
            g[0] += 1; g[1] += d
    for k, (cnt, d, fl) in sorted(groups.items(), key=lambda t: -t[1][1]):
        tf = fl / d / 1e6 if fl else 0.0
        # (a Winograd F(2x2,3x3) row executes 16/36 of the direct count: its ceiling is 36/16 higher)
        cap = 838.9 * (36 / 16 if k.endswith(" W2") else 1.0)
        print("%-46s x%-3d %9.1f us  %5.1f%%  %s%s" % (k, cnt, d, 100 * d / tot, ("%.1f TF" % tf) if fl else "",
                                                     "  (above the FP16 peak / 3: misaligned)" if tf > cap else ""))
    print("total %.1f us (sum of the rows: %.1f us), %d of %d convs mapped"
          % (tot, sum(g[1] for g in groups.values()), ci, len(convs)))


if __name__ == "__main__":
    main(sys.argv[1])
