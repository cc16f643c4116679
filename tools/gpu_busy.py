"""GPU busy fraction over the tail of a rocprofv3 kernel trace: the union of kernel
intervals / wall span, for the kernels after the last gap longer than --skip-gap-ms
(i.e. the last timed phase), plus the largest idle gaps.  usage:
  python3 tools/archive/gpu_busy.py run_kernel_trace.csv [--tail-s 2.0]"""
import csv
import sys


def main(path, tail_s=2.0):
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:50])
                   for r in csv.DictReader(open(path))))
    end = max(e for _, e, _ in rows)
    rows = [r for r in rows if r[0] >= end - tail_s * 1e9]
    busy, cur_s, cur_e, gaps = 0, rows[0][0], rows[0][1], []
    for s, e, n in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = rows[-1][1] - rows[0][0]
    print("span %.1f ms, busy %.1f ms (%.1f%%), %d kernels" % (span / 1e6, busy / 1e6, 100 * busy / span, len(rows)))
    gaps.sort(reverse=True)
    print("idle total %.1f ms; largest gaps (ms, next kernel):" % (sum(g for g, _ in gaps) / 1e6))
    for g, n in gaps[:12]:
        print("  %.2f  %s" % (g / 1e6, n))


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[3]) if len(sys.argv) > 3 else 2.0)
