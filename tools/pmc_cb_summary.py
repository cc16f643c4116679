"""Per-kernel averages of the counters collected by tools/archive/gpu_pmc_cb.sh."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(set))
for f in glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:60]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]].add(r.get("Dispatch_Id"))
for k, m in agg.items():
    print(k)
    for c, v in sorted(m.items()):
        print("   %-36s %16.1f" % (c, v / len(cnt[k][c])))
