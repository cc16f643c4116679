# wino_f16 vs conv_x3 on one shape under SQ counters (where the Winograd step's cycles go).
# usage: bash tools/w2_pmc.sh <tag> [shape...]   (gpurun_out/<tag>)
export TMPDIR=/tmp
T=${1:-w2pmc}; O=gpurun_out/$T; mkdir -p $O
S=${2:-"3 384 128 46 82 32"}
P1="SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES"
for algo in w2 x3; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$algo.trace -o run -- tools/convbench $S 10 $algo 1 > $O/$algo.trace.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $O/$algo.p1 -o run -- tools/convbench $S 10 $algo 1 > $O/$algo.p1.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d $O/$algo.p2 -o run -- tools/convbench $S 10 $algo 1 > $O/$algo.p2.log 2>&1 || exit 1
done
python3 - <<PY
import csv, glob, collections
for algo in ("w2", "x3"):
    tot = collections.defaultdict(float); n = collections.Counter()
    for p in ("p1", "p2"):
        f = glob.glob("$O/%s.%s/**/*counter_collection.csv" % (algo, p), recursive=True)[0]
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "wino_f16" not in k and "conv_x3" not in k: continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(algo, {k: round(v / max(n[k], 1), 1) for k, v in sorted(tot.items())})
PY
