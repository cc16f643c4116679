# Effective clock and MFMA busy of the conv kernels in Mode R batch 32 (net 184x328), DEEP off / on:
# kernel trace (durations) + one SQ/GRBM pass each.  usage: bash tools/archive/gpu_clockR.sh <tag>
export TMPDIR=/tmp
T=${1:-clkr}; O=gpurun_out/$T; mkdir -p $O
B="python3 bench.py --scale 0.5 --no-cpu --no-mode-r --e2e-steps 0 --steps 10 --warmup 2"
for d in 0 1; do
  ISLPOSE_X3_DEEP=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace$d -o run -- $B > $O/trace$d.log 2>&1 &&
  ISLPOSE_X3_DEEP=$d timeout -s KILL 300 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/sq$d -o run -- $B > $O/sq$d.log 2>&1 || exit 1
done
for d in 0 1; do
  python3 - $O $d <<'PY'
import csv, glob, sys, collections
O, d = sys.argv[1], sys.argv[2]
f = glob.glob(O + "/sq%s/**/*counter_collection.csv" % d, recursive=True)[0]
c = collections.defaultdict(float)
for r in csv.DictReader(open(f)):
    if "conv_x3_f16" in r["Kernel_Name"]:
        c[r["Counter_Name"]] += float(r["Counter_Value"])
t = glob.glob(O + "/trace%s/**/*kernel_trace.csv" % d, recursive=True)[0]
dur = 0.0; n = 0
for r in csv.DictReader(open(t)):
    if "conv_x3_f16" in r["Kernel_Name"]:
        dur += float(r["End_Timestamp"]) - float(r["Start_Timestamp"]); n += 1
# the SQ pass ran the same command: scale its cycles by the trace's duration
clk = c["GRBM_GUI_ACTIVE"] / 8 / dur
print("deep=%s conv launches %d  sum %.3f ms  GRBM clock %.3f GHz  MFMA busy %.3f  wait_any %.3f wait_inst %.3f" % (
    d, n, dur / 1e6, clk, c["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (c["GRBM_GUI_ACTIVE"] / 8),
    c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]))
PY
done
