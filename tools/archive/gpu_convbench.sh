# Conv microbenchmarks + SQ counters (development).  usage: bash tools/archive/gpu_convbench.sh <tag> [algos]
set -o pipefail
export TMPDIR=/tmp
T=${1:-cb}; A=${2:-x3,direct,wino}; O=gpurun_out/$T; mkdir -p $O
CB=tools/convbench
for s in "3 128 128 46 82 32" "3 384 128 46 82 32" "3 96 96 46 82 32" "3 256 256 92 164 32" "3 64 64 368 656 32" "1 384 512 46 82 32" "3 3 64 368 656 32"; do
  timeout -k 10 120 $CB $s 20 $A 2 >> $O/cb.txt 2>&1 || { echo "convbench failed: $s"; cat $O/cb.txt; exit 1; }
done
cat $O/cb.txt
[ -n "$NOPMC" ] && exit 0
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc1 -o run -- $CB 3 128 128 46 82 32 5 x3 1 > $O/pmc1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc2 -o run -- $CB 3 128 128 46 82 32 5 x3 1 > $O/pmc2.log 2>&1
echo pmc rc=$?
