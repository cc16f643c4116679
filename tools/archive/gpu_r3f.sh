# Round 3: where a small-grid (Mode R 23x41, batch 32) step goes -- generic-loop ablations
# (development build, ISLPOSE_X3_ABL: 1 no compute, 2 no input staging, 4 no weight DMA,
# 8 no barrier) and an SQ/LDS counter pass of the plain kernel.
T=${1:-r3f}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
export CONVBENCH_SPLIT=1
for shp in "3 128 128 23 41 32" "3 384 128 23 41 32" "1 384 512 23 41 32"; do
  for ab in 0 1 2 4 6 8 9 15; do
    echo "== $shp abl=$ab" >> $O/abl.txt
    ISLPOSE_X3_ABL=$ab timeout -k 10 60 tools/convbench $shp 200 x3 2 >> $O/abl.txt 2>&1 || exit 1
  done
done
cat $O/abl.txt | grep -v "^conv\|round 0"
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o run -- tools/convbench 3 128 128 23 41 32 50 x3 1 > $O/pmc.log 2>&1
echo pmc rc=$?
f=$(find $O/pmc -name "*counter_collection.csv" | head -1)
[ -n "$f" ] && python3 -c "
import csv,collections
d=collections.defaultdict(float); n=collections.Counter()
for r in csv.DictReader(open('$f')):
    if 'conv_x3_f16' in r['Kernel_Name']:
        d[r['Counter_Name']]+=float(r['Counter_Value']); n[r['Counter_Name']]+=1
for k in sorted(d): print(k, d[k]/max(1,n[k]))
"
exit 0
