# Fused Mconv6 -> Mconv7 pair ablations (development build, ISLPOSE_X3_ABL bits: 1 no MFMAs,
# 2 no input staging, 4 no weight DMA, 8 no barrier, 32 Mconv7 filters not loaded, 64 no
# epilogue) on the Mode N shapes (46x82, batch 32).  Wrong results by design: timing only.
# usage: bash tools/archive/cb_f67.sh <tag>
export TMPDIR=/tmp
T=${1:-f67}; O=gpurun_out/$T; mkdir -p $O
for shp in "1 384 512" "1 288 256"; do
  for abl in 0 32 64 1 4 2 65 7 71; do
    echo "== $shp ABL=$abl" >> $O/cb.txt
    ISLPOSE_X3_ABL=$abl timeout -k 10 60 tools/convbench $shp 46 82 32 100 x3f 2 >> $O/cb.txt 2>&1 || exit 1
  done
done
python3 - <<PY
import re
cur=None
for line in open("$O/cb.txt"):
    if line.startswith("=="): cur=line.strip()
    m=re.search(r"round 1 x3f\s+([\d.]+) us", line)
    if m: print(cur, m.group(1))
PY
