# Generic-loop ablations (development build, ISLPOSE_X3_ABL bits: 1 no MFMAs, 2 no input
# staging, 4 no weight DMA, 8 no barrier, 16 no prologue, 64 no epilogue) on Mode R batch-32
# stage layers (23x41, two K groups).  Wrong results by design: timing only.
# usage: bash tools/cb_abl.sh <tag>
export TMPDIR=/tmp
T=${1:-abl}; O=gpurun_out/$T; mkdir -p $O
for shp in "3 128 128" "3 384 128" "3 96 96"; do
  for abl in 0 1 2 4 6 8 64 7 71; do
    echo "== $shp ABL=$abl" >> $O/cb.txt
    ISLPOSE_X3_ABL=$abl timeout -k 10 60 tools/convbench $shp 23 41 32 200 x3 2 >> $O/cb.txt 2>&1 || exit 1
  done
done
python3 - <<PY
import re
cur=None
for line in open("$O/cb.txt"):
    if line.startswith("=="): cur=line.strip()
    m=re.search(r"round 1 x3\s+([\d.]+) us", line)
    if m: print(cur, m.group(1))
PY
