#!/bin/bash
# Batch-1 layer shapes (Mode R 23x41) on tools/convbench: the wave-range kernel vs the split-K
# launches + reduce (ISLPOSE_X3_WR=0), then the wave-range phase stamps.  usage: bash tools/cb_wr.sh <tag>
export TMPDIR=/tmp
T=$1; O=gpurun_out/$T; mkdir -p $O
export CONVBENCH_SPLIT=1 CONVBENCH_CS=384
for shp in "3 128 128" "3 384 128" "3 288 96" "1 512 52" "1 384 512"; do
  for wr in 1 0; do
    echo "== $shp WR=$wr" >> $O/cb.txt
    ISLPOSE_X3_WR=$wr timeout -k 10 60 tools/convbench $shp 23 41 1 300 x3 3 >> $O/cb.txt 2>&1 || exit 1
  done
  echo "== $shp stamps" >> $O/cb.txt
  CONVBENCH_WRSTAMP=1 timeout -k 10 60 tools/convbench $shp 23 41 1 50 x3 1 >> $O/cb.txt 2>&1 || exit 1
done
