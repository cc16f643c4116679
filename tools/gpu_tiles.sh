# Tile-family A/B per layer shape (default 512-px tiles vs ISLPOSE_X3_TILES=small).
# usage: bash tools/gpu_tiles.sh <tag>
set -o pipefail
export TMPDIR=/tmp
T=${1:-tiles}; O=gpurun_out/$T; mkdir -p $O
CB=tools/convbench
for s in "1 512 52 46 82 32" "1 512 26 46 82 32" "1 256 52 46 82 32" "1 256 26 46 82 32" "1 288 256 46 82 32" \
         "1 384 512 46 82 32" "3 384 128 46 82 32" "3 128 128 46 82 32" "3 96 96 46 82 32" "3 288 96 46 82 32" \
         "3 512 512 46 82 32" "3 256 256 92 164 32"; do
  for t in big small; do
    if [ $t = small ]; then export ISLPOSE_X3_TILES=small; else unset ISLPOSE_X3_TILES; fi
    echo "== $s tiles=$t" >> $O/tiles.txt
    timeout -k 10 120 $CB $s 20 x3 2 >> $O/tiles.txt 2>&1 || { echo "convbench failed: $s"; tail $O/tiles.txt; exit 1; }
  done
done
cat $O/tiles.txt
