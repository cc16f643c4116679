# Tile-family A/B per layer shape (default 512-px tiles vs ISLPOSE_X3_TILES=small).
# usage: bash tools/archive/gpu_tiles.sh <tag> [shapes-file]
set -o pipefail
export TMPDIR=/tmp
T=${1:-tiles}; O=gpurun_out/$T; mkdir -p $O
CB=tools/convbench
SHAPES=${2:-tools/tiles_shapes.txt}
while read -r s; do
  [ -z "$s" ] && continue
  for t in big small; do
    if [ $t = small ]; then export ISLPOSE_X3_TILES=small; else unset ISLPOSE_X3_TILES; fi
    echo "== $s tiles=$t" >> $O/tiles.txt
    timeout -k 10 120 $CB $s 20 x3 2 >> $O/tiles.txt 2>&1 || { echo "convbench failed: $s"; tail $O/tiles.txt; exit 1; }
  done
done < $SHAPES
cat $O/tiles.txt
