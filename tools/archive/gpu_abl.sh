# Ablations of the generic x3 loop on Mode R's 23x41 stage shapes (development build,
# ISLPOSE_X3_ABL bits: 1 no compute, 2 no input staging, 4 no weight DMA, 8 no barrier;
# wrong results, timing only).  usage: bash tools/archive/gpu_abl.sh <tag>
T=${1:-abl}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for s in "3 128 128 23 41 32" "3 384 128 23 41 32" "3 96 96 23 41 32" "1 384 512 23 41 32"; do
  for a in 0 1 2 4 8 6 14 7; do
    echo "== $s abl=$a" >> $O/abl.txt
    ISLPOSE_X3_ABL=$a timeout -k 10 60 tools/convbench $s 20 x3 2 >> $O/abl.txt 2>&1 || { tail $O/abl.txt; exit 1; }
  done
done
grep "==\|round 1" $O/abl.txt
