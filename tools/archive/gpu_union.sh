# Row-union staging A/B (VAR 512 vs the per-(pair, ky) runs), per layer shape.
# usage: bash tools/archive/gpu_union.sh <tag>
set -o pipefail
export TMPDIR=/tmp
T=${1:-union}; O=gpurun_out/$T; mkdir -p $O
CB=tools/convbench
for s in "3 128 128 46 82 32" "3 384 128 46 82 32" "3 96 96 46 82 32" "3 288 96 46 82 32" "3 512 512 46 82 32" \
         "3 256 512 46 82 32" "3 256 256 92 164 32" "3 128 256 92 164 32" "3 128 128 184 328 32"; do
  for u in 1 0; do
    export ISLPOSE_X3_UNION=$u
    echo "== $s union=$u" >> $O/u.txt
    timeout -k 10 120 $CB $s 20 x3 3 >> $O/u.txt 2>&1 || { echo "convbench failed: $s"; tail $O/u.txt; exit 1; }
  done
done
