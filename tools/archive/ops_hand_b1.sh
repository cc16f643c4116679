# Per-op tables of the hand net at one crop per scale (the per-frame call) and of the body at
# Mode R batch 1.  usage: bash tools/ops_hand_b1.sh <tag>
export TMPDIR=/tmp
T=${1:-hb1}; O=gpurun_out/$T; mkdir -p $O
for s in 184 368 552 736; do
  timeout -k 10 200 python3 tools/op_table.py --kind hand --batch 1 --h $s --w $s --runs 5 > $O/ops_hand_b1_$s.txt 2>&1 || exit 1
done
timeout -k 10 200 python3 tools/op_table.py --kind body25 --batch 1 --h 184 --w 328 --runs 20 > $O/ops_body_b1.txt 2>&1
