# Round 4: where the Mode R post's time goes (kernel traces with and without the blur bands,
# one SQ counter pass of the banded run).
T=${1:-r4g}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
P="python3 tools/post_prof.py --batch 32 --iters 5"
ISLPOSE_BLUR_BANDS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t1 -o run -- $P > $O/t1.log 2>&1 &&
ISLPOSE_BLUR_BANDS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t0 -o run -- $P > $O/t0.log 2>&1 &&
ISLPOSE_BLUR_BANDS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $O/sq -o run -- $P > $O/sq.log 2>&1
rc=$?
tail -2 $O/t1.log $O/t0.log
exit $rc
