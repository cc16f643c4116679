# Round-3 HEAD checkpoint: the -m gpu suite, then the round profile (bench, kernel trace,
# FETCH / WRITE / SQ passes, per-layer table, stamp clock) of the shipped kernels.
T=${1:-r3g}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -3 $O/gputest.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
bash tools/profile_round.sh $T/prof
