# Generic loop: DMA pieces spread between the taps (ISLPOSE_X3_SPREAD=1) vs all at the step's top.
export TMPDIR=/tmp
O=gpurun_out/${1:-abs}; mkdir -p $O
for s in "7 128 128 92 92 32" "7 128 128 46 46 32" "7 128 128 23 41 32" "3 64 64 368 656 32" "3 128 128 184 328 32" \
         "3 64 128 184 328 32" "3 256 256 184 184 32" "1 384 512 46 82 32" "1 512 52 46 82 32" "1 128 512 92 92 32"; do
  for v in 0 1; do
    echo "== $s spread=$v" >> $O/h.txt
    ISLPOSE_X3_SPREAD=$v timeout -k 10 120 tools/convbench $s 10 x3 3 >> $O/h.txt 2>&1 || { tail $O/h.txt; exit 1; }
  done
done
grep -E "==|round 2" $O/h.txt
ISLPOSE_X3_SPREAD=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_body.py tests/test_gpu_hand.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo parity failed; tail -20 $O/parity.log; exit 1; }
tail -1 $O/parity.log
