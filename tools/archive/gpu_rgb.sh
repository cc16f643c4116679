# conv1_1 kernel: parity tests, then body and hand layer tables with and without it.
export TMPDIR=/tmp
O=gpurun_out/${1:-rgb}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_body.py tests/test_gpu_hand.py tests/test_gpu_configs.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 0; do
  ISLPOSE_RGB_CONV=$r timeout -k 10 300 python3 tools/net_layers.py body25 32 368x656 > $O/body_$r.txt 2>/dev/null && grep -E "==|c3->" $O/body_$r.txt
  ISLPOSE_RGB_CONV=$r timeout -k 10 300 python3 tools/net_layers.py hand 32 736 > $O/hand_$r.txt 2>/dev/null && grep -E "==|c3->" $O/hand_$r.txt
done
