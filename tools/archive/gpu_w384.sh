# 7x7 on 384-pixel tiles (ISLPOSE_X3_WIDE7=3) vs the default: parity (hand nets vs oracle) and A/B.
export TMPDIR=/tmp
T=${1:-w384}; O=gpurun_out/$T; mkdir -p $O
ISLPOSE_X3_WIDE7=3 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_hand.py tests/test_gpu_body.py -m gpu -v --timeout 200 --timeout-method thread -k "hand or coco" > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; fi
for m in 2 3; do
  ISLPOSE_X3_WIDE7=$m timeout -k 10 300 python3 -u tools/net_layers.py hand 32 368 552 736 > $O/hand_w$m.txt 2>/dev/null || exit 1
done
for r in 1 2; do for m in 2 3; do
  ISLPOSE_X3_WIDE7=$m timeout -k 10 600 python3 -u tools/bench_configs.py --config c3 > $O/c3_w$m.$r.json 2>> $O/err || exit 1
done; done
grep -h "k7\|==" $O/hand_w2.txt; echo; grep -h "k7\|==" $O/hand_w3.txt
cat $O/c3_w*.json | python3 -c "import sys,json; [print(json.loads(l)['frames_per_s']) for l in sys.stdin]"
