# Two-stage fused post (large frames): body / compat / configs tests, C5, Mode R bench.
export TMPDIR=/tmp
T=${1:-fuse2}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_body.py tests/test_gpu_compat.py tests/test_gpu_configs.py tests/test_pipeline.py -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; fi
for r in 1 2; do for fb in 0 1; do
  ISLPOSE_FUSED_BLUR=$fb timeout -k 10 600 python3 -u tools/bench_configs.py --config c5 --c5-overlap-only > $O/c5_f$fb.$r.json 2>> $O/err || exit 1
done; done
cat $O/c5_f*.json | python3 -c "import sys,json; [print(json.loads(l)['overlap_frames_per_s']) for l in sys.stdin]"
