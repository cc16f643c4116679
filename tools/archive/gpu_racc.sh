# resize_acc unroll check: body / hand / pyramid post parity, then C3 / C4 timings (tools/bench_configs.py).
T=${1:-racc}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_body.py tests/test_gpu_hand.py tests/test_gpu_compat.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread \
  -k "post or golden or fused or estimate or hand or pyramid or designed or c4 or scale" > $O/test.log 2>&1; rc=$?
tail -3 $O/test.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/bench_configs.py --config c4 --steps 5 > $O/c4.log 2>&1 && tail -5 $O/c4.log &&
timeout -k 10 600 python -u tools/bench_configs.py --config c3 --steps 5 > $O/c3.log 2>&1 && tail -5 $O/c3.log
