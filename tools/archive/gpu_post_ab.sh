# Post kernels: parity tests, then post timing and the bench.
export TMPDIR=/tmp
O=gpurun_out/${1:-pab}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_body.py tests/test_gpu_hand.py tests/test_gpu_compat.py tests/test_gpu_configs.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 tools/post_timing.py > $O/post.txt 2>&1 && cat $O/post.txt
timeout -k 10 300 python3 tools/post_timing.py 0.5 > $O/post_r.txt 2>&1 && cat $O/post_r.txt
timeout -k 10 300 python3 bench.py --no-cpu --e2e-steps 0 > $O/b.json 2>> $O/bench.err || exit 1
python3 -c "import json; d=json.load(open('$O/b.json')); print(d['value'], d['ms_per_step'], d['post'])"
