# C5 pipeline: GPU parity of the overlapped pipeline, then the C5 throughput (sequential vs overlap).
export TMPDIR=/tmp
O=gpurun_out/${1:-c5}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_pipeline.py tests/test_gpu_configs.py -k "pipeline or c5" > $O/tests.log 2>&1 &&
timeout -k 10 400 python3 tools/bench_configs.py --config c5 --batch 32 > $O/c5.json 2> $O/c5.err
rc=$?
tail -5 $O/tests.log; cat $O/c5.json; tail -3 $O/c5.err
exit $rc
