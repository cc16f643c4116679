export TMPDIR=/tmp
O=gpurun_out/r5q; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fused.py -k c12 tests/test_gpu_body.py::test_timed_config_forward_vs_oracle > $O/tests.log 2>&1 &&
bash tools/ab_bench.sh r5q p1: p2:ISLPOSE_C12=2 p1b: p2b:ISLPOSE_C12=2 &&
timeout -k 10 200 python3 tools/op_table.py --batch 32 --runs 5 > $O/ops_p1.txt 2>&1 &&
ISLPOSE_C12=2 timeout -k 10 200 python3 tools/op_table.py --batch 32 --runs 5 > $O/ops_p2.txt 2>&1
