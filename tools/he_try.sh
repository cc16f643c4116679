export TMPDIR=/tmp
O=gpurun_out/${1:-fin1}; mkdir -p $O
timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/frame.json 2>$O/frame.err && cat $O/frame.json
