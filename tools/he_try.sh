export TMPDIR=/tmp
O=gpurun_out/${1:-frs}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- python3 tools/bench_configs.py --config frame --frame-count 16 --frame-repeat 1 > $O/t.log 2>&1
