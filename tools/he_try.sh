export TMPDIR=/tmp
O=gpurun_out/${1:-he6}; mkdir -p $O
timeout -k 10 300 python3 tools/bench_configs.py --config frame --frame-count 64 > $O/frame.json 2>$O/frame.err &&
timeout -k 10 300 python3 tools/frame_cprof.py 48 > $O/cprof.txt 2>&1 &&
timeout -k 10 300 python3 tools/upload_micro.py > $O/upload.txt 2>&1
rc=$?; cat $O/frame.json; head -45 $O/cprof.txt; cat $O/upload.txt; exit $rc
