export TMPDIR=/tmp
O=gpurun_out/${1:-bl1}; mkdir -p $O
for v in d FUSED d LIST; do
  case $v in
    d) timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/f_$v.json 2>>$O/f.err || exit 1;;
    FUSED) ISLPOSE_FUSED_BLUR=0 timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/f_$v.json 2>>$O/f.err || exit 1;;
    LIST) ISLPOSE_BLUR_LIST=0 timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/f_$v.json 2>>$O/f.err || exit 1;;
  esac
  python3 -c "import json; d=json.load(open('$O/f_$v.json')); print('$v', d['frames_per_s'], d['body_ms_per_frame'], d['hand_ms_per_frame'])"
done
