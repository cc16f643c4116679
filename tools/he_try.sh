export TMPDIR=/tmp
O=gpurun_out/${1:-he17}; mkdir -p $O
for g in 11 01 11 01; do
  ISLPOSE_FRAME_GRAPH=$g timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/frame_$g.json 2>>$O/frame.err || exit 1
  python3 -c "import json; d=json.load(open('$O/frame_$g.json')); print('$g', d['frames_per_s'], d['body_ms_per_frame'], d['hand_ms_per_frame'])"
done
