# FRAME leg A/B of the host-side upload copy.  usage: bash tools/ab_upload.sh <tag>
export TMPDIR=/tmp
T=${1:-up}; O=gpurun_out/$T; mkdir -p $O
for k in 1 2 3; do
  timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/frame_$k.json 2> $O/frame_$k.err || exit 1
  python3 -c "
import json; d=json.load(open('$O/frame_$k.json')); print('$k', d['frames_per_s'], d['body_ms_per_frame'], d['hand_ms_per_frame'])"
done
