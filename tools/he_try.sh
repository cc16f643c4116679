export TMPDIR=/tmp
O=gpurun_out/${1:-lz3}; mkdir -p $O
for z in d 10 d 10; do
  if [ $z = d ]; then timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/f_$z.json 2>>$O/f.err || exit 1
  else ISLPOSE_LIMB_Z=$z timeout -k 10 300 python3 tools/bench_configs.py --config frame > $O/f_$z.json 2>>$O/f.err || exit 1; fi
  python3 -c "import json; d=json.load(open('$O/f_$z.json')); print('$z', d['frames_per_s'], d['body_ms_per_frame'], d['hand_ms_per_frame'])"
done
