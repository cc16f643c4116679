export TMPDIR=/tmp
O=gpurun_out/${1:-hf2}; mkdir -p $O
for v in old new old new; do
  if [ $v = old ]; then ISLPOSE_LIB=tools/ab_lib/libislpose_07a1d98.so timeout -k 10 400 python3 bench.py --no-cpu --frame-count 0 --no-mode-r --e2e-steps 0 > $O/b_$v.json 2>>$O/b.err || exit 1
  else timeout -k 10 400 python3 bench.py --no-cpu --frame-count 0 --no-mode-r --e2e-steps 0 > $O/b_$v.json 2>>$O/b.err || exit 1; fi
  python3 -c "import json; d=json.load(open('$O/b_$v.json')); print('$v', d['value'], d['roofline']['frac'])"
done
