# Multi-rank rehearsal on a one-GPU box: bench.py --gpus 2 (self-spawned ranks) and under
# torch.distributed.run (the driver's launch), both ranks on the one card.  usage: bash tools/mg_rehearsal.sh
export TMPDIR=/tmp
O=gpurun_out/r6mg; mkdir -p $O
timeout -k 10 400 python3 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --e2e-steps 0 --no-mode-r > $O/spawn2.json 2> $O/spawn2.err &&
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --e2e-steps 0 --no-mode-r > $O/run2.json 2> $O/run2.err
rc=$?
python3 -c "
import json
for f in ('spawn2','run2'):
    try:
        d=json.load(open('$O/'+f+'.json')); print(f, d['value'], d['n_gpus'], d['ranks'], 'frame', (d.get('frame') or {}).get('frames_per_s'))
    except Exception as e: print(f, 'n/a', e)
"
exit $rc
