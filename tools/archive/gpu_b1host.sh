# Batch-1 host vs GPU time, with the HIP runtime's device-memory kernel arguments on / off.
T=${1:-b1host}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/b1_host.py > $O/default.txt 2>&1 && cat $O/default.txt &&
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python -u tools/b1_host.py > $O/devk1.txt 2>&1 && cat $O/devk1.txt &&
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 200 python -u tools/b1_host.py > $O/devk0.txt 2>&1 && cat $O/devk0.txt &&
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python -u bench.py --scale 0.5 --batch 1 --steps 60 --warmup 5 --no-cpu --no-mode-r --e2e-steps 0 > $O/b1_k1.json 2>> $O/bench.err &&
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 300 python -u bench.py --scale 0.5 --batch 1 --steps 60 --warmup 5 --no-cpu --no-mode-r --e2e-steps 0 > $O/b1_k0.json 2>> $O/bench.err &&
timeout -k 10 300 python -u bench.py --scale 0.5 --batch 1 --steps 60 --warmup 5 --no-cpu --no-mode-r --e2e-steps 0 > $O/b1_kd.json 2>> $O/bench.err &&
python3 -c "
import json
for k in ('k1','k0','kd'):
    x=json.load(open('$O/b1_%s.json'%k)); print(k, x['value'], x['ms_per_step'])
"
