# Graph replay A/B on the host-heavy configs: C5 (pipelined 1080p video, JSON writer thread) and C3.
T=${1:-graphc5}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for v in 0 1; do
    if [ $v = 0 ]; then export ISLPOSE_NET_GRAPH=0; else unset ISLPOSE_NET_GRAPH; fi
    timeout -k 10 400 python -u tools/bench_configs.py --config c5 > $O/c5_g$v$i.log 2>&1 || exit 1
  done
done
for v in 0 1; do
  if [ $v = 0 ]; then export ISLPOSE_NET_GRAPH=0; else unset ISLPOSE_NET_GRAPH; fi
  timeout -k 10 400 python -u tools/bench_configs.py --config c3 --steps 5 > $O/c3_g$v.log 2>&1 || exit 1
done
for f in $O/c5_g*.log $O/c3_g*.log; do echo $f; grep -h frames_per_s $f | cut -c1-200; done
