# Batch-1 host enqueue vs GPU time (isl_net_forward without the synchronous range check), graph replay on / off.
T=${1:-b1host2}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/b1_host.py > $O/on.txt 2>&1 && cat $O/on.txt &&
ISLPOSE_NET_GRAPH=0 timeout -k 10 200 python -u tools/b1_host.py > $O/off.txt 2>&1 && cat $O/off.txt &&
timeout -k 10 200 python -u tools/b1_host.py --batch 32 > $O/on32.txt 2>&1 && cat $O/on32.txt &&
ISLPOSE_NET_GRAPH=0 timeout -k 10 200 python -u tools/b1_host.py --batch 32 > $O/off32.txt 2>&1 && cat $O/off32.txt
