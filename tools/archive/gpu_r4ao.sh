# Round 4: kernel trace of the batch-1 Mode R bench step (where a frame's 1.7 ms go).
T=${1:-r4ao}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- python3 bench.py --no-cpu --no-mode-r --e2e-steps 0 --scale 0.5 --batch 1 --steps 40 --warmup 5 > $O/b1.json 2> $O/b1.err
