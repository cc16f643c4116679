# Where C5's time goes: host profile (cProfile) and kernel trace of one short C5 run.
export TMPDIR=/tmp
O=gpurun_out/${1:-c5p}; mkdir -p $O
timeout -k 10 300 python3 -m cProfile -o $O/prof.out tools/bench_configs.py --config c5 --c5-batch 32 --c5-frames 64 --c5-videos 1 > $O/c5.json 2> $O/c5.err &&
python3 -c "import pstats; pstats.Stats('$O/prof.out').sort_stats('cumulative').print_stats(45)" > $O/prof_cum.txt &&
python3 -c "import pstats; pstats.Stats('$O/prof.out').sort_stats('tottime').print_stats(30)" > $O/prof_tot.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/bench_configs.py --config c5 --c5-batch 32 --c5-frames 64 --c5-videos 1 > $O/trace.log 2>&1
rc=$?
cat $O/c5.json
exit $rc
