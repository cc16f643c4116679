# Host profile (cProfile, main thread) of the C5 overlapped pass only.
export TMPDIR=/tmp
O=gpurun_out/${1:-c5h}; mkdir -p $O
timeout -k 10 300 python3 -m cProfile -o $O/prof.out tools/bench_configs.py --config c5 --c5-batch 32 --c5-frames 96 --c5-videos 2 --c5-overlap-only > $O/c5.json 2> $O/c5.err &&
python3 -c "import pstats; pstats.Stats('$O/prof.out').sort_stats('cumulative').print_stats(60)" > $O/prof_cum.txt &&
python3 -c "import pstats; pstats.Stats('$O/prof.out').sort_stats('tottime').print_stats(40)" > $O/prof_tot.txt
rc=$?
cat $O/c5.json
exit $rc
