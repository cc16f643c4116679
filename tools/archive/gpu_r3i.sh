# Round-3 checkpoint: smoke, -m gpu suite, bench Mode N / Mode R (b32, b1), per-op tables.
T=${1:-r3i}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
exec_rc=0
bash tools/archive/gpu_r3h.sh $T
