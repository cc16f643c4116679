export TMPDIR=/tmp; mkdir -p gpurun_out/r1p
B="python3 bench.py --no-cpu --steps 3 --warmup 1"
timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/r1p/bench.json 2> gpurun_out/r1p/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1p/trace -o run -- $B > gpurun_out/r1p/trace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r1p/fetch -o run -- $B > gpurun_out/r1p/fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r1p/write -o run -- $B > gpurun_out/r1p/write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r1p/sq -o run -- $B > gpurun_out/r1p/sq.log 2>&1
echo rc=$?
cat gpurun_out/r1p/bench.json
