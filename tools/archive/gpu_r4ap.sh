# Round 4: register-resident person assembly -- the post tests, then kernel traces of the batch-1 /
# batch-32 Mode R post with it (default) and with the table merge (ISLPOSE_ASM_REG=0).
T=${1:-r4ap}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_body.py::test_assemble_register_merge_equals_table" "tests/test_gpu_body.py::test_body_post_golden_bit_exact" \
  "tests/test_gpu_body.py::test_designed_maps_batch_bit_exact" "tests/test_gpu_body.py::test_body_estimate_end_to_end" \
  tests/test_gpu_blur_filter.py tests/test_gpu_configs.py tests/test_gpu_compat.py > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; fi
for r in 1 0; do
  ISLPOSE_ASM_REG=$r timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t1_$r -o run -- python3 tools/post_prof.py --batch 1 --iters 20 > $O/t1_$r.log 2>&1 &&
  ISLPOSE_ASM_REG=$r timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t32_$r -o run -- python3 tools/post_prof.py --batch 32 --iters 5 > $O/t32_$r.log 2>&1 || exit 1
done
grep -h post_ms $O/*.log
for d in t1_1 t1_0 t32_1 t32_0; do grep -h assemble $O/$d/run_kernel_stats.csv | cut -d, -f1-5 | sed "s/^/$d /"; done
timeout -k 10 120 python3 tools/asm_prof.py 1 > $O/asm_b1_reg.txt 2>&1 &&
ISLPOSE_ASM_REG=0 timeout -k 10 120 python3 tools/asm_prof.py 1 > $O/asm_b1_tab.txt 2>&1 &&
timeout -k 10 120 python3 tools/asm_prof.py 32 > $O/asm_b32_reg.txt 2>&1
