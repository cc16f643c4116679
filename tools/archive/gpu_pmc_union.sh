export TMPDIR=/tmp
for u in 1 2; do
  ISLPOSE_X3_UNION=$u bash tools/archive/gpu_pmc_cb.sh pmc_u$u "3 128 128 46 82 32" x3 || exit 1
  python tools/pmc_cb_summary.py gpurun_out/pmc_u$u > gpurun_out/pmc_u$u/summary.txt
  cat gpurun_out/pmc_u$u/summary.txt
done
