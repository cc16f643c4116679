# A/B: bench with and without the per-op HIP events in the timed region (interleaved)
set -o pipefail
O=gpurun_out/opt; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu --e2e-steps 0 --steps 20 > $O/on.$i.json 2>> $O/err.log || exit 1
  timeout -k 10 300 python bench.py --no-cpu --e2e-steps 0 --steps 20 --no-op-timing > $O/off.$i.json 2>> $O/err.log || exit 1
  echo "pair $i: on $(python -c "import json;print(json.load(open('$O/on.$i.json'))['value'])") off $(python -c "import json;print(json.load(open('$O/off.$i.json'))['value'])")"
done
