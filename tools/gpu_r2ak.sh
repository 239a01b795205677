# Round-2 GPU session AK: one geometry launch per synth10k step (DevicePlan.slice) -- parity, then the headline bench.
set -o pipefail
mkdir -p gpurun_out/r2ak
timeout -k 10 400 python -u -m pytest tests/test_plan_gpu.py tests/test_bench_job_gpu.py tests/test_synth10k_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2ak/tests.log 2>&1; rc=$?
echo tests=$rc; tail -1 gpurun_out/r2ak/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r2ak/tests.log | head -8; exit 1; }
for k in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r2ak/bench$k.json 2> gpurun_out/r2ak/bench.err || { echo "bench failed"; tail -5 gpurun_out/r2ak/bench.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r2ak/bench$k.json')); print('synth10k', round(d['value']), round(d['ms_per_step'],2), round(d['roofline']['frac'],3), {k: round(v,3) for k,v in d['step_breakdown_ms'].items()})"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 --scaling strong > gpurun_out/r2ak/bench_strong.json 2> gpurun_out/r2ak/bench.err || { echo "strong failed"; tail -5 gpurun_out/r2ak/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r2ak/bench_strong.json')); print('strong', round(d['value']), round(d['ms_per_step'],2))"
