# Round-2 GPU session AN: per-batch scales overlapped on side streams + one zero kernel instead of the
# two-fill memset in the validated launch -- bench-job parity, then the headline bench.
set -o pipefail
mkdir -p gpurun_out/r2an
timeout -k 10 500 python -u -m pytest tests/test_bench_job_gpu.py tests/test_synth10k_gpu.py tests/test_vsg_stack_more_gpu.py tests/test_distributed_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2an/tests.log 2>&1; rc=$?
echo tests=$rc; tail -1 gpurun_out/r2an/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r2an/tests.log | head -8; exit 1; }
for k in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r2an/bench$k.json 2> gpurun_out/r2an/bench.err || { echo "bench failed"; tail -5 gpurun_out/r2an/bench.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r2an/bench$k.json')); print('synth10k', round(d['value']), round(d['ms_per_step'],2), round(d['roofline']['frac'],3), {k: round(v,3) for k,v in d['step_breakdown_ms'].items()})"
done
