# Round-2 GPU session B: validated (fused-validity) stack launch -- tests, then bench fused vs separate.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_plan_gpu.py tests/test_synth10k_gpu.py tests/test_vsg_gpu.py tests/test_bench_job_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/b_tests.log 2>&1; rc=$?
echo tests=$rc; tail -15 gpurun_out/b_tests.log
[ $rc -eq 0 ] || exit 1
for wl in synth10k weights; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --steps 5 > gpurun_out/b_$wl.json 2> gpurun_out/b_$wl.err || { tail -20 gpurun_out/b_$wl.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/b_$wl.json')); print('$wl fused', round(d['value']), round(d['ms_per_step'],2), d['step_breakdown_ms'], round(d['roofline']['frac'],3), round(d['roofline']['correlation_frac'],3))"
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --steps 5 --separate-validity > gpurun_out/b_${wl}_sep.json 2> gpurun_out/b_${wl}_sep.err || { tail -20 gpurun_out/b_${wl}_sep.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/b_${wl}_sep.json')); print('$wl separate', round(d['value']), round(d['ms_per_step'],2), d['step_breakdown_ms'])"
done
