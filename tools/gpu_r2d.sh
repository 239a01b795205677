# Round-2 GPU session D: pivot tables -- parity tests, then bench with / without tables.
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/d_summary.txt
timeout -k 10 400 python -u -m pytest tests/test_vsg_gpu.py tests/test_boot_gpu.py tests/test_fk_gpu.py tests/test_synth10k_gpu.py tests/test_bench_job_gpu.py tests/test_integration_gpu.py tests/test_vsg_stack_more_gpu.py tests/test_sliding_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/d_tests.log 2>&1; rc=$?
echo tests=$rc; tail -15 gpurun_out/d_tests.log
[ $rc -eq 0 ] || exit 1
summ() { python -c "import json,sys; d=json.load(open('$1')); b=d['step_breakdown_ms']; print('$2', round(d['value']), 'step', round(d['ms_per_step'],2), {k: round(v,2) for k,v in b.items()}, 'frac', round(d['roofline']['frac'],3))"; }
for wl in synth10k weights; do
  for v in "" "--no-pivot-table" "--separate-validity" "--separate-validity --no-pivot-table"; do
    timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --steps 4 --warmup 1 $v > gpurun_out/d.json 2> gpurun_out/d.err || { echo "$wl $v failed"; tail -5 gpurun_out/d.err; exit 1; }
    summ gpurun_out/d.json "$wl $v" | tee -a gpurun_out/d_summary.txt
  done
done
