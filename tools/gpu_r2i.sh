# Round-2 GPU session I: LDS-DMA ring scan -- validity parity tests, then A/B of ring sizes.
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/i_summary.txt
timeout -k 10 400 python -u -m pytest tests/test_vsg_gpu.py tests/test_synth10k_gpu.py tests/test_bench_job_gpu.py tests/test_vsg_stack_more_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/i_tests.log 2>&1; rc=$?
echo tests=$rc; tail -4 gpurun_out/i_tests.log
[ $rc -eq 0 ] || exit 1
summ() { python -c "import json,sys; d=json.load(open('$1')); b=d['step_breakdown_ms']; print('$2', round(d['value']), 'step', round(d['ms_per_step'],2), 'stack', round(b['stack'],3), 'frac', round(d['roofline']['frac'],3))"; }
for v in default ring0 ring8 default; do
  lib=""; [ $v = default ] || lib=das_diff_veh_amd/lib/variants/$v.so
  for wl in synth10k weights; do
    DVH_LIB=$lib timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --steps 4 --warmup 1 > gpurun_out/i.json 2> gpurun_out/i.err || { echo "$v $wl failed"; tail -5 gpurun_out/i.err; exit 1; }
    summ gpurun_out/i.json "$v $wl" | tee -a gpurun_out/i_summary.txt
  done
done
