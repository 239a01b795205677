# Round-2 GPU session P: f-v cell-staged tiled kernel -- parity, then sliding / time-lapse A/B.
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/p_summary.txt
timeout -k 10 600 python -u -m pytest tests/test_fv_batch_gpu.py tests/test_disp_gpu.py tests/test_boot_gpu.py tests/test_tli_gpu.py tests/test_sliding_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/p_tests.log 2>&1; rc=$?
echo tests=$rc; tail -4 gpurun_out/p_tests.log
[ $rc -eq 0 ] || exit 1
for c in 1 0 1; do
  DVH_FV_CELLS=$c timeout -k 10 300 python bench.py --workload sliding --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/p.json 2> gpurun_out/p.err || { echo "sliding $c failed"; tail -5 gpurun_out/p.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/p.json')); print('sliding cells=$c', round(d['value']), round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['step_breakdown_ms'].items()})" | tee -a gpurun_out/p_summary.txt
  DVH_FV_CELLS=$c timeout -k 10 200 python tools/bench_timelapse.py > gpurun_out/p_tl.json 2> gpurun_out/p_tl.err || { echo "tl $c failed"; tail -5 gpurun_out/p_tl.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/p_tl.json')); print('timelapse cells=$c', round(d['value']), round(d['ms_per_step'],3), {k: round(x['us'],1) for k,x in d['kernels'].items()}, d['parity'])" | tee -a gpurun_out/p_summary.txt
done
