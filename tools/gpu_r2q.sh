# Round-2 GPU session Q: tdft GEMM double-buffered rounds -- dispersion parity, then time-lapse / sliding A/B.
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/q_summary.txt
timeout -k 10 600 python -u -m pytest tests/test_fv_batch_gpu.py tests/test_disp_gpu.py tests/test_fk_gpu.py tests/test_boot_gpu.py tests/test_tli_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/q_tests.log 2>&1; rc=$?
echo tests=$rc; tail -4 gpurun_out/q_tests.log
[ $rc -eq 0 ] || exit 1
for v in default tdftold tu4 default; do
  lib=""; [ $v = default ] || lib=das_diff_veh_amd/lib/variants/$v.so
  DVH_LIB=$lib timeout -k 10 200 python tools/bench_timelapse.py > gpurun_out/q_tl.json 2> gpurun_out/q_tl.err || { echo "tl $v failed"; tail -5 gpurun_out/q_tl.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/q_tl.json')); print('timelapse $v', round(d['value']), round(d['ms_per_step'],3), {k: round(x['us'],1) for k,x in d['kernels'].items()}, round(d['kernels']['tdft_gemm_kernel']['frac'],3), d['parity'])" | tee -a gpurun_out/q_summary.txt
done
