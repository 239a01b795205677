# Round-2 GPU session AA: row-block time-DFT GEMM (tdft_rows_kernel, LDS-staged twiddles) -- dispersion
# parity, then time-lapse / sliding A/B against the split-K kernel (DVH_TDFT_ROWS=0).
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/aa_summary.txt
timeout -k 10 500 python -u -m pytest tests/test_fv_batch_gpu.py tests/test_disp_gpu.py tests/test_fk_gpu.py tests/test_boot_gpu.py tests/test_tli_gpu.py tests/test_sliding_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/aa_tests.log 2>&1; rc=$?
echo tests=$rc; tail -3 gpurun_out/aa_tests.log
[ $rc -eq 0 ] || exit 1
tl() {  # tag, then env assignments
  tag=$1; shift
  env "$@" timeout -k 10 200 python tools/bench_timelapse.py > gpurun_out/aa_tl.json 2> gpurun_out/aa_tl.err || { echo "tl $tag failed"; tail -5 gpurun_out/aa_tl.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/aa_tl.json')); print('timelapse $tag', round(d['value']), round(d['ms_per_step'],3), {k: round(x['us'],1) for k,x in d['kernels'].items()}, d['parity'])" | tee -a gpurun_out/aa_summary.txt
}
tl rows A=1 && tl splitk DVH_TDFT_ROWS=0 && tl rows2 A=1 && tl rows3 A=1 || exit 1
for m in 1; do
  DVH_TDFT_ROWS=$m timeout -k 10 300 python bench.py --workload sliding --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/aa_sl.json 2> gpurun_out/aa_sl.err || { echo "sliding $m failed"; tail -5 gpurun_out/aa_sl.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/aa_sl.json')); print('sliding rows=$m', round(d['value']), round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['step_breakdown_ms'].items()})" | tee -a gpurun_out/aa_summary.txt
done
