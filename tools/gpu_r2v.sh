# Round-2 GPU session V: MFMA f-v kernel, two-stage sample pipeline -- parity, then variants on the time-lapse batch.
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/v_summary.txt
timeout -k 10 400 python -u -m pytest tests/test_fv_batch_gpu.py tests/test_disp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/v_tests.log 2>&1; rc=$?
echo tests=$rc; tail -4 gpurun_out/v_tests.log
[ $rc -eq 0 ] || exit 1
tl() {  # tag, then env assignments
  tag=$1; shift
  env "$@" timeout -k 10 200 python tools/bench_timelapse.py > gpurun_out/v_tl.json 2> gpurun_out/v_tl.err || { echo "tl $tag failed"; tail -5 gpurun_out/v_tl.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/v_tl.json')); print('timelapse $tag', round(d['value']), round(d['ms_per_step'],3), {k: round(x['us'],1) for k,x in d['kernels'].items()}, d['parity'])" | tee -a gpurun_out/v_summary.txt
}
V=das_diff_veh_amd/lib/variants
tl default A=1 && tl il6 DVH_LIB=$V/il6.so && tl il3 DVH_LIB=$V/il3.so && tl nt0 DVH_LIB=$V/nt0.so && tl sb0 DVH_LIB=$V/sb0.so && tl blds0 DVH_LIB=$V/blds0.so && tl G2 DVH_FV_MG=2 && tl default2 A=1 || exit 1
