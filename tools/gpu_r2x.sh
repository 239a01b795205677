# Round-2 GPU session X: MFMA f-v kernel with compact tables (q, packed interval/cell), GI images per wave.
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/x_summary.txt
V=das_diff_veh_amd/lib/variants
timeout -k 10 400 python -u -m pytest tests/test_fv_batch_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/x_tests.log 2>&1; rc=$?
echo tests=$rc; tail -3 gpurun_out/x_tests.log
[ $rc -eq 0 ] || exit 1
DVH_LIB=$V/gi1.so timeout -k 10 400 python -u -m pytest tests/test_fv_batch_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/x_tests1.log 2>&1; rc=$?
echo tests_gi1=$rc; tail -2 gpurun_out/x_tests1.log
[ $rc -eq 0 ] || exit 1
tl() {  # tag, then env assignments
  tag=$1; shift
  env "$@" timeout -k 10 200 python tools/bench_timelapse.py > gpurun_out/x_tl.json 2> gpurun_out/x_tl.err || { echo "tl $tag failed"; tail -5 gpurun_out/x_tl.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/x_tl.json')); print('timelapse $tag', round(d['value']), round(d['ms_per_step'],3), {k: round(x['us'],1) for k,x in d['kernels'].items()}, d['parity'])" | tee -a gpurun_out/x_summary.txt
}
tl gi2 A=1 && tl gi1 DVH_LIB=$V/gi1.so && tl gi2nopair DVH_LIB=$V/gi2sb0.so && tl gi2_G4 DVH_FV_MG=4 && tl gi1_G1 DVH_LIB=$V/gi1.so DVH_FV_MG=1 && tl cells DVH_FV_MFMA=0 && tl gi2b A=1 || exit 1
for m in 1; do
  DVH_FV_MFMA=$m timeout -k 10 300 python bench.py --workload sliding --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/x_sl.json 2> gpurun_out/x_sl.err || { echo "sliding $m failed"; tail -5 gpurun_out/x_sl.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/x_sl.json')); print('sliding mfma=$m', round(d['value']), round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['step_breakdown_ms'].items()})" | tee -a gpurun_out/x_summary.txt
done
