# Round-2 GPU session AC: MFMA f-v kernel, MFMAs interleaved with the sampling (sched_group_barrier).
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ac_summary.txt
V=das_diff_veh_amd/lib/variants
for lib in il4 il8; do
  DVH_LIB=$V/$lib.so timeout -k 10 400 python -u -m pytest tests/test_fv_batch_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ac_tests_$lib.log 2>&1; rc=$?
  echo tests_$lib=$rc; tail -1 gpurun_out/ac_tests_$lib.log
  [ $rc -eq 0 ] || exit 1
done
tl() {  # tag, then env assignments
  tag=$1; shift
  env "$@" timeout -k 10 200 python tools/bench_timelapse.py > gpurun_out/ac_tl.json 2> gpurun_out/ac_tl.err || { echo "tl $tag failed"; tail -5 gpurun_out/ac_tl.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/ac_tl.json')); print('timelapse $tag', round(d['value']), round(d['ms_per_step'],3), {k: round(x['us'],1) for k,x in d['kernels'].items()}, d['parity'])" | tee -a gpurun_out/ac_summary.txt
}
tl default A=1 && tl il4 DVH_LIB=$V/il4.so && tl il8 DVH_LIB=$V/il8.so && tl default2 A=1 || exit 1
