# Round-2 GPU session T: MFMA-filter f-v kernel v2 (host weights, register ring one tile ahead, rolled edge tiles)
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/t_summary.txt
timeout -k 10 400 python -u -m pytest tests/test_fv_batch_gpu.py tests/test_disp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_tests.log 2>&1; rc=$?
echo tests=$rc; tail -4 gpurun_out/t_tests.log
[ $rc -eq 0 ] || exit 1
tl() {  # tag, then env assignments
  tag=$1; shift
  env "$@" timeout -k 10 200 python tools/bench_timelapse.py > gpurun_out/t_tl.json 2> gpurun_out/t_tl.err || { echo "tl $tag failed"; tail -5 gpurun_out/t_tl.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/t_tl.json')); print('timelapse $tag', round(d['value']), round(d['ms_per_step'],3), {k: round(x['us'],1) for k,x in d['kernels'].items()}, d['parity'])" | tee -a gpurun_out/t_summary.txt
}
tl mfma_wpe3 DVH_FV_MFMA=1 && tl cells DVH_FV_MFMA=0 && tl mfma_wpe4 DVH_FV_MFMA=1 DVH_LIB=das_diff_veh_amd/lib/variants/wpe4.so && tl mfma_wpe2 DVH_FV_MFMA=1 DVH_LIB=das_diff_veh_amd/lib/variants/wpe2.so && tl mfma_nosb DVH_FV_MFMA=1 DVH_LIB=das_diff_veh_amd/lib/variants/nosb.so && tl mfma_G2 DVH_FV_MFMA=1 DVH_FV_MG=2 && tl mfma_wpe3b DVH_FV_MFMA=1 || exit 1
for m in 1 0; do
  DVH_FV_MFMA=$m timeout -k 10 300 python bench.py --workload sliding --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/t_sl.json 2> gpurun_out/t_sl.err || { echo "sliding $m failed"; tail -5 gpurun_out/t_sl.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/t_sl.json')); print('sliding mfma=$m', round(d['value']), round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['step_breakdown_ms'].items()})" | tee -a gpurun_out/t_summary.txt
done
