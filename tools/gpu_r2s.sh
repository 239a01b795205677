# Round-2 GPU session S: MFMA-filter f-v kernel (dvh_disp_fv_mfma) -- parity, then time-lapse / sliding A/B.
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/s_summary.txt
timeout -k 10 400 python -u -m pytest tests/test_fv_batch_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s_tests.log 2>&1; rc=$?
echo tests=$rc; tail -4 gpurun_out/s_tests.log
[ $rc -eq 0 ] || exit 1
for m in 1 0 1; do
  DVH_FV_MFMA=$m timeout -k 10 200 python tools/bench_timelapse.py > gpurun_out/s_tl.json 2> gpurun_out/s_tl.err || { echo "tl $m failed"; tail -5 gpurun_out/s_tl.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/s_tl.json')); print('timelapse mfma=$m', round(d['value']), round(d['ms_per_step'],3), {k: round(x['us'],1) for k,x in d['kernels'].items()}, d['parity'])" | tee -a gpurun_out/s_summary.txt
done
for g in 1 2 4 8; do
  DVH_FV_MFMA=1 DVH_FV_MG=$g timeout -k 10 200 python tools/bench_timelapse.py > gpurun_out/s_tl.json 2> gpurun_out/s_tl.err || { echo "tl G=$g failed"; tail -5 gpurun_out/s_tl.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/s_tl.json')); print('timelapse mfma G=$g', round(d['value']), round(d['ms_per_step'],3), {k: round(x['us'],1) for k,x in d['kernels'].items()}, d['parity'])" | tee -a gpurun_out/s_summary.txt
done
for m in 1 0; do
  DVH_FV_MFMA=$m timeout -k 10 300 python bench.py --workload sliding --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/s_sl.json 2> gpurun_out/s_sl.err || { echo "sliding $m failed"; tail -5 gpurun_out/s_sl.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/s_sl.json')); print('sliding mfma=$m', round(d['value']), round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['step_breakdown_ms'].items()})" | tee -a gpurun_out/s_summary.txt
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
DVH_FV_MFMA=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s -o s --output-format csv -- python tools/bench_timelapse.py > /dev/null 2> gpurun_out/s_prof.err; echo prof=$?
