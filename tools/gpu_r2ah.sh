# Round-2 GPU session AH: VALU register-ring f-v kernel (dvh_disp_fv_ring) -- parity, then time-lapse / sliding A/B.
set -o pipefail
mkdir -p gpurun_out/r2ah
timeout -k 10 400 python -u -m pytest tests/test_fv_batch_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2ah/tests.log 2>&1; rc=$?
echo tests=$rc; tail -3 gpurun_out/r2ah/tests.log
[ $rc -eq 0 ] || exit 1
tl() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python tools/bench_timelapse.py > gpurun_out/r2ah/tl.json 2> gpurun_out/r2ah/tl.err || { echo "tl $tag failed"; tail -5 gpurun_out/r2ah/tl.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/r2ah/tl.json')); print('timelapse $tag', round(d['value']), {k: round(x['us'],1) for k,x in d['kernels'].items()}, d['parity'])"
}
tl mfma A=1 && tl ring DVH_FV_RING=1 && tl ring_G1 DVH_FV_RING=1 DVH_FV_MG=1 && tl ring_G4 DVH_FV_RING=1 DVH_FV_MG=4 || exit 1
for m in 1; do
  DVH_FV_RING=$m timeout -k 10 300 python bench.py --workload sliding --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/r2ah/sl.json 2> gpurun_out/r2ah/sl.err || { echo "sliding $m failed"; tail -5 gpurun_out/r2ah/sl.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r2ah/sl.json')); print('sliding ring=$m', round(d['value']), round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['step_breakdown_ms'].items()})"
done
