# Round-2 GPU session AG: single ds_read_b64 instead of merged ds_read2_b64 (8 vs 2 + 2 LDS cycles):
# the f-v kernel's FK corners (default now) and the correlation FFT's stage reads (DVH_NO_READ2 build).
set -o pipefail
mkdir -p gpurun_out/r2ag
V=das_diff_veh_amd/lib/variants
timeout -k 10 400 python -u -m pytest tests/test_fv_batch_gpu.py tests/test_timelapse_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2ag/tests.log 2>&1; rc=$?
echo tests=$rc; tail -1 gpurun_out/r2ag/tests.log
[ $rc -eq 0 ] || exit 1
DVH_LIB=$V/fftnr2.so timeout -k 10 500 python -u -m pytest tests/test_vsg_gpu.py tests/test_synth10k_gpu.py tests/test_sliding_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2ag/tests_fft.log 2>&1; rc=$?
echo tests_fftnr2=$rc; tail -1 gpurun_out/r2ag/tests_fft.log
[ $rc -eq 0 ] || exit 1
tl() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python tools/bench_timelapse.py > gpurun_out/r2ag/tl.json 2> gpurun_out/r2ag/tl.err || { echo "tl $tag failed"; tail -5 gpurun_out/r2ag/tl.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/r2ag/tl.json')); print('timelapse $tag', round(d['value']), {k: round(x['us'],1) for k,x in d['kernels'].items()}, d['parity']['picks_ok'])"
}
bn() {
  tag=$1; wl=$2; shift; shift
  env "$@" timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r2ag/b.json 2> gpurun_out/r2ag/b.err || { echo "bench $tag failed"; tail -5 gpurun_out/r2ag/b.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/r2ag/b.json')); r=d['roofline']; print('$wl $tag', round(d['value']), round(d['ms_per_step'],2), 'launch', round(r['launch_ms'],3), 'frac', round(r['frac'],3))"
}
tl nor2 A=1 && tl read2 DVH_LIB=$V/nor2_0.so && tl nor2b A=1 || exit 1
bn default synth10k A=1 && bn fftnr2 synth10k DVH_LIB=$V/fftnr2.so && bn default2 synth10k A=1 && bn fftnr2b synth10k DVH_LIB=$V/fftnr2.so || exit 1
bn default sliding A=1 && bn fftnr2 sliding DVH_LIB=$V/fftnr2.so || exit 1
