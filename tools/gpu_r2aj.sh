# Round-2 GPU session AJ: the validity scan in the correlation's pass order (DVH_SCAN_ORDER) and with
# cache-allocating loads (DVH_SCAN_AUX=0): does the scan re-read what the correlation just loaded from the caches?
set -o pipefail
mkdir -p gpurun_out/r2aj
V=das_diff_veh_amd/lib/variants
DVH_LIB=$V/scanord_a0.so timeout -k 10 400 python -u -m pytest tests/test_synth10k_gpu.py tests/test_vsg_stack_more_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2aj/tests.log 2>&1; rc=$?
echo tests=$rc; tail -1 gpurun_out/r2aj/tests.log
[ $rc -eq 0 ] || exit 1
bn() {
  tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r2aj/b_$tag.json 2> gpurun_out/r2aj/b.err || { echo "bench $tag failed"; tail -5 gpurun_out/r2aj/b.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/r2aj/b_$tag.json')); r=d['roofline']; print('$tag', round(d['value']), round(d['ms_per_step'],2), 'launch', round(r['launch_ms'],3), 'frac', round(r['frac'],3))"
}
bn default A=1 && bn scanord DVH_LIB=$V/scanord.so && bn scanord_a0 DVH_LIB=$V/scanord_a0.so && bn a0 DVH_LIB=$V/a0.so && bn default2 A=1 && bn scanord2 DVH_LIB=$V/scanord.so && bn scanord_a0_2 DVH_LIB=$V/scanord_a0.so || exit 1
