# Round-2 GPU session AL: the complement scan (DVH_SCAN_COMPLEMENT: the scan skips what the correlation
# waves validate, traffic ~1.0x) again, now with the scan in the correlation's pass order.
set -o pipefail
mkdir -p gpurun_out/r2al
V=das_diff_veh_amd/lib/variants
DVH_LIB=$V/compl_ord.so timeout -k 10 400 python -u -m pytest tests/test_synth10k_gpu.py tests/test_vsg_stack_more_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2al/tests.log 2>&1; rc=$?
echo tests=$rc; tail -1 gpurun_out/r2al/tests.log
[ $rc -eq 0 ] || exit 1
bn() {
  tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r2al/b_$tag.json 2> gpurun_out/r2al/b.err || { echo "bench $tag failed"; tail -5 gpurun_out/r2al/b.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/r2al/b_$tag.json')); r=d['roofline']; print('$tag', round(d['value']), round(d['ms_per_step'],2), 'launch', round(r['launch_ms'],3), 'frac', round(r['frac'],3))"
}
bn default A=1 && bn compl_ord DVH_LIB=$V/compl_ord.so && bn compl_idx DVH_LIB=$V/compl_idx.so && bn default2 A=1 && bn compl_ord2 DVH_LIB=$V/compl_ord.so || exit 1
