# Round-2 GPU session AQ: same-box A/B of tools/variants/scales_overlap.patch (committed tree, patched, committed again).
set -o pipefail
mkdir -p gpurun_out/r2aq
cp das_diff_veh_amd/lib/libdvh.so gpurun_out/r2aq_base.so
bn() {
  tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r2aq/b_$tag.json 2> gpurun_out/r2aq/b.err || { echo "bench $tag failed"; tail -5 gpurun_out/r2aq/b.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/r2aq/b_$tag.json')); print('$tag', round(d['value']), round(d['ms_per_step'],2), round(d['roofline']['launch_ms'],3), {k: round(v,3) for k,v in d['step_breakdown_ms'].items()})"
}
bn base A=1 || exit 1
cp bench.py gpurun_out/r2aq_bench_base.py
patch -p1 < tools/variants/scales_overlap.patch > /dev/null || { echo "patch failed"; exit 1; }
timeout -k 10 600 python -c "from das_diff_veh_amd.build import build; build()" > /dev/null || { echo "build failed"; exit 1; }
bn patched A=1 || exit 1
cp das_diff_veh_amd/lib/libdvh.so gpurun_out/r2aq_patched.so
DVH_LIB=gpurun_out/r2aq_base.so bn base_lib_patched_bench A=1 || exit 1
cp gpurun_out/r2aq_bench_base.py bench.py
bn patched_lib_base_bench A=1 && bn base2 DVH_LIB=gpurun_out/r2aq_base.so || exit 1
rm -f gpurun_out/r2aq_*.so
