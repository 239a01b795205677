T="tests/test_vsg_gpu.py tests/test_vsg_stack_more_gpu.py tests/test_synth10k_gpu.py tests/test_sliding_gpu.py tests/test_bench_job_gpu.py"
for e in f500 q; do DVH_VSG_ENGINE=$e timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t5_$e.log 2>&1; rc=$?; echo "tests $e"; tail -2 gpurun_out/t5_$e.log | cut -c 1-300; [ $rc -eq 0 ] || exit 1; done
run() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 3 $BARGS > gpurun_out/b5_$tag.json 2> gpurun_out/b5_$tag.err || exit 1; python -c "import json; d=json.load(open('gpurun_out/b5_$tag.json')); r=d['roofline']; print('$tag', round(d['value']), round(d['ms_per_step'],2), 'launch', round(r['launch_ms'],3), 'frac', round(r['frac'],3))"; }
run f500_skip DVH_VSG_ENGINE=f500
run f500_noskip DVH_VSG_ENGINE=f500 DVH_LIB=das_diff_veh_amd/lib/variants/noskip.so
run q_skip DVH_VSG_ENGINE=q
run q_noskip DVH_VSG_ENGINE=q DVH_LIB=das_diff_veh_amd/lib/variants/noskip.so
BARGS=--separate-validity run q_sep DVH_VSG_ENGINE=q
