# A/B timing of variant libraries (built with `python -m das_diff_veh_amd.build variants/X.so DEF=1`)
set -o pipefail
for v in "$@"; do
  DVH_LIB=variants/$v.so timeout -k 10 300 python -m pytest tests/test_vsg_gpu.py -m gpu -q -x > gpurun_out/ab_tests_$v.log 2>&1; echo tests_$v=$?; tail -1 gpurun_out/ab_tests_$v.log
done
for v in "$@"; do
  DVH_LIB=variants/$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/ab_$v.json 2>/dev/null || { echo "$v failed"; break; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v', round(d['ms_per_step'],3), 'ms/step; stack', round(d['roofline']['launch_ms'],3), 'ms', round(d['roofline']['frac']*100,2),'%')"
done
