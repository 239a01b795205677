set -o pipefail
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/ab_tests.log 2>&1; echo tests_rc=$?; tail -2 gpurun_out/ab_tests.log
for v in "$@"; do
  DVH_LIB=variants/$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/ab_$v.json 2>/dev/null || { echo "$v failed"; break; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v', round(d['ms_per_step'],3), 'ms/step; stack', round(d['roofline']['launch_ms'],3), 'ms', round(d['roofline']['frac']*100,2),'%')"
done
