# Parity tests of the VSG kernels with a variant library, then its bench.   bash tools/variant_check.sh NAME...
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  DVH_LIB=variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_vsg_gpu.py tests/test_vsg_stack_more_gpu.py tests/test_integration_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/vc_$v.log 2>&1; rc=$?
  echo "$v tests=$rc: $(tail -1 gpurun_out/vc_$v.log)"
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/vc_$v.log | head -8; continue; }
  DVH_LIB=variants/$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/vc_$v.json 2>/dev/null || { echo "$v bench failed"; continue; }
  python -c "import json;d=json.load(open('gpurun_out/vc_$v.json'));r=d['roofline'];print('$v', round(d['ms_per_step'],3),'ms/step; stack', round(r['launch_ms'],4),'ms', round(r['frac']*100,2),'%')"
done
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/vc_default.json 2>/dev/null && python -c "import json;d=json.load(open('gpurun_out/vc_default.json'));r=d['roofline'];print('default', round(d['ms_per_step'],3),'ms/step; stack', round(r['launch_ms'],4),'ms', round(r['frac']*100,2),'%')"
