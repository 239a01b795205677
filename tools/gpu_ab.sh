# GPU session: full GPU test suite, then A/B benches (default lib, DVH_PAIRED=0, variant libs), then
# a rocprofv3 kernel-stats run of the default bench.   bash tools/gpu_ab.sh [variant ...]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo gpu_tests=$rc; tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit 1
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2], round(d['ms_per_step'],3),'ms/step', round(d['value']/1e6,3),'Mwin/s; stack', round(r['launch_ms'],4),'ms', round(r['frac']*100,2),'%')" "$1" "$2"; }
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/ab_default.json 2> gpurun_out/ab_default.err || { echo default bench failed; tail -5 gpurun_out/ab_default.err; exit 1; }
summ gpurun_out/ab_default.json default
DVH_PAIRED=0 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/ab_legacy.json 2>/dev/null && summ gpurun_out/ab_legacy.json legacy
for v in "$@"; do
  DVH_LIB=variants/$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/ab_$v.json 2>/dev/null || { echo "$v failed"; break; }
  summ gpurun_out/ab_$v.json $v
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r1 --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err; echo prof=$?
