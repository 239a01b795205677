# Round-2 GPU session AB (final profiles): full GPU suite + smoke, headline PMC passes (calibrated traffic),
# headline bench with CPU baseline + rocprofv3 stats, time-lapse bench + stats + PMC, sliding bench.
#     bash tools/gpu_r2ab.sh TAG
set -o pipefail
tag=${1:-r2h}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1; rc=$?
echo gpu_tests=$rc; tail -2 gpurun_out/ab_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ab_smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/ab_smoke.log; exit 1; }
tail -1 gpurun_out/ab_smoke.log
bash tools/pmc.sh $tag > gpurun_out/ab_pmc.log 2>&1 || { echo pmc failed; tail -5 gpurun_out/ab_pmc.log; exit 1; }
cp profiles/${tag}_pmc_summary.json gpurun_out/
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/ab_bench.err || { echo bench failed; tail -5 gpurun_out/ab_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${tag}_bench.json')); r=d['roofline']; print('bench', round(d['value']), round(d['ms_per_step'],2), 'frac', round(r['frac'],3), 'traffic', r['traffic'], r['traffic_source'], 'valu', d.get('valu_roofline',{}).get('frac'))"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab -o ${tag}_bench --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${tag}_prof_bench.json 2> gpurun_out/ab_prof.err; echo prof=$?
timeout -k 10 200 python tools/bench_timelapse.py --out gpurun_out/${tag}_timelapse.json > /dev/null 2> gpurun_out/ab_tl.err || { echo tl failed; tail -5 gpurun_out/ab_tl.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab -o ${tag}_tl --output-format csv -- python tools/bench_timelapse.py > /dev/null 2> gpurun_out/ab_proftl.err; echo proftl=$?
bash tools/pmc_timelapse.sh $tag > gpurun_out/ab_pmctl.log 2>&1; echo pmctl=$?
timeout -k 10 300 python bench.py --workload sliding --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/${tag}_bench_sliding.json 2> gpurun_out/ab_sl.err || { echo sliding failed; tail -5 gpurun_out/ab_sl.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${tag}_bench_sliding.json')); print('sliding', round(d['value']), round(d['ms_per_step'],2))"
