# End-of-round GPU session: full GPU test suite, smoke, PMC passes + bench line (with CPU baseline)
# + rocprofv3 kernel stats for the headline workload, then the time-lapse bench / PMC / stats.
# Brings back only summaries (gpurun merges <= 64 MiB).   bash tools/gpu_final.sh TAG
set -o pipefail
tag=${1:-r1}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo gpu_tests=$rc; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash tools/pmc.sh $tag > gpurun_out/pmc.log 2>&1 || { echo pmc failed; tail -5 gpurun_out/pmc.log; exit 1; }
cp profiles/${tag}_pmc_summary.json gpurun_out/
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail -5 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 200 python tools/bench_timelapse.py --out gpurun_out/tl.json 2> gpurun_out/tl.err || { echo tl failed; tail -5 gpurun_out/tl.err; exit 1; }
bash tools/pmc_timelapse.sh $tag > gpurun_out/pmc_tl.log 2>&1 || { echo pmc tl failed; tail -5 gpurun_out/pmc_tl.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o $tag --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err; echo prof=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tl -o ${tag}_timelapse --output-format csv -- python tools/bench_timelapse.py > gpurun_out/prof_tl.json 2> gpurun_out/prof_tl.err; echo prof_tl=$?
find gpurun_out -name '*kernel_trace.csv' -delete
rm -rf gpurun_out/pmc_${tag} gpurun_out/pmc_${tag}_timelapse
du -sh gpurun_out
