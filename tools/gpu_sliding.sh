# Sliding-pivot workload (BASELINE configs[3]) on one GPU: its parity tests, PMC passes, bench line
# and rocprofv3 kernel stats.   bash tools/gpu_sliding.sh TAG
set -o pipefail
tag=${1:-r1}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sliding_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sl_tests.log 2>&1 || { tail -30 gpurun_out/sl_tests.log; exit 1; }
tail -1 gpurun_out/sl_tests.log
bash tools/pmc.sh $tag sliding > gpurun_out/pmc_sl.log 2>&1 || { echo pmc failed; tail -5 gpurun_out/pmc_sl.log; exit 1; }
timeout -k 10 400 python bench.py --workload sliding --steps 5 --warmup 1 > gpurun_out/sl_bench.json 2> gpurun_out/sl_bench.err || { tail -5 gpurun_out/sl_bench.err; exit 1; }
cat gpurun_out/sl_bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sl -o ${tag}_sliding --output-format csv -- python bench.py --workload sliding --steps 5 --warmup 1 > gpurun_out/prof_sl_bench.json 2> gpurun_out/prof_sl.err; echo prof=$?
# bring back only the summaries (gpurun merges at most 64 MiB of gpurun_out/)
cp profiles/${tag}_pmc_summary_sliding.json gpurun_out/
find gpurun_out -name '*kernel_trace.csv' -delete
rm -rf gpurun_out/pmc_${tag}_sliding
ls -la gpurun_out gpurun_out/prof_sl/* | head -20
