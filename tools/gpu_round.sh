# One GPU session: variant A/B (+ their VSG tests), full GPU suite, bench with CPU baseline, rocprofv3 kernel stats.
set -o pipefail
bash tools/ab.sh "$@" || exit 1
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo gpu_tests=$rc; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail -5 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r1 --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err; echo prof=$?
find gpurun_out/prof -name "*stats*" | head
