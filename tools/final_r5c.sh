# Round-5 closing measurements after the last kernel changes (sosfiltfilt matrix-pipe scan, EngP1024 stage tables):
# GPU tests + smoke, the prep and w = 499 lines with CPU baselines, their kernel statistics, the sosfiltfilt kernels'
# PMC, and the host-fed line under rocprofv3 (the staging's asynchronous copies complete under the profiler).
set -o pipefail
mkdir -p gpurun_out
source <(sed -n '/^bench_line()/,/^}/p' tools/gpu.sh)
bash tools/gpu.sh tests || exit 1
bench_line gpurun_out/r5c_bench_prep.json --workload prep --steps 20 --warmup 3 || exit 1
bench_line gpurun_out/r5c_bench_w499.json --w499 || exit 1
bench_line gpurun_out/r5c_bench_weights_w499.json --workload weights --w499 || exit 1
bash tools/gpu.sh prof r5c prep || exit 1
bash tools/gpu.sh profw499 r5c || exit 1
timeout -k 10 400 bash tools/pmc_cmd.sh prep_r5c sosm -- python bench.py --workload prep --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/pmcc_prep_r5c.log 2>&1 || { echo pmc prep failed; tail -3 gpurun_out/pmcc_prep_r5c.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5c_speeds_host -o r5c_speeds_host --output-format csv \
  -- python bench.py --workload speeds-host --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r5c_speeds_host.json \
  2> gpurun_out/prof_r5c_speeds_host.err || { echo speeds-host prof failed; tail -5 gpurun_out/prof_r5c_speeds_host.err; exit 1; }
find gpurun_out -name '*kernel_trace.csv' -delete
grep -ci "timeout\|timed out" gpurun_out/prof_r5c_speeds_host.err || true
echo done
