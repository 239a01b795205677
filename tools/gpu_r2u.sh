# Round-2 GPU session U: MFMA f-v kernel as the default for large batches -- dispersion-path GPU tests,
# time-lapse bench + rocprofv3 kernel stats + PMC, sliding bench.   bash tools/gpu_r2u.sh TAG
set -o pipefail
tag=${1:-r2c}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_fv_batch_gpu.py tests/test_disp_gpu.py tests/test_fk_gpu.py tests/test_boot_gpu.py tests/test_tli_gpu.py tests/test_sliding_gpu.py tests/test_distributed_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/u_tests.log 2>&1; rc=$?
echo tests=$rc; tail -3 gpurun_out/u_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/bench_timelapse.py --out gpurun_out/${tag}_timelapse.json > /dev/null 2> gpurun_out/u_tl.err || { echo tl failed; tail -5 gpurun_out/u_tl.err; exit 1; }
cat gpurun_out/${tag}_timelapse.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_u -o ${tag}_tl --output-format csv -- python tools/bench_timelapse.py > /dev/null 2> gpurun_out/u_prof.err; echo prof=$?
bash tools/pmc_timelapse.sh $tag > gpurun_out/u_pmc.log 2>&1; echo pmc=$?; tail -3 gpurun_out/u_pmc.log
timeout -k 10 300 python bench.py --workload sliding --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/${tag}_bench_sliding.json 2> gpurun_out/u_sl.err || { echo sliding failed; tail -5 gpurun_out/u_sl.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${tag}_bench_sliding.json')); print('sliding', round(d['value']), round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['step_breakdown_ms'].items()})"
