# Round-2 GPU session AD: f-v parity at the MFMA kernel's smallest axes; bench.py --workload timelapse
# (1 rank with the CPU baseline; 2 ranks on the one GPU over gloo as a multi-rank rehearsal).
set -o pipefail
mkdir -p gpurun_out/r2ad
timeout -k 10 400 python -u -m pytest tests/test_fv_batch_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2ad/tests.log 2>&1; rc=$?
echo tests=$rc; tail -1 gpurun_out/r2ad/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --workload timelapse > gpurun_out/r2ad/timelapse.json 2> gpurun_out/r2ad/timelapse.err || { echo tl failed; tail -20 gpurun_out/r2ad/timelapse.err; exit 1; }
cat gpurun_out/r2ad/timelapse.json
DVH_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 5 --warmup 1 --workload timelapse > gpurun_out/r2ad/timelapse_2.json 2> gpurun_out/r2ad/timelapse_2.err || { echo "tl 2 ranks failed"; tail -20 gpurun_out/r2ad/timelapse_2.err; exit 1; }
python -c "import json; d=json.loads([l for l in open('gpurun_out/r2ad/timelapse_2.json') if l.startswith('{')][-1]); print('2 ranks', d['n_gpus'], round(d['value']), round(d['ms_per_step'],3), d['scaling'], d['parity'])"
