# Round-2 GPU session K: the bench's multi-rank step rehearsed with 2 ranks on the box's one GPU (gloo).
set -o pipefail
mkdir -p gpurun_out/r2k
export DVH_DIST_BACKEND=gloo
port=29531
for a in "weights --scaling weak" "weights --scaling strong" "synth10k --scaling strong" "sliding --scaling weak"; do
  port=$((port+1)); set -- $a
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --steps 3 --warmup 1 --workload $1 $2 $3 > gpurun_out/r2k/$1_$3.json 2> gpurun_out/r2k/$1_$3.err || { echo "$a failed"; tail -20 gpurun_out/r2k/$1_$3.err; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/r2k/$1_$3.json') if l.startswith('{')][-1]); print('$a', d['n_gpus'], round(d['value']), round(d['ms_per_step'],2), d['scaling'], d['config']['windows_per_step'], d['config']['windows_per_step_this_rank'], d['cpu_baseline'])"
done
