# A/B of variant libraries on the stack launch (tools/exp_stack.py, HIP events), one box, one session:
#     bash tools/ab_stack.sh "WORKLOAD_ARGS" base v1 v2 ...     (base = das_diff_veh_amd/lib/libdvh.so, vN = variants/vN.so)
# -> gpurun_out/ab_<lib>_<tag>.json per library; every step under its own time limit, the first failure ends the run.
set -o pipefail
wargs=$1; shift
tag=$(echo "$wargs" | tr -c 'a-z0-9' '_' | cut -c1-24)
for v in "$@"; do
  lib=das_diff_veh_amd/lib/libdvh.so; [ "$v" = base ] || lib=variants/$v.so
  DVH_LIB=$lib timeout -k 10 240 python tools/exp_stack.py $wargs > gpurun_out/ab_${v}_$tag.json 2> gpurun_out/ab_${v}_$tag.err \
    || { echo "$v failed"; tail -3 gpurun_out/ab_${v}_$tag.err; exit 1; }
  echo "$v: $(cat gpurun_out/ab_${v}_$tag.json)"
done
