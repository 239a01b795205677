# Round-2 GPU session AO: tools/variants/scales_overlap.patch applied on the box (the local tree stays at the
# measured state), library rebuilt there, then tools/gpu_r2an.sh (parity + bench).
set -o pipefail
patch -p1 < tools/variants/scales_overlap.patch > /dev/null || { echo "patch failed"; exit 1; }
timeout -k 10 600 python -c "from das_diff_veh_amd.build import build; print(build())" || { echo "build failed"; exit 1; }
bash tools/gpu_r2an.sh
