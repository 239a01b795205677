# PMC passes for the bench's dominant kernel (one counter group per pass, kernel trace only).
# Writes gpurun_out/pmc_<tag>/... and the summary profiles/<tag>_pmc_summary.json.
set -o pipefail
tag=${1:-r1}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_$tag
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d gpurun_out/pmc_$tag/p$i -o pmc --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/pmc_$tag/p$i.err || { echo "pmc pass $i failed"; exit 1; }
done
python tools/pmc_summary.py gpurun_out/pmc_$tag profiles/${tag}_pmc_summary.json
