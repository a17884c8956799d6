# GPU: PMC passes over the EfficientZero one-launch search (conv_bench --kind ez; kernel-trace only,
# one counter set per run). usage: bash tools/gpu_ez_pmc.sh <tag>
set -e
out=gpurun_out/${1:-ezp}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for set in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "WRITE_SIZE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d $out/pmc_$i -o pmc --output-format csv -- \
    python3 tools/conv_bench.py --kind ez --searches 2 --warmup 1 > $out/pmc_$i.log 2>&1
done
