# GPU: SQ counters of the fused LSTM kernel (two --pmc passes, each a kernel-trace-only run)
set -e
out=gpurun_out/${1:-lsp}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set -d $out/pmc_$i -o pmc --output-format csv -- \
    python3 tools/lstm_bench.py --iters 40 > $out/pmc_$i.log 2>&1
done
