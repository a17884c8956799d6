# GPU: GPU test suite, then the conv search kernel stats and benches (Breakout MZ, Pong EZ)
set -e
mkdir -p gpurun_out/t
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t/gpu_tests.log 2>&1
for k in ez mz; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/t/prof -o $k --output-format csv -- python3 tools/conv_bench.py --searches 3 --kind $k > gpurun_out/t/prof_$k.log 2>&1
  timeout -k 10 150 python tools/conv_bench.py --kind $k > gpurun_out/t/conv_$k.json 2>gpurun_out/t/conv_$k.err
done
# SQ counters of the conv trunk (each pass its own kernel-trace-only run)
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/t/pmc_$i -o run --output-format csv -- python3 tools/conv_bench.py --searches 1 --warmup 1 --kind mz > gpurun_out/t/pmc_$i.log 2>&1
done
