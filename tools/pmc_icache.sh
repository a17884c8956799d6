# GPU: instruction-cache and wait counters of the fused bench kernel (separate --pmc passes,
# kernel-trace only). Writes gpurun_out/pmc_ic_*/ and prints per-kernel sums.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for set in "SQC_ICACHE_MISSES SQC_ICACHE_HITS" "SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/pmc_ic_$i -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_ic_$i.log 2>&1
done
