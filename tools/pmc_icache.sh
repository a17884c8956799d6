# GPU: instruction-cache counters of the one-launch searches (one --pmc pass per workload, kernel-trace only).
# usage: bash tools/pmc_icache.sh OUT_DIR
set -e
out=${1:-gpurun_out/icache}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
set_="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set_ -d $out/res -o pmc --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --configs none --secondary none > $out/res.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set_ -d $out/conv -o pmc --output-format csv -- \
  python3 bench.py --workload breakout --steps 5 --warmup 2 --no-cpu-baseline --configs none > $out/conv.log 2>&1
