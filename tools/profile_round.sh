# GPU: the round's profile set of the default bench command (usage: bash tools/profile_round.sh OUT_DIR)
#   kernel trace + stats of `bench.py` (the headline config-2 search and config 5's Breakout collect
#   step), PMC passes (each counter group in its own pass, kernel-trace only: FETCH_SIZE, WRITE_SIZE,
#   TCC hit/miss), and the full bench line with the CPU baseline.
set -e
out=${1:-gpurun_out/prof}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o fused --output-format csv -- \
  python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $out/bench_traced.log 2>&1
python3 tools/kstats_grid.py $out/trace/fused_kernel_trace.csv > $out/trace/kernel_stats_by_grid.csv
# the headline alone (its kernel's stats not merged with config 1's launches of the same kernel)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_headline -o headline --output-format csv -- \
  python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --configs none --secondary none > $out/bench_headline_traced.log 2>&1
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set -d $out/pmc_$i -o pmc --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $out/pmc_$i.log 2>&1
done
timeout -k 10 300 python3 bench.py > $out/bench.json 2>&1
