# GPU: round 6's closing set into gpurun_out/final_r06 (copied to profiles/r06/final afterwards).
#   part a: the -m gpu suite, smoke(), tools/profile_round.sh (kernel stats of the default bench command,
#           PMC passes, the full bench line: headline + configs 1, 3, 4, 5 with their CPU baselines)
#   part b: the Breakout collect-step trace, Philox / zero-heads lines, phase timings, the Pong EZ trace
#           (must end with the tool's finalisation: the round-4 exit-time fault)
# usage: bash tools/gpu_final_r06.sh a|b
set -e
out=gpurun_out/final_r06
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export LZM_REPORT_DIR="$GRAFT_REPO_ROOT/$out"
if [ "$1" = "a" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $out/gpu_tests.log 2>&1
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
  bash tools/profile_round.sh $out/prof
else
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_breakout -o breakout --output-format csv -- \
    python3 bench.py --workload breakout --step collect --steps 30 --warmup 3 --no-cpu-baseline --configs none \
    > $out/trace_breakout.log 2>&1
  timeout -k 10 200 python bench.py --no-cpu-baseline --configs none --secondary none --rng philox > $out/bench_philox.json 2>&1
  timeout -k 10 200 python bench.py --no-cpu-baseline --configs none --secondary none --zero-heads > $out/bench_zero_heads.json 2>&1
  timeout -k 10 150 python tools/phase_timing.py > $out/phase_timing.txt 2>&1
  timeout -k 10 150 python tools/phase_timing.py --zero-heads > $out/phase_timing_zero_heads.txt 2>&1
  timeout -k 10 150 python tools/conv_phase_timing.py --kind mz > $out/conv_phase_mz.txt 2>&1
  timeout -k 10 150 python tools/conv_phase_timing.py --kind ez > $out/conv_phase_ez.txt 2>&1
  timeout -k 10 120 python tools/az_phase_timing.py > $out/az_phase.txt 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_conv_ez -o conv_ez --output-format csv -- \
    python3 tools/conv_bench.py --kind ez --searches 3 > $out/trace_conv_ez.log 2>&1
fi
