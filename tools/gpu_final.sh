# GPU: the round's closing set into gpurun_out/f_<tag> — GPU tests, smoke, the profile set of the
# default bench command (kernel stats, PMC passes, the bench line with its CPU baseline and config 5's
# sharded collect step), the conv benches with their CPU baselines (Breakout MZ, Pong EZ) and kernel
# traces, the Philox / zero-heads / collect-mode / config-1 lines, the phase timings.
# usage: bash tools/gpu_final.sh <tag> [--no-tests]
set -e
tag=${1:-r04}
out=gpurun_out/f_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export LZM_REPORT_DIR="$GRAFT_REPO_ROOT/$out"
if [ "$2" != "--no-tests" ]; then  # (--no-tests: the second half after tools/gpu_final_a.sh)
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $out/gpu_tests.log 2>&1
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
  bash tools/profile_round.sh $out/prof
fi
for k in mz ez; do
  timeout -k 10 300 python tools/conv_bench.py --kind $k --cpu-baseline-secs 30 > $out/conv_$k.json 2>$out/conv_$k.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_conv_mz -o conv_mz --output-format csv -- \
  python3 tools/conv_bench.py --kind mz --searches 3 > $out/trace_conv_mz.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --secondary none --rng philox > $out/bench_philox.json 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --secondary none --zero-heads > $out/bench_zero_heads.json 2>&1
timeout -k 10 200 python bench.py --step collect --secondary none --no-cpu-baseline > $out/bench_collect.json 2>$out/bench_collect.err
timeout -k 10 300 python bench.py --workload breakout --cpu-baseline-secs 30 > $out/bench_breakout.json 2>$out/bench_breakout.err
# config 1 (8 envs x 25 sims): the GPU search at that shape and the pure-Python ptree restatement on
# this box's host (1 thread, MLP on torch-CPU)
timeout -k 10 120 python bench.py --envs 8 --sims 25 --no-cpu-baseline --secondary none > $out/bench_c1_gpu.json 2>$out/bench_c1_gpu.err
timeout -k 10 120 python tools/ptree_bench.py --secs 15 > $out/ptree_c1_cpu.json 2>$out/ptree_c1_cpu.err
timeout -k 10 150 python tools/phase_timing.py > $out/phase_timing.txt 2>&1
timeout -k 10 150 python tools/phase_timing.py --zero-heads > $out/phase_timing_zero_heads.txt 2>&1
timeout -k 10 150 python tools/conv_phase_timing.py --kind ez > $out/conv_phase_ez.txt 2>&1
timeout -k 10 150 python tools/conv_phase_timing.py --kind mz > $out/conv_phase_mz.txt 2>&1
# last: under rocprofv3 the Pong process (cooperative launches) segfaults in the tool's teardown after
# the trace files are written (round 4; the unprofiled run exits cleanly), and nothing may follow a
# segfault in the same call
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_conv_ez -o conv_ez --output-format csv -- \
  python3 tools/conv_bench.py --kind ez --searches 3 > $out/trace_conv_ez.log 2>&1
