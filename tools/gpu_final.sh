# GPU: the round's closing set — GPU tests, smoke, the profile set of the headline bench (kernel stats,
# PMC passes, bench line with the CPU baseline), the conv benches (Breakout one launch: kernel trace),
# Philox / zero-heads lines, the collect-mode line. usage: bash tools/gpu_final.sh <tag>
set -e
tag=${1:-r03}
out=gpurun_out/f_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
bash tools/profile_round.sh $tag
for k in mz ez; do
  timeout -k 10 150 python tools/conv_bench.py --kind $k > $out/conv_$k.json 2>$out/conv_$k.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_conv_mz -o conv_mz --output-format csv -- \
  python3 tools/conv_bench.py --kind mz --searches 3 > $out/trace_conv_mz.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_conv_ez -o conv_ez --output-format csv -- \
  python3 tools/conv_bench.py --kind ez --searches 3 > $out/trace_conv_ez.log 2>&1
timeout -k 10 120 python bench.py --no-cpu-baseline --rng philox > $out/bench_philox.json 2>&1
timeout -k 10 120 python bench.py --no-cpu-baseline --zero-heads > $out/bench_zero_heads.json 2>&1
timeout -k 10 200 python bench.py --step collect --no-cpu-baseline > $out/bench_collect.json 2>$out/bench_collect.err
# config 1 (8 envs x 25 sims): the GPU search at that shape and the pure-Python ptree restatement on
# this box's host (1 thread, MLP on torch-CPU)
timeout -k 10 120 python bench.py --envs 8 --sims 25 --no-cpu-baseline > $out/bench_c1_gpu.json 2>$out/bench_c1_gpu.err
timeout -k 10 120 python tools/ptree_bench.py --secs 15 > $out/ptree_c1_cpu.json 2>$out/ptree_c1_cpu.err
# EfficientZero one-launch: phase timing; MuZero conv phase timing
timeout -k 10 150 python tools/conv_phase_timing.py --kind ez > $out/conv_phase_ez.txt 2>&1
timeout -k 10 150 python tools/conv_phase_timing.py --kind mz > $out/conv_phase_mz.txt 2>&1
