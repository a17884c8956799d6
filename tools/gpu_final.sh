# GPU: the round's closing set — GPU tests, smoke, the profile set of the headline bench (kernel stats,
# PMC passes, bench line), the conv benches
set -e
mkdir -p gpurun_out/f
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/f/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f/smoke.log 2>&1
bash tools/profile_round.sh r02g
for k in mz ez; do
  timeout -k 10 150 python tools/conv_bench.py --kind $k > gpurun_out/f/conv_$k.json 2>gpurun_out/f/conv_$k.err
done
timeout -k 10 120 python bench.py --no-cpu-baseline --rng philox > gpurun_out/f/bench_philox.json 2>&1
timeout -k 10 120 python bench.py --no-cpu-baseline --zero-heads > gpurun_out/f/bench_zero_heads.json 2>&1
