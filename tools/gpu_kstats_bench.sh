# GPU: collect-step tests, then kernel stats of the default bench command and the bench line
set -e
mkdir -p gpurun_out/k
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_collect.py tests/test_gpu_fused.py tests/test_initial.py -x -q --timeout 120 --timeout-method thread > gpurun_out/k/tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/k/trace -o fused --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/k/bench_traced.log 2>&1
timeout -k 10 150 python bench.py --no-cpu-baseline > gpurun_out/k/bench.json 2>&1
