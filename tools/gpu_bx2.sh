# GPU: split trunk iteration — conv tests, kernel stats (Breakout MZ), conv benches
set -e
mkdir -p gpurun_out/b2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -v --timeout 120 --timeout-method thread > gpurun_out/b2/tests.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/b2/prof -o mz --output-format csv -- python3 tools/conv_bench.py --searches 3 --kind mz > gpurun_out/b2/prof_mz.log 2>&1
for k in mz ez; do
  timeout -k 10 150 python tools/conv_bench.py --kind $k > gpurun_out/b2/conv_$k.json 2>gpurun_out/b2/conv_$k.err
done
