# GPU: verification of the committed library — GPU tests, smoke, default bench line
set -e
mkdir -p gpurun_out/v
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v/smoke.log 2>&1
timeout -k 10 150 python bench.py > gpurun_out/v/bench.json 2>gpurun_out/v/bench.err
