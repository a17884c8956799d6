# GPU: quick check of the current tree — GPU tests, smoke, the default bench line (CPU-baseline
# variants included) and the collect-mode line (usage: bash tools/gpu_check.sh <tag>)
set -e
tag=${1:-chk}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 300 python bench.py > $out/bench.json 2>$out/bench.err
timeout -k 10 200 python bench.py --step collect --no-cpu-baseline > $out/bench_collect.json 2>$out/bench_collect.err
