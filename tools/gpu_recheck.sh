# GPU: the -m gpu suite, smoke() and the default bench line on the tree as it stands (a re-check after a rebuild)
set -e
out=${1:-gpurun_out/recheck}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $out/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 300 python bench.py > $out/bench.json 2>&1
