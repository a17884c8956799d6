# GPU: the initial-inference / fused / collector tests on the in-tree build, the headline A/B (variants A, B) and
# the initial-inference kernel's time in a headline trace
set -e
out=${1:-gpurun_out/ii_check}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_collect.py tests/test_gpu_collector.py tests/test_gpu_muzero_collector.py tests/test_gpu_divergence.py tests/test_gpu_policy_modes.py -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1
bash tools/ab_libs.sh $out/ab A B A B
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o hl --output-format csv -- \
  python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --configs none --secondary none > $out/trace.log 2>&1
