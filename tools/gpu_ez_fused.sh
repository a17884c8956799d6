# GPU: the EfficientZero one-launch search (lzm_search_conv_ez) — parity tests, then the Pong bench
# (one launch vs the generic path) and a kernel trace. usage: bash tools/gpu_ez_fused.sh <tag>
set -e
tag=${1:-ez1}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -v --timeout 120 --timeout-method thread \
  -k "fused_conv_search_equals_generic and ez or pools_equal or full_config_tree_parity" > $out/tests.log 2>&1
timeout -k 10 150 python tools/conv_bench.py --kind ez > $out/conv_ez_fused.json 2>$out/conv_ez_fused.err
timeout -k 10 150 python tools/conv_bench.py --kind ez --rng philox > $out/conv_ez_fused_philox.json 2>$out/conv_ez_fused_philox.err
timeout -k 10 150 python tools/conv_bench.py --kind ez --fused 0 > $out/conv_ez_generic.json 2>$out/conv_ez_generic.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o ez --output-format csv -- \
  python3 tools/conv_bench.py --kind ez --searches 3 > $out/trace.log 2>&1
