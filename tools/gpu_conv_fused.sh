# GPU: the one-launch conv search (lzm_search_conv) — conv tests, then fused vs generic Breakout benches
set -e
out=gpurun_out/${1:-cf}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -v --timeout 120 --timeout-method thread > $out/conv_tests.log 2>&1
timeout -k 10 150 python tools/conv_bench.py --kind mz --fused 1 > $out/conv_mz_fused.json 2>$out/conv_mz_fused.err
timeout -k 10 150 python tools/conv_bench.py --kind mz --fused 0 > $out/conv_mz_generic.json 2>$out/conv_mz_generic.err
timeout -k 10 150 python tools/conv_bench.py --kind mz --fused 1 --rng philox > $out/conv_mz_fused_philox.json 2>$out/conv_mz_fused_philox.err
