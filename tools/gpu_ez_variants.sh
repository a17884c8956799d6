# GPU: EZ one-launch — parity tests with the default library, then phase timing of build variants
# (diaglibs/*.so via LZM_LIB). usage: bash tools/gpu_ez_variants.sh <tag> <variant>...
set -e
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread \
  -k "fused_conv_search_equals_generic and ez or pools_equal or full_config_tree_parity and ez" > $out/tests.log 2>&1
timeout -k 10 150 python tools/conv_bench.py --kind ez > $out/conv_ez_fused.json 2>$out/conv_ez_fused.err
timeout -k 10 150 python tools/conv_phase_timing.py --kind ez > $out/phase.txt 2>&1
for v in "$@"; do
  LZM_LIB=$PWD/diaglibs/$v.so timeout -k 10 150 python tools/conv_phase_timing.py --kind ez --no-check > $out/phase_$v.txt 2>&1
done
