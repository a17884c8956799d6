# GPU: Breakout one-launch A/B + collect-line repeat. usage: bash tools/gpu_mz_ab.sh <tag> <variant>
set -e
tag=$1; v=$2
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread \
  -k "fused_conv_search_equals_generic and mz or full_config_tree_parity and mz" > $out/tests.log 2>&1
for lib in default $v; do
  L=""; [ "$lib" != default ] && L=$PWD/diaglibs/$lib.so
  for rep in 1 2; do
    LZM_LIB=$L timeout -k 10 150 python tools/conv_bench.py --kind mz > $out/conv_mz_${lib}_$rep.json 2>/dev/null
    LZM_LIB=$L timeout -k 10 200 python bench.py --step collect --no-cpu-baseline > $out/collect_${lib}_$rep.json 2>/dev/null
  done
done
