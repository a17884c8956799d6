# GPU: headline kernel A/B — GPU tests with the default library, then bench lines (glibc, zero heads)
# and phase timing for the default library and each diaglibs/<variant>.so. usage:
#   bash tools/gpu_res_ab.sh <tag> <variant>...
set -e
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1
for v in default "$@"; do
  lib=""; [ "$v" != default ] && lib=$PWD/diaglibs/$v.so
  for rep in 1 2; do
    LZM_LIB=$lib timeout -k 10 150 python bench.py --no-cpu-baseline > $out/bench_${v}_$rep.json 2>/dev/null
  done
  LZM_LIB=$lib timeout -k 10 150 python bench.py --no-cpu-baseline --zero-heads > $out/bench_${v}_zero.json 2>/dev/null
  LZM_LIB=$lib LZM_PHASE_TIMING=1 timeout -k 10 150 python tools/phase_timing.py > $out/phase_$v.txt 2>&1
done
