# GPU: EZ one-launch A/B of build variants (diaglibs/<v>.so): Pong bench twice + phase timing each.
# usage: bash tools/gpu_ez_ab.sh <tag> <variant>...
set -e
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in default "$@"; do
  L=""; [ "$v" != default ] && L=$PWD/diaglibs/$v.so
  for rep in 1 2; do
    LZM_LIB=$L timeout -k 10 150 python tools/conv_bench.py --kind ez > $out/conv_ez_${v}_$rep.json 2>/dev/null
  done
  LZM_LIB=$L timeout -k 10 150 python tools/conv_phase_timing.py --kind ez > $out/phase_$v.txt 2>&1
done
