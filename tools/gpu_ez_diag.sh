# GPU: EZ one-launch phase timing of diagnostic library builds only (diaglibs/*.so via LZM_LIB;
# results invalid, cycles valid). usage: bash tools/gpu_ez_diag.sh <tag> <variant>...
set -e
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  LZM_LIB=$PWD/diaglibs/$v.so timeout -k 10 150 python tools/conv_phase_timing.py --kind ez --no-check > $out/phase_$v.txt 2>&1
done
