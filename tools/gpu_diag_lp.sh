set -e
mkdir -p gpurun_out/ezd
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for d in 1 2 3 4; do
  LZM_LIB=$PWD/diaglibs/lp$d.so timeout -k 10 150 python tools/conv_phase_timing.py --kind ez --no-check > gpurun_out/ezd/phase_lp$d.txt 2>&1
done
