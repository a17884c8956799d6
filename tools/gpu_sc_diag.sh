# GPU: conv one-launch search phase timing with the trunk / head weight loads removed (diagnostic
# builds via LZM_LIB; results invalid, cycles valid)
set -e
out=gpurun_out/${1:-scd}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 150 python tools/conv_phase_timing.py --rng philox > $out/base_philox.txt 2>&1
LZM_LIB=lightzero_amd/liblzm_diagw.so timeout -k 10 150 python tools/conv_phase_timing.py --rng philox --no-check > $out/diagw_philox.txt 2>&1
LZM_LIB=lightzero_amd/liblzm_diagh.so timeout -k 10 150 python tools/conv_phase_timing.py --rng philox --no-check > $out/diagh_philox.txt 2>&1
