# GPU: phase cycles of the fused AlphaZero search at 1, 2 and 4 boards per workgroup, then the AZ tests
set -e
out=${1:-gpurun_out/az_phase}
mkdir -p $out
timeout -k 10 120 python tools/az_phase_timing.py > $out/phase_r2.txt 2>&1
LZM_AZ_BOARDS_PER_WG=1 timeout -k 10 120 python tools/az_phase_timing.py > $out/phase_r1.txt 2>&1
LZM_AZ_BOARDS_PER_WG=4 timeout -k 10 120 python tools/az_phase_timing.py > $out/phase_r4.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_alphazero.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
