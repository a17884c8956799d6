# GPU: the AlphaZero tests, then the phase cycles and the bench object of the fused AlphaZero search
set -e
out=${1:-gpurun_out/az_check}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_alphazero.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 120 python tools/az_phase_timing.py > $out/phase.txt 2>&1
LZM_AZ_BOARDS_PER_WG=2 timeout -k 10 120 python tools/az_phase_timing.py > $out/phase_r2.txt 2>&1
timeout -k 10 300 python tools/az_bench.py --no-reference > $out/az_bench.json 2>&1
