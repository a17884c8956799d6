# GPU: per-phase cycles of the one-launch conv searches (Breakout MuZero, Pong EfficientZero)
set -e
out=${1:-gpurun_out/conv_phase}
mkdir -p $out
timeout -k 10 150 python tools/conv_phase_timing.py --kind mz > $out/conv_phase_mz.txt 2>&1
timeout -k 10 150 python tools/conv_phase_timing.py --kind ez > $out/conv_phase_ez.txt 2>&1
timeout -k 10 200 python tools/conv_bench.py --kind ez --searches 10 > $out/conv_bench_ez.txt 2>&1
timeout -k 10 200 python tools/conv_bench.py --kind mz --searches 10 > $out/conv_bench_mz.txt 2>&1
