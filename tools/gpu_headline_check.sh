# GPU: the -m gpu suite, then the headline bench line (no CPU baselines, no secondary configs) and its phase cycles
set -e
out=${1:-gpurun_out/headline_check}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/gpu_tests.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --configs none --secondary none > $out/bench.json 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --configs none --secondary none --zero-heads > $out/bench_zero_heads.json 2>&1
timeout -k 10 150 python tools/phase_timing.py > $out/phase_timing.txt 2>&1
