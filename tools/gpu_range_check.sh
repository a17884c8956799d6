# GPU: the conv / split-range / config 3 and 5 tests on the in-tree build, then Breakout and Pong A/Bs (variants A, B)
set -e
out=${1:-gpurun_out/range_check}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_split_range.py tests/test_gpu_config5.py tests/test_gpu_config3.py -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1
bash tools/ab_conv_bench.sh $out/ab_mz mz A B
bash tools/ab_conv_bench.sh $out/ab_ez ez A B
