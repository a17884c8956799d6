# GPU: the conv / config 5 / config 3 tests on the in-tree build, then the Breakout conv-bench A/B (variants A, B)
set -e
out=${1:-gpurun_out/conv_ab}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_config5.py tests/test_gpu_split_range.py tests/test_gpu_muzero_collector.py -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1
bash tools/ab_conv_bench.sh $out/ab_mz mz A B
