# GPU: the conv walks dividing instead of reading the pb_c table (Q) against HEAD (N): Breakout / Pong conv-bench
# A/Bs, Breakout phase cycles of Q, the conv tests on Q
set -e
out=${1:-gpurun_out/pbt_ab}
mkdir -p $out
bash tools/ab_conv_bench.sh $out/mz mz N Q
bash tools/ab_conv_bench.sh $out/ez ez N Q
LZM_LIB=lightzero_amd/liblzm_varQ.so timeout -k 10 120 python tools/conv_phase_timing.py --kind mz > $out/phase_mz_Q.txt 2>&1
LZM_LIB=lightzero_amd/liblzm_varQ.so timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_config5.py tests/test_gpu_config3.py tests/test_gpu_split_range.py -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1
