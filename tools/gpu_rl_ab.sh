# GPU: the conv walks with readlane child records (variant R) against HEAD (A): Breakout and Pong conv-bench
# A/Bs, Breakout phase cycles of R, then the conv tests on R
set -e
out=${1:-gpurun_out/rl_ab}
mkdir -p $out
bash tools/ab_conv_bench.sh $out/mz mz A R
bash tools/ab_conv_bench.sh $out/ez ez A R
LZM_LIB=lightzero_amd/liblzm_varR.so timeout -k 10 120 python tools/conv_phase_timing.py --kind mz > $out/phase_mz_R.txt 2>&1
LZM_LIB=lightzero_amd/liblzm_varR.so timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_config5.py tests/test_gpu_config3.py tests/test_gpu_split_range.py -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1
