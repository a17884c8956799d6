# GPU: the LDS-resident head half (LZM_CONV_PIN) on Breakout: conv-bench A/B off/on, phase cycles, conv tests
set -e
out=${1:-gpurun_out/pin_ab}
export LZM_LIB=${LZM_LIB:-lightzero_amd/liblzm_varP.so}
mkdir -p $out
bash tools/ab_env_conv.sh $out/ab1 mz LZM_CONV_PIN
bash tools/ab_env_conv.sh $out/ab2 mz LZM_CONV_PIN
LZM_CONV_PIN=0 timeout -k 10 120 python tools/conv_phase_timing.py --kind mz > $out/phase_pin0.txt 2>&1
LZM_CONV_PIN=1 timeout -k 10 120 python tools/conv_phase_timing.py --kind mz > $out/phase_pin1.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_config5.py tests/test_gpu_split_range.py -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1
