# GPU: the LDS-resident value-head half (LZM_CONV_PIN) on Pong EZ: conv-bench A/B off/on, phase cycles, EZ tests
set -e
out=${1:-gpurun_out/pin_ez}
export LZM_LIB=${LZM_LIB:-lightzero_amd/liblzm_varP.so}
mkdir -p $out
bash tools/ab_env_conv.sh $out/ab1 ez LZM_CONV_PIN
bash tools/ab_env_conv.sh $out/ab2 ez LZM_CONV_PIN
LZM_CONV_PIN=0 timeout -k 10 120 python tools/conv_phase_timing.py --kind ez > $out/phase_pin0.txt 2>&1
LZM_CONV_PIN=1 timeout -k 10 120 python tools/conv_phase_timing.py --kind ez > $out/phase_pin1.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_config3.py tests/test_gpu_split_range.py -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1
