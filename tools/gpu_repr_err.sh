# GPU: the DownSample parity tests with the achieved error printed, for this build and liblzm_varB.so (the
# three-term bf16 build), then the config 3 / 5 GPU tests
set -e
mkdir -p gpurun_out/r05af
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_config5.py -k "downsample" > gpurun_out/r05af/fp16.log 2>&1
LZM_LIB=lightzero_amd/liblzm_varB.so timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_config5.py -k "downsample" > gpurun_out/r05af/bf16x3.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_config5.py tests/test_gpu_config3.py > gpurun_out/r05af/cfg.log 2>&1
