mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -v --timeout 120 --timeout-method thread -k "trunk" > gpurun_out/conv_tests.log 2>&1 \
&& timeout -k 10 150 python tools/conv_bench.py --kind mz --precision bf16x3 > gpurun_out/conv_mz_bx.json 2>&1 \
&& timeout -k 10 150 python tools/conv_bench.py --kind mz --precision f32 > gpurun_out/conv_mz_f32.json 2>&1 \
&& timeout -k 10 150 python tools/conv_bench.py --kind ez --precision bf16x3 > gpurun_out/conv_ez_bx.json 2>&1 \
&& timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
&& timeout -k 10 120 python bench.py > gpurun_out/bench.json 2>gpurun_out/bench.err
