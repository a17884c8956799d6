# GPU: fused EZ LSTM gate GEMM + cell — conv tests, Pong bench (fused vs rocBLAS), kernel trace
set -e
out=gpurun_out/${1:-ls}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > $out/conv_tests.log 2>&1
timeout -k 10 200 python tools/conv_bench.py --kind ez > $out/conv_ez.json 2>$out/conv_ez.err
LZM_LSTM_FUSED=0 timeout -k 10 200 python tools/conv_bench.py --kind ez > $out/conv_ez_rocblas.json 2>$out/conv_ez_rocblas.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_ez -o ez -- python tools/conv_bench.py --kind ez --searches 3 > $out/prof_ez.log 2>&1
