# GPU: full GPU test suite, then the conv benches (both configs, default split-bf16 trunk) and the headline bench
set -e
mkdir -p gpurun_out/s
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s/gpu_tests.log 2>&1
for k in mz ez; do
  timeout -k 10 150 python tools/conv_bench.py --kind $k > gpurun_out/s/conv_$k.json 2>gpurun_out/s/conv_$k.err
done
timeout -k 10 150 python tools/conv_bench.py --kind mz --precision f32 > gpurun_out/s/conv_mz_f32.json 2>>gpurun_out/s/conv_mz.err
timeout -k 10 150 python tools/conv_bench.py --kind ez --precision f32 > gpurun_out/s/conv_ez_f32.json 2>>gpurun_out/s/conv_ez.err
timeout -k 10 150 python bench.py > gpurun_out/s/bench.json 2>gpurun_out/s/bench.err
