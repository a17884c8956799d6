set -e
mkdir -p gpurun_out/conv
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -v --timeout 120 --timeout-method thread > gpurun_out/conv/tests.log 2>&1
for k in ez mz; do
  timeout -k 10 200 python tools/conv_bench.py --kind $k --graph 1 > gpurun_out/conv/bench_${k}_graph.json 2>gpurun_out/conv/bench_${k}.err
  timeout -k 10 200 python tools/conv_bench.py --kind $k --graph 0 --searches 3 > gpurun_out/conv/bench_${k}_eager.json 2>>gpurun_out/conv/bench_${k}.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/conv/prof_mz -o mz --output-format csv -- python3 tools/conv_bench.py --kind mz --graph 1 --searches 3 > gpurun_out/conv/prof_mz.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/conv/prof_ez -o ez --output-format csv -- python3 tools/conv_bench.py --kind ez --graph 1 --searches 3 > gpurun_out/conv/prof_ez.log 2>&1
