# GPU: conv-trunk iteration loop — native-trunk parity test, the MZ/EZ conv benches, MZ kernel stats
set -e
mkdir -p gpurun_out/cq
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -k "native or parity" > gpurun_out/cq/tests.log 2>&1
timeout -k 10 200 python tools/conv_bench.py --kind mz > gpurun_out/cq/mz.json
timeout -k 10 200 python tools/conv_bench.py --kind ez > gpurun_out/cq/ez.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cq/prof -o mz --output-format csv -- python3 tools/conv_bench.py --kind mz --searches 3 > gpurun_out/cq/prof.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cq/prof -o ez --output-format csv -- python3 tools/conv_bench.py --kind ez --searches 3 > gpurun_out/cq/prof_ez.log 2>&1
