set -e
mkdir -p gpurun_out/cq
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_search.py -x -q --timeout 120 --timeout-method thread > gpurun_out/cq/tests.log 2>&1
for f in 1 0; do
timeout -k 10 200 env LZM_FUSE=$f python tools/conv_bench.py --kind mz > gpurun_out/cq/mz_$f.json
timeout -k 10 200 env LZM_FUSE=$f python tools/conv_bench.py --kind ez > gpurun_out/cq/ez_$f.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cq/prof -o mz --output-format csv -- python3 tools/conv_bench.py --kind mz --searches 3 > gpurun_out/cq/prof.log 2>&1
