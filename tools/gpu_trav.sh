# GPU: GPU test suite; look-back traverse phase timing (stamped instantiation) at Breakout MZ and Pong EZ;
# conv search kernel stats and benches
set -e
mkdir -p gpurun_out/t
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t/gpu_tests.log 2>&1
(export LZM_PHASE_TIMING=1; timeout -k 10 200 python tools/trav_timing.py --kind mz > gpurun_out/t/trav_mz.txt 2>&1)
(export LZM_PHASE_TIMING=1; timeout -k 10 200 python tools/trav_timing.py --kind ez > gpurun_out/t/trav_ez.txt 2>&1)
for k in mz ez; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/t/prof -o $k --output-format csv -- python3 tools/conv_bench.py --searches 3 --kind $k > gpurun_out/t/prof_$k.log 2>&1
  timeout -k 10 150 python tools/conv_bench.py --kind $k > gpurun_out/t/conv_$k.json 2>gpurun_out/t/conv_$k.err
done
