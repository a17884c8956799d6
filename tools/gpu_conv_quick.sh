# GPU: conv one-launch search — tests, phase timing (glibc, philox), bench
set -e
out=gpurun_out/${1:-cq}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > $out/conv_tests.log 2>&1
timeout -k 10 150 python tools/conv_phase_timing.py > $out/phase_glibc.txt 2>&1
timeout -k 10 150 python tools/conv_phase_timing.py --rng philox > $out/phase_philox.txt 2>&1
timeout -k 10 150 python tools/conv_bench.py --kind mz --fused 1 > $out/conv_mz_fused.json 2>$out/conv_mz_fused.err
