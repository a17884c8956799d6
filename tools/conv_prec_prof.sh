# GPU: split-bf16 conv trunk iteration — parity tests, then kernel stats (rocprofv3 --kernel-trace --stats)
# of the Breakout MZ search per trunk variant: f32, bf16x3 at weight read-ahead 3 / 5 / 8 chunks, and
# the no-weight-load ablation (LZM_CONV_DIAG=1, results invalid, duration only)
set -e
mkdir -p gpurun_out/cp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -v --timeout 120 --timeout-method thread -k "trunk" > gpurun_out/cp/tests.log 2>&1
prof() {  # name, env..., then conv_bench args
  local n=$1; shift
  (export "$@"; timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/cp/prof -o $n --output-format csv -- python3 tools/conv_bench.py --searches 3 --kind mz > gpurun_out/cp/$n.log 2>&1)
}
prof mz_warm LZM_CONV_PRECISION=f32
prof mz_f32 LZM_CONV_PRECISION=f32
prof mz_bx3 LZM_CONV_PRECISION=bf16x3 LZM_CONV_AHEAD=3
prof mz_bx5 LZM_CONV_PRECISION=bf16x3 LZM_CONV_AHEAD=5
prof mz_bx8 LZM_CONV_PRECISION=bf16x3 LZM_CONV_AHEAD=8
prof mz_bxnow LZM_CONV_PRECISION=bf16x3 LZM_CONV_DIAG=1
