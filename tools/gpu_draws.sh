# GPU: lane-parallel draws — tree/fused/conv tests, zero-heads phase timing, bench lines
set -e
out=gpurun_out/${1:-dr}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_fused.py tests/test_gpu_conv.py tests/test_gpu_search.py tests/test_gpu_reanalyze.py tests/test_gpu_reuse.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 150 python tools/phase_timing.py --zero-heads > $out/phase_zero_heads.txt 2>&1
timeout -k 10 300 python bench.py --zero-heads --no-cpu-baseline > $out/bench_zero_heads.json 2>$out/bench_zero_heads.err
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench.json 2>$out/bench.err
timeout -k 10 150 python tools/conv_phase_timing.py > $out/conv_phase_glibc.txt 2>&1
timeout -k 10 150 python tools/conv_bench.py --kind mz --fused 1 > $out/conv_mz_fused.json 2>$out/conv_mz_fused.err
