# GPU: one iteration on search_res_kernel — fused/tree tests, bench (random, zero heads, Philox), phase timing, SQ pass
set -e
out=gpurun_out/${1:-ri}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_fused.py tests/test_gpu_search.py tests/test_gpu_reanalyze.py tests/test_gpu_collect.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench.json 2>$out/bench.err
timeout -k 10 300 python bench.py --zero-heads --no-cpu-baseline > $out/bench_zero_heads.json 2>$out/bench_zero_heads.err
timeout -k 10 300 python bench.py --rng philox --no-cpu-baseline > $out/bench_philox.json 2>$out/bench_philox.err
timeout -k 10 150 python tools/phase_timing.py > $out/phase.txt 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS -d $out/pmc -o pmc --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $out/pmc.log 2>&1
