# GPU: fused parity tests, then per-R phase timing and bench (usage: bash tools/rsweep.sh "1 8")
set -e
timeout -k 10 400 python -m pytest tests/test_gpu_fused.py -x -q > gpurun_out/t.log 2>&1
for R in ${1:-1 2 4 8}; do
  timeout -k 10 200 python tools/phase_timing.py --roots $R > gpurun_out/phase_r$R.log 2>&1
  LZM_ROOTS_PER_WG=$R timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_r$R.log 2>&1
done
