# GPU: fused-kernel duration under each LZM_DIAG_MODE (timing experiments; results are invalid)
set -e
for m in 0 1 2 4 5 6; do
  LZM_DIAG_MODE=$m timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/diag_$m.log 2>&1 || true
done
