# Final build of round 4 (after LZM_RES_SEEDW1 and the removal of the off-by-default experiment paths; the closing set in the parent directory is the build
# before it — conv kernels unchanged since). Two gpurun calls:
#   gpu_tests.log, smoke.log, kernel_stats.csv <- bash tools/gpu_final_a.sh r04b (236 passed; smoke
#       bit-exact; rocprofv3 --kernel-trace --stats of bench.py --steps 20 --warmup 3 --no-cpu-baseline;
#       the first --pmc pass then printed nothing for 180 s on that box and the call was ended, so the
#       PMC summary stays the closing set's: ../pmc.json, same kernels' memory traffic)
#   bench.json, bench_zero_heads.json, bench_philox.json, bench_collect.json, phase_timing*.txt <-
python3 bench.py
python bench.py --no-cpu-baseline --secondary none --zero-heads
python bench.py --no-cpu-baseline --secondary none --rng philox
python bench.py --step collect --secondary none --no-cpu-baseline
python tools/phase_timing.py; python tools/phase_timing.py --zero-heads
# gpu_tests.log, smoke.log, bench_nobaseline.json re-run on the final code (after the cleanup):
#   bash tools/gpu.sh gpurun_out/f_r04d alltests smoke bench:--no-cpu-baseline,--secondary,none  (236 passed)
# Closing set on the final code (after the fused representation-network epilogue):
#   bash tools/gpu_final_a.sh r04e -> gpu_tests.log (236 passed), smoke.log, kernel_stats.csv, pmc.json
#   (three --pmc passes, tools/pmc_latest.py), bench.json (bench.py defaults: CPU baseline, config 5 object),
#   divergence_*.json
# Closing set on the final code (after the native 8x8 representation tail), two steps in one call:
#   bash tools/gpu_final_a.sh r04f -> gpu_tests.log (236 passed), smoke.log, kernel_stats.csv, pmc.json, bench.json
#   bash tools/gpu.sh gpurun_out/f_r04f bench:--workload,breakout,--no-cpu-baseline
#        bench:--workload,breakout,--no-cpu-baseline,--step,collect -> bench_breakout_search_step.json,
#        bench_breakout_collect_step.json
