# GPU commands behind this profile set (round 2, third session, final code), one gpurun call: bash tools/gpu_final.sh
#   gpu_tests.log, smoke.log   <- pytest tests -m gpu; __graft_entry__.smoke()
#   kernel_stats.csv           <- tools/profile_round.sh r02g: rocprofv3 --kernel-trace --stats of
#                                 `python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline`
#   pmc.json                   <- python tools/pmc_latest.py gpurun_out/prof_r02g search_res_kernel
#                                 (three --pmc passes, each its own kernel-trace-only run)
#   bench.json                 <- `python3 bench.py` (defaults, with the CPU baseline leg)
#   conv_mz.json, conv_ez.json <- tools/conv_bench.py --kind mz|ez (split-bf16 trunk, default)
#   bench_philox.json, bench_zero_heads.json <- bench.py --rng philox / --zero-heads
bash tools/gpu_final.sh
# after the last trunk change (commit e74b1c8): bash tools/gpu_verify.sh
#   gpu_tests_final.log, smoke_final.log, bench_final.json (21.95 M sims/s)
