# GPU commands behind this profile set (round 2, second session; commit e21b067), one gpurun call:
#   kernel_stats.csv  <- tools/profile_round.sh r02e: rocprofv3 --kernel-trace --stats of
#                        `python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline`
#   pmc.json          <- python tools/pmc_latest.py gpurun_out/prof_r02e search_res_kernel
#                        (three --pmc passes of tools/profile_round.sh: FETCH_SIZE | WRITE_SIZE |
#                        TCC_HIT_sum TCC_MISS_sum, each its own kernel-trace-only run)
#   bench.json        <- tools/profile_round.sh's last step: `python3 bench.py` (defaults, with the
#                        CPU baseline leg)
bash tools/profile_round.sh r02e
LZM_PHASE_TIMING=1 timeout -k 10 200 python tools/phase_timing.py > phase_timing.txt
LZM_PHASE_TIMING=1 timeout -k 10 200 python tools/phase_timing.py --zero-heads > phase_timing_zero_heads.txt
timeout -k 10 120 python bench.py --no-cpu-baseline --rng philox > bench_philox.json
timeout -k 10 120 python bench.py --no-cpu-baseline --zero-heads > bench_zero_heads.json
