# GPU commands behind this profile set (round 3, closing run, after the pipelined Breakout heads), one gpurun call:
#   bash tools/gpu_final.sh r03d
#     gpu_tests.log, smoke.log          <- pytest tests -m gpu (214 passed); __graft_entry__.smoke()
#     kernel_stats.csv, pmc.json, bench.json <- tools/profile_round.sh r03d (rocprofv3 --kernel-trace --stats
#                                          of bench.py --steps 20 --warmup 3 --no-cpu-baseline; three --pmc
#                                          passes; bench.py defaults incl. the CPU-baseline variants);
#                                          pmc.json = python tools/pmc_latest.py gpurun_out/prof_r03d search_res_kernel
#     conv_mz.json, conv_ez.json        <- tools/conv_bench.py --kind mz|ez (one launch per search each)
#     conv_mz_kernel_stats.csv, conv_ez_kernel_stats.csv <- rocprofv3 --kernel-trace --stats of
#                                          tools/conv_bench.py --kind mz|ez --searches 3
#     conv_phase_ez.txt, conv_phase_mz.txt <- tools/conv_phase_timing.py --kind ez|mz (stamped builds)
#     bench_philox.json, bench_zero_heads.json, bench_collect.json <- bench.py --rng philox / --zero-heads /
#                                          --step collect
#     bench_c1_gpu.json, ptree_c1_cpu.json <- config 1 (8 envs x 25 sims): bench.py --envs 8 --sims 25;
#                                          tools/ptree_bench.py (ptree restatement, 1 host thread)
bash tools/gpu_final.sh r03d
