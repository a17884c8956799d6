# GPU commands behind this profile set (round 4, closing run), two gpurun calls:
#   bash tools/gpu_final_a.sh r04
#     gpu_tests.log, smoke.log          <- pytest tests -m gpu (236 passed); __graft_entry__.smoke()
#     kernel_stats.csv, pmc.json, bench.json <- tools/profile_round.sh (rocprofv3 --kernel-trace --stats
#                                          of bench.py --steps 20 --warmup 3 --no-cpu-baseline, which also
#                                          runs config 5's collect step; three --pmc passes; bench.py
#                                          defaults incl. the CPU-baseline variants);
#                                          pmc.json = python tools/pmc_latest.py gpurun_out/f_r04/prof
#                                          search_res_kernel search_conv_kernel
#     divergence_*.json                 <- tests/test_gpu_divergence.py, tests/test_gpu_conv.py (LZM_REPORT_DIR)
#   bash tools/gpu_final.sh r04 --no-tests
#     conv_mz.json, conv_ez.json        <- tools/conv_bench.py --kind mz|ez --cpu-baseline-secs 30
#     conv_mz_kernel_stats.csv, conv_ez_kernel_stats.csv <- rocprofv3 --kernel-trace --stats of
#                                          tools/conv_bench.py --kind mz|ez --searches 3 (the Pong process
#                                          segfaults in rocprofv3's teardown after writing the files)
#     bench_philox.json, bench_zero_heads.json, bench_collect.json <- bench.py --rng philox / --zero-heads /
#                                          --step collect
#     bench_breakout.json               <- bench.py --workload breakout --cpu-baseline-secs 30
#     bench_c1_gpu.json, ptree_c1_cpu.json <- config 1 (8 envs x 25 sims)
#     phase_timing.txt, phase_timing_zero_heads.txt, conv_phase_ez.txt, conv_phase_mz.txt <- stamped builds
# Earlier round-4 A/B files (ab_*.txt) name their builds inside; tools/ab_libs.sh made them.
bash tools/gpu_final_a.sh r04 && bash tools/gpu_final.sh r04 --no-tests
