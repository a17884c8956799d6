# GPU commands behind this profile set (round 3), one gpurun call each:
#   bash tools/gpu_final.sh r03a
#     gpu_tests.log, smoke.log          <- pytest tests -m gpu; __graft_entry__.smoke()
#     kernel_stats.csv, pmc.json, bench.json <- tools/profile_round.sh r03a (rocprofv3 --kernel-trace --stats
#                                          of bench.py --steps 20 --warmup 3 --no-cpu-baseline; three --pmc
#                                          passes; bench.py defaults incl. the CPU-baseline variants);
#                                          pmc.json = python tools/pmc_latest.py gpurun_out/prof_r03a search_res_kernel
#     conv_mz.json, conv_ez.json        <- tools/conv_bench.py --kind mz|ez (Breakout: one-launch search;
#                                          Pong: generic path with the fused LSTM step)
#     conv_mz_kernel_stats.csv, conv_ez_kernel_stats.csv <- rocprofv3 --kernel-trace --stats of
#                                          tools/conv_bench.py --kind mz|ez --searches 3 (Breakout: ONE
#                                          search_conv_kernel launch per search)
#     bench_philox.json, bench_zero_heads.json, bench_collect.json <- bench.py --rng philox / --zero-heads /
#                                          --step collect (the collect line ends with the trajectory return)
#   bash tools/gpu_conv_iter.sh / gpu_draws.sh: conv_phase_glibc.txt, phase_zero_heads_draws.txt,
#     conv_mz_fused*.json, conv_mz_generic.json, tests_draws.log (iteration points)
#   bash tools/gpu_lstm_pmc.sh lsp1: lstm_sq.txt (SQ counters of ez_lstm_gemm_cell_kernel, tools/lstm_bench.py)
