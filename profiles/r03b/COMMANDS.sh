# GPU commands behind this profile set (round 3, second session), one gpurun call each:
#   bash tools/gpu_final.sh r03b
#     gpu_tests.log, smoke.log          <- pytest tests -m gpu (207 passed); __graft_entry__.smoke()
#     kernel_stats.csv, pmc.json, bench.json <- tools/profile_round.sh r03b (rocprofv3 --kernel-trace --stats
#                                          of bench.py --steps 20 --warmup 3 --no-cpu-baseline; three --pmc
#                                          passes; bench.py defaults incl. the CPU-baseline variants);
#                                          pmc.json = python tools/pmc_latest.py gpurun_out/prof_r03b search_res_kernel
#     conv_mz.json, conv_ez.json        <- tools/conv_bench.py --kind mz|ez (both one-launch searches now)
#     conv_mz_kernel_stats.csv, conv_ez_kernel_stats.csv <- rocprofv3 --kernel-trace --stats of
#                                          tools/conv_bench.py --kind mz|ez --searches 3 (ONE search kernel
#                                          launch per search: search_conv_kernel / search_conv_ez_kernel)
#     conv_phase_ez.txt, conv_phase_mz.txt <- tools/conv_phase_timing.py --kind ez|mz (stamped builds)
#     bench_philox.json, bench_zero_heads.json, bench_collect.json <- bench.py --rng philox / --zero-heads /
#                                          --step collect
#     bench_c1_gpu.json, ptree_c1_cpu.json <- config 1 (8 envs x 25 sims): bench.py --envs 8 --sims 25;
#                                          tools/ptree_bench.py (the ptree restatement, 1 host thread, MLP on
#                                          torch-CPU)
#   bash tools/gpu_res_ab.sh res1 base: phase_timing.txt (tools/phase_timing.py, headline kernel, stamped build)
#   bash tools/gpu_ez_variants.sh ez7: ez_phase_coalesced.txt; bash tools/gpu_ez_diag.sh ez6 ezd1 ezd2 ezd4 ezd6:
#     phase_ezd*.txt (EZ diagnostic builds: 1 no trunk layers, 2 one W slice for every tile, 4 one xin row
#     block for every tile, 6 both; results invalid, cycles valid)
