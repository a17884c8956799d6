# GPU: per-phase cycle counts of repr_conv_kernel's tile loop from a diagnostic build (liblzm_varD.so: clock64
# stamps, printf of blocks 0 / 100, waves 0 / 7), tools/repr_bench.py at B = 256
set -e
mkdir -p ${1:-gpurun_out/r05y}
LZM_LIB=lightzero_amd/liblzm_varD.so timeout -k 10 120 python3 tools/repr_bench.py --batches 256 --reps 1 > ${1:-gpurun_out/r05y}/diag.log 2>&1
grep REPRDIAG ${1:-gpurun_out/r05y}/diag.log | sort | uniq | head -60 > ${1:-gpurun_out/r05y}/diag_summary.txt
