# GPU: the default bench's conv objects (config 5 = the Breakout secondary, config 3) for two library builds,
# interleaved twice. usage: bash tools/gpu_bench_ab.sh OUT_DIR A B
set -e
out=$1; shift
mkdir -p "$out"
for rep in 1 2; do
  for v in "$@"; do
    LZM_LIB=lightzero_amd/liblzm_var$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --configs 3 > "$out/b_${v}_$rep.json" 2>&1
    python3 -c "import json;d=json.loads(open('$out/b_${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', $rep, d['value'], d['config5']['ms_per_step'], d['config3']['ms_per_step'])" >> "$out/summary.txt"
  done
done
cat "$out/summary.txt"
