# GPU: tools/az_bench.py (config 4's fused search) against several builds (lightzero_amd/liblzm_var<X>.so, LZM_LIB),
# interleaved, twice each. usage: bash tools/ab_az.sh OUT_DIR A B ...
set -e
out=$1; shift
mkdir -p "$out"
for rep in 1 2; do
  for v in "$@"; do
    LZM_LIB=lightzero_amd/liblzm_var$v.so timeout -k 10 200 python tools/az_bench.py --no-reference --searches 30 > "$out/az_${v}_$rep.json" 2>&1
    python3 -c "import json;d=json.loads(open('$out/az_${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', $rep, round(d['value']/1e6,2), round(d['kernel_ms_per_search']*1e3,1))" >> "$out/summary.txt"
  done
done
cat "$out/summary.txt"
