# GPU: tools/conv_bench.py with an environment variable off / on, interleaved twice.
# usage: bash tools/ab_env_conv.sh OUT_DIR KIND VAR
set -e
out=$1; kind=$2; var=$3
mkdir -p "$out"
for rep in 1 2; do
  for v in 0 1; do
    env $var=$v timeout -k 10 200 python tools/conv_bench.py --kind $kind --searches 20 > "$out/c_${v}_$rep.json" 2>&1
    python3 -c "import json;d=json.loads(open('$out/c_${v}_$rep.json').read().strip().splitlines()[-1]);print('$var=$v', $rep, d['value'], d.get('ms_per_search'))" >> "$out/summary.txt"
  done
done
cat "$out/summary.txt"
