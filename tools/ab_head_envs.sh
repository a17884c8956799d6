# GPU: bench.py at another batch size, the committed-HEAD copy in _ab_head/ against the working
# tree, twice each. usage: bash tools/ab_head_envs.sh ENVS
set -e
n=$1
out=gpurun_out/ab_envs_$n; mkdir -p $out
for rep in 1 2; do
  (cd _ab_head && timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --envs $n > ../$out/head_$rep.json 2>&1)
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --envs $n > $out/cur_$rep.json 2>&1
done
for f in $out/*.json; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], d['roofline']['launch_us'])"; done
