# GPU: the conv / config 5 GPU tests on this build, then the Breakout collect-step bench against
# lightzero_amd/liblzm_varB.so (the previous build), interleaved twice. usage: bash tools/gpu_w1r_check.sh OUT
set -e
out=$1
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_config5.py > $out/t.log 2>&1
for rep in 1 2; do
  for v in cur B; do
    lib=lightzero_amd/liblzmcts.so
    [ "$v" != cur ] && lib=lightzero_amd/liblzm_var$v.so
    LZM_LIB=$lib timeout -k 10 200 python bench.py --workload breakout --step collect --steps 20 --warmup 3 --no-cpu-baseline --configs none > $out/b5_${v}_$rep.json 2>&1
    python3 -c "import json;d=json.loads(open('$out/b5_${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', $rep, 'config5', d['value'], d['ms_per_step'])" >> $out/summary.txt
  done
done
cat $out/summary.txt
