# GPU box entry point (one parameterised script for every gpurun call; replaces the one-off wrappers).
# usage: bash tools/gpu.sh <out-dir> <step> [<step> ...]
#   tests:<pytest args, comma-separated>   e.g. tests:tests/test_gpu_config5.py,-k,breakout
#   alltests                              the whole -m gpu suite
#   smoke                                 __graft_entry__.smoke()
#   bench:<bench.py args, comma-separated> one bench line into <out>/bench_<n>.json
#   conv:<mz|ez>[,args]                   tools/conv_bench.py line
#   profile                               tools/profile_round.sh into <out>
#   cmd:<command, comma-separated>        any other command (own timeout 300 s)
# Every step runs under its own time limit; the first failing step ends the call.
set -e
out=$1
shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export LZM_REPORT_DIR="$GRAFT_REPO_ROOT/$out"  # tests write their measured reports here (tests/divergence.py)
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  arg=${step#*:}
  [ "$arg" = "$step" ] && arg=""
  args=${arg//,/ }
  case $kind in
    tests) timeout -k 10 900 python -u -m pytest -v --timeout 240 --timeout-method thread $args \
             > "$out/tests_$n.log" 2>&1 ;;
    alltests) timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
             > "$out/gpu_tests.log" 2>&1 ;;
    smoke) timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 ;;
    bench) timeout -k 10 400 python -u bench.py $args > "$out/bench_$n.json" 2> "$out/bench_$n.err" ;;
    conv) timeout -k 10 300 python -u tools/conv_bench.py --kind $args > "$out/conv_$n.json" 2> "$out/conv_$n.err" ;;
    profile) bash tools/profile_round.sh "$out" ;;
    cmd) timeout -k 10 300 $args > "$out/cmd_$n.log" 2>&1 ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
  echo "step $n ($kind) done" >&2
done
