# GPU: first half of the round's closing set into gpurun_out/f_<tag> — the whole -m gpu suite, smoke,
# and the profile set of the default bench command (tools/profile_round.sh). Second half:
# tools/gpu_final.sh <tag> --no-tests. usage: bash tools/gpu_final_a.sh <tag>
set -e
tag=${1:-r04}
out=gpurun_out/f_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export LZM_REPORT_DIR="$GRAFT_REPO_ROOT/$out"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $out/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
bash tools/profile_round.sh $out/prof
