# GPU: the DownSample parity tests (tests/test_gpu_config5.py), then tools/repr_ab.sh over the given builds.
# usage: bash tools/gpu_repr_check.sh OUT TAG...
set -e
out=$1; shift
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_config5.py -k "downsample or folded_initial or conv_collect_step" > $out/t.log 2>&1
bash tools/repr_ab.sh $out/ab "$@"
