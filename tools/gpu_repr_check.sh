set -e
mkdir -p gpurun_out/r05x
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_config5.py -k "downsample or folded_initial or conv_collect_step" > gpurun_out/r05x/t.log 2>&1
bash tools/repr_ab.sh gpurun_out/r05x/ab cur A
