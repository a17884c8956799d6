"""Timing of the DownSample launches (lzm_repr_downsample, csrc/lzm_repr.h) at several batch sizes, to split each
layer's time into a fixed per-launch part and a per-tile part (run under rocprofv3 --kernel-trace --stats, or
read the HIP-event total printed here).

    python tools/repr_bench.py [--batches 64,256,1024] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from lightzero_amd.conv_infer import FoldedConvInitial  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="64,256,1024")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    fi = FoldedConvInitial(bench.build_conv_model(dev, seed=0))
    assert fi.repr_native is not None
    out = {}
    for B in (int(x) for x in a.batches.split(",")):
        obs = torch.rand(B, 4, 64, 64, device=dev)
        with torch.no_grad():
            for _ in range(3):
                fi._downsample_native(obs)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                fi._downsample_native(obs)
            e1.record()
            torch.cuda.synchronize()
        out[B] = round(e0.elapsed_time(e1) * 1e3 / a.reps, 1)
    print(json.dumps({"us_per_downsample": out}))


if __name__ == "__main__":
    main()
