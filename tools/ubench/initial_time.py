"""Diagnostic (not shipped): the MLP initial-inference launch timed alone, back to back (warm L2),
against its duration inside the collect step (rocprofv3 trace), to tell its own latency from cache
effects. Prints one JSON line."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from lightzero_amd.initial import FusedInitialInference  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model = bench.build_model(dev, False, 0)
    ii = FusedInitialInference(model)
    B = 256
    obs = torch.from_numpy(np.random.default_rng(0).normal(size=(B, 4)).astype(np.float32)).to(dev)
    for _ in range(5):
        ii.initial_inference(obs)
    torch.cuda.synchronize()
    res = {}
    for n in (1, 10, 100):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            ii.initial_inference(obs)
        e.record()
        torch.cuda.synchronize()
        res[f"us_per_call_x{n}"] = round(s.elapsed_time(e) * 1e3 / n, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
