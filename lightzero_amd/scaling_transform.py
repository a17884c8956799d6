"""InverseScalarTransform (reference: lzero/policy/scaling_transform.py:97-128) as one HIP kernel.

``__call__(logits)`` -> [rows, 1] float32 on the logits' device: softmax over the categorical
support (skipped when every row already sums to 1 within allclose tolerance, as
``ensure_softmax`` does, :36-62), expectation over [-support_size, support_size], then
h^-1(x) = sign(x) * (((sqrt(1 + 4 eps (|x| + 1 + eps)) - 1) / (2 eps))^2 - 1), eps = 0.001.
"""
import torch

from ._lib import call, ptr, require_gpu, stream_ptr


class InverseScalarTransform:
    def __init__(self, support_size: int, device='cuda', categorical_distribution: bool = True) -> None:
        self.support_size = int(support_size)
        self.device = device
        self.categorical_distribution = bool(categorical_distribution)

    def __call__(self, logits: torch.Tensor, epsilon: float = 0.001) -> torch.Tensor:
        if abs(epsilon - 0.001) > 0:
            raise ValueError("only the reference epsilon (0.001) is implemented on device")
        require_gpu()
        x = logits.detach().float().contiguous()
        rows = x.shape[0]
        V = x.shape[1] if x.dim() > 1 else 1
        if self.categorical_distribution and V != 2 * self.support_size + 1:
            raise ValueError(f"support length {V} != 2*{self.support_size}+1")
        out = torch.empty((rows, 1), dtype=torch.float32, device=x.device)
        call("lzm_inverse_scalar_transform", ptr(x), int(rows), int(V), int(self.categorical_distribution), ptr(out),
             stream_ptr())
        return out
