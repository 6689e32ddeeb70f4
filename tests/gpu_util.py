"""Helpers shared by the gpu-marked tests: host<->device u64 transfers."""
import numpy as np
import torch


def to_dev(a: np.ndarray) -> torch.Tensor:
    a = np.ascontiguousarray(a, dtype=np.uint64)
    return torch.from_numpy(a.view(np.int64)).to("cuda:0")


def to_host(t: torch.Tensor) -> np.ndarray:
    torch.cuda.synchronize()
    return t.detach().cpu().numpy().view(np.uint64)


def umax_torch(t: torch.Tensor, dim: int) -> torch.Tensor:
    """Unsigned max with torch int64 ops: flip the sign bit, signed max, flip back."""
    sign = torch.tensor(-(2**63), dtype=torch.int64, device=t.device)
    return (t ^ sign).amax(dim=dim) ^ sign
