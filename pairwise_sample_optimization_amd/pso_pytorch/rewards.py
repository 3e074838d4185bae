"""Drop-in for pso_pytorch/rewards.py:5-9 `light_reward()`: `_fn(images, prompts, metadata) -> (np.array, {})` with
the per-image mean computed by the HIP `pso_row_mean` kernel when the images are a GPU tensor (NHWC bf16 decode
output or any [B, ...] bf16 / float tensor)."""
import numpy as np
import torch

from .. import kernels as K


def light_reward():
    def _fn(images, prompts, metadata):
        if isinstance(images, torch.Tensor) and images.is_cuda:
            x = images if images.dtype == torch.bfloat16 else images.to(torch.bfloat16)
            r = K.row_mean(x.contiguous())
        else:
            r = torch.as_tensor(np.asarray(images)).reshape(len(images), -1).float().mean(1)
        return np.array(r.cpu().detach()), {}
    return _fn
