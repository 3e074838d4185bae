"""Reward functions of the sampling phase, device-resident (the trainer's `reward_fn(decoded images) -> [2B, m]`).

* `light_reward()` -- pso_pytorch/rewards.py:5-9 (`images.reshape(B, -1).mean(1)`): the deterministic synthetic scorer
  SURVEY §8d names for the epoch metric; one `pso_row_mean` launch.
* `pickscore_reward(selector, input_ids)` -- the trainers' PickScore reward (T:632-647 / D:644-649): uint8
  quantisation + CLIPImageProcessor + CLIP-H + matched cosine, all on the GPU (pso_pytorch/pickscore_utils.Selector).
"""
from . import kernels as K


def light_reward():
    def _fn(img):
        return K.row_mean(img)
    return _fn


def pickscore_reward(selector, input_ids):
    """input_ids [n_images, L]: one prompt row per decoded image (image order 2b + k -> prompt b: repeat_interleave)."""
    def _fn(img):
        return selector.score_tensor(img, input_ids)
    return _fn
