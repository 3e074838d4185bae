"""Drop-in for pso_pytorch/pickscore_utils.py:12-62 (`Selector`): the PickScore reward, GPU-resident.

Reference: `Selector(device, cache_dir)` loads CLIPProcessor("laion/CLIP-ViT-H-14-laion2B-s32B-b79K") and
CLIPModel("yuvalkirstain/PickScore_v1") from the hub; `score(images, prompt, softmax=False)` takes PIL images (made
from the uint8 numpy arrays of T:632-640), runs the processor (PIL bicubic resize / crop / normalise) and the model,
and returns diag(text_n @ image_n^T) (or softmax(logit_scale * scores)) as numpy.

Here the checkpoint / tokenizer come from local directories (no network); without them the model is the ViT-H/14
PickScore architecture with synthetic weights.  `score` keeps the reference's signature (PIL images or uint8 arrays
accepted); `score_tensor` is the device path the trainer uses: decoded images NHWC bf16 in [-1, 1] -> quantise ->
resize -> CLIP-H -> cosine of matched rows, with no host round trip (the reference's `.cpu().numpy()` + PIL
conversion, the last host round trip of the epoch)."""
import numpy as np
import torch

from ..clip import CLIPModel, CLIPTextConfig, CLIPVisionConfig, CLIP_MEAN, CLIP_STD
from .. import kernels as K


class Selector:
    def __init__(self, device, cache_dir=None, model_path=None, processor_path=None, seed=0, text_config=None,
                 vision_config=None):
        self.device = torch.device(device)
        if model_path is not None:
            self.model = CLIPModel.from_pretrained(model_path).to(self.device)
        else:
            with torch.device(self.device):
                self.model = CLIPModel(text_config or CLIPTextConfig.pickscore_h(),
                                       vision_config or CLIPVisionConfig())
            self.model.init_weights(seed)
        self.tokenizer = None
        self.mean, self.std = CLIP_MEAN, CLIP_STD
        if processor_path is not None:
            from ..prompts import load_tokenizer
            self.tokenizer = load_tokenizer(processor_path)
            import json
            import os
            pp = os.path.join(processor_path, "preprocessor_config.json")
            if os.path.exists(pp):
                with open(pp) as f:
                    cfg = json.load(f)
                self.mean, self.std = tuple(cfg.get("image_mean", self.mean)), tuple(cfg.get("image_std", self.std))

    def tokenize(self, prompt):
        """processor(text=prompt, padding=True, truncation=True, max_length=77) -> input_ids [B, L]."""
        if self.tokenizer is None:
            raise RuntimeError("no tokenizer directory was given (processor_path); pass input_ids instead")
        return self.tokenizer(list(prompt) if not isinstance(prompt, str) else [prompt], padding=True,
                              truncation=True, max_length=77, return_tensors="pt").input_ids

    @torch.no_grad()
    def score_tensor(self, img_nhwc, input_ids, softmax=False):
        """img_nhwc [B, H, W, 3]: bf16 in [-1, 1] (the VAE decode output, quantised as T:632-633 does) or uint8;
        input_ids [B, L] (one prompt per image) -> scores [B] fp32 on the device."""
        image_embs = self.model.image_features_from_images(img_nhwc, self.mean, self.std)
        text_embs = self.model.get_text_features(input_ids.to(self.device))
        scores = K.cosine_rows(text_embs, image_embs)
        if softmax:
            return torch.softmax(self.model.logit_scale.exp() * scores, dim=-1)
        return scores

    def score(self, images, prompt, softmax=False, input_ids=None):
        """Reference signature: images = list of PIL images / uint8 HWC arrays (or a decoded NHWC tensor), prompt =
        list of strings -> numpy scores."""
        if isinstance(images, torch.Tensor):
            img = images
        else:
            img = torch.from_numpy(np.stack([np.asarray(im, dtype=np.uint8) for im in images])).to(self.device)
        ids = input_ids if input_ids is not None else self.tokenize(prompt)
        s = self.score_tensor(img, ids, softmax)
        return s.cpu().numpy()
