"""Drop-in for pso_pytorch/prompt_dataset.py:11-66 (`PromptDataset` + its collate functions).

The reference reads the packaged asset `pso_pytorch/assets/4k_training_prompts.json` (a JSON list of records with a
caption key); that asset is not shipped with this build, so the file (or the records) is passed in.  Records,
`__getitem__` -> {"prompt": ...}, and the collate functions' outputs (padding="max_length", truncation, max_length =
tokenizer.model_max_length, "pt" tensors) are the reference's."""
import json

from torch.utils.data import Dataset


class PromptDataset(Dataset):
    def __init__(self, path=None, caption_key="caption", records=None):
        if records is None:
            if path is None:
                raise ValueError("PromptDataset needs the prompts JSON (the reference's 4k_training_prompts.json) or "
                                 "records=[{caption_key: ...}, ...]")
            with open(path, "r") as f:
                records = json.load(f)
        self.meta = list(records)
        self.caption_key = caption_key

    def __len__(self):
        return len(self.meta)

    def __getitem__(self, idx):
        return {"prompt": self.meta[idx][self.caption_key]}

    @staticmethod
    def _ids(tokenizer, prompts):
        return tokenizer(prompts, return_tensors="pt", padding="max_length", truncation=True,
                         max_length=tokenizer.model_max_length).input_ids

    @staticmethod
    def sd_collate_fn(examples, tokenizer):
        prompts = [e["prompt"] for e in examples]
        return dict(prompts=prompts, input_ids=PromptDataset._ids(tokenizer, prompts))

    @staticmethod
    def sdxl_collate_fn(examples, tokenizer, tokenizer_2):
        prompts = [e["prompt"] for e in examples]
        return dict(prompts=prompts, input_ids_one=PromptDataset._ids(tokenizer, prompts),
                    input_ids_two=PromptDataset._ids(tokenizer_2, prompts))
