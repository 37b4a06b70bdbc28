"""SpatialVLAProcessor: the AutoProcessor half of the drop-in (reference model/processing_spatialvla.py:35-254).

Host-side (CPU) preprocessing, not a kernel target: prompt assembly (PaliGemma layout: 256 <image> tokens + bos +
prompt + "\\n" [+ action suffix + eos]), tokenization, the image processor, per-dataset camera intrinsics scaled to
the model's image size, labels for training, and `decode_actions` (action tokens -> un-normalised 7-DoF actions).
Same constructor arguments, call signature, BatchFeature keys and error behaviour as the reference, so a checkpoint
directory's processor_config.json (statistics, bin_policy, intrinsic_config, action_config, ...) loads unchanged.

The reference imports PaliGemma helpers that transformers 5 removed (make_batched_images, build_string_from_input,
_is_str_or_image, _validate_images_text_input_order); their transformers-4.47 behaviour is restated below.
"""
import logging as _logging
from typing import Dict, List, Optional, Union

import numpy as np
import torch
from transformers.feature_extraction_utils import BatchFeature
from transformers.image_utils import is_valid_image
from transformers.processing_utils import ProcessingKwargs, ProcessorMixin, TextKwargs
from transformers.tokenization_utils_base import AddedToken

from .action_tokenizer import SpatialActionTokenizer, unnormalize_actions

logger = _logging.getLogger(__name__)

IMAGE_TOKEN = "<image>"
# PaliGemma's extra vocabulary: 1024 location + 128 segmentation tokens (transformers paligemma EXTRA_TOKENS)
EXTRA_TOKENS = [f"<loc{i:0>4}>" for i in range(1024)] + [f"<seg{i:0>3}>" for i in range(128)]


class SpatialVLATextKwargs(TextKwargs, total=False):
    suffix: Optional[Union[str, List[str]]]  # the training target text (PaliGemmaTextKwargs.suffix)


class SpatialVLAProcessorKwargs(ProcessingKwargs, total=False):
    text_kwargs: SpatialVLATextKwargs
    # transformers 4.47 PaliGemmaProcessorKwargs defaults (the reference's pin, requirements.txt:20)
    _defaults = {"text_kwargs": {"padding": False}, "images_kwargs": {"data_format": "channels_first"}}


def _is_str_or_image(elem) -> bool:
    return isinstance(elem, str) or is_valid_image(elem)


def _looks_like_text(x) -> bool:
    return isinstance(x, str) or (isinstance(x, (list, tuple)) and len(x) > 0 and all(isinstance(t, str) for t in x))


def _looks_like_images(x) -> bool:
    if is_valid_image(x):
        return True
    if isinstance(x, (list, tuple)) and x:
        return _looks_like_images(x[0])
    return False


def _flatten_images(images) -> list:
    """make_batched_images: a list of lists of images -> one flat list; an image or flat list -> a list."""
    if isinstance(images, (list, tuple)) and images and isinstance(images[0], (list, tuple)):
        return [img for sub in images for img in sub]
    if isinstance(images, (list, tuple)):
        return list(images)
    return [images]


def _prompt_string(prompt: str, bos_token: str, image_seq_len: int, image_token: str, num_images: int) -> str:
    """build_string_from_input: image tokens for every image, then bos, the prompt and a newline."""
    return f"{image_token * image_seq_len * num_images}{bos_token}{prompt}\n"


class SpatialVLAProcessor(ProcessorMixin):
    attributes = ["image_processor", "tokenizer"]
    valid_kwargs = ["chat_template"]
    image_processor_class = "SiglipImageProcessor"
    tokenizer_class = ("GemmaTokenizer", "GemmaTokenizerFast")

    def __init__(self, image_processor=None, tokenizer=None, chat_template=None, statistics: Optional[dict] = None,
                 bin_policy=None, intrinsic_config=None, action_config=None, num_obs_steps=1, obs_delta=1,
                 action_chunk_size=1, min_sigma=0.0, **kwargs):
        """Reference :40-101."""
        if image_processor is None:
            raise ValueError("You need to specify an `image_processor`.")
        if tokenizer is None:
            raise ValueError("You need to specify a `tokenizer`.")
        if not hasattr(image_processor, "image_seq_length"):
            raise ValueError("Image processor is missing an `image_seq_length` attribute.")
        self.image_seq_length = image_processor.image_seq_length
        if not hasattr(tokenizer, "image_token"):
            tokenizer.add_special_tokens(
                {"additional_special_tokens": [AddedToken(IMAGE_TOKEN, normalized=False, special=True)]})
            self.image_token_id = tokenizer.convert_tokens_to_ids(IMAGE_TOKEN)
        else:
            self.image_token_id = tokenizer.image_token_id
        tokenizer.add_tokens(EXTRA_TOKENS)
        tokenizer.add_bos_token = False
        tokenizer.add_eos_token = False
        super().__init__(image_processor, tokenizer, chat_template=chat_template)

        self.statistics = statistics if statistics else {}
        self.bin_policy = bin_policy
        self.min_sigma = min_sigma
        self.intrinsic_config = intrinsic_config
        self.action_config = action_config
        self.num_obs_steps = num_obs_steps
        self.obs_delta = obs_delta
        self.action_chunk_size = action_chunk_size
        height, width = image_processor.size["height"], image_processor.size["width"]
        # camera matrices of each dataset scaled to the model's image size (:87-95): row 0 by width/W, row 1 by
        # height/H, in float32 as the reference's torch arithmetic
        self.dataset_intrinsics = {}
        for k, v in (intrinsic_config or {}).items():
            K = torch.tensor(v["intrinsic"]).float()
            K[:2] *= torch.tensor([width / v["width"], height / v["height"]])[:, None]
            self.dataset_intrinsics[k] = K
        self.action_tokenizer = SpatialActionTokenizer(
            tokenizer=tokenizer, num_bins=action_config["num_bins"], bin_policy=bin_policy,
            use_spherical=action_config["use_spherical"], min_sigma=min_sigma)

    def __call__(self, images=None, text: Union[str, List[str], None] = None, unnorm_key: Optional[str] = None,
                 suffix_actions: Optional[np.ndarray] = None, **kwargs) -> BatchFeature:
        """Reference :103-192 -> BatchFeature{input_ids, attention_mask[, token_type_ids, labels], pixel_values,
        intrinsic}.  suffix_actions (n, 7) become the action-token suffix (+ eos) with token_type_ids 1 and labels."""
        if _looks_like_text(images) and _looks_like_images(text):
            images, text = text, images  # _validate_images_text_input_order: (text, images) given positionally
        output_kwargs = self._merge_kwargs(SpatialVLAProcessorKwargs, tokenizer_init_kwargs=self.tokenizer.init_kwargs,
                                           **kwargs)
        if suffix_actions is not None:
            suffix = "".join(self.action_tokenizer(suffix_actions).flatten())
        else:
            suffix = output_kwargs["text_kwargs"].pop("suffix", None)
        return_token_type_ids = suffix is not None

        if images is None:
            raise ValueError("`images` are expected as arguments to a `PaliGemmaProcessor` instance.")
        if text is None:
            logger.warning("You are using PaliGemma without a text prefix. It will perform as a picture-captioning "
                           "model.")
            text = ""
        if _is_str_or_image(text):
            text = [text]

        if not any(IMAGE_TOKEN in sample for sample in text):
            if isinstance(text, list) and isinstance(images, list) and len(images) != len(text):
                raise ValueError(f"Received {len(images)} images for {len(text)} prompts. Each prompt should be "
                                 "associated with an image or list of images.")
            if is_valid_image(images):
                images = [[images]]
            elif isinstance(images, list) and is_valid_image(images[0]):
                images = [[image] for image in images]
            elif not (isinstance(images, list) and isinstance(images[0], list) and is_valid_image(images[0][0])):
                raise ValueError("images must be an image, list of images or list of list of images")
            if suffix is not None and _is_str_or_image(suffix):
                suffix = [suffix]
            if suffix is not None:
                suffix = [sfx + self.tokenizer.eos_token for sfx in suffix]
            input_strings = [
                _prompt_string(prompt, self.tokenizer.bos_token, self.image_seq_length, IMAGE_TOKEN,
                               len(image_list) if isinstance(image_list, list) else 1)
                for prompt, image_list in zip(text, images)]
            images = _flatten_images(images)
        else:
            input_strings = []
            for sample in text:  # image tokens already in the prompt: expand each, bos after the last one
                s = sample.replace(IMAGE_TOKEN, IMAGE_TOKEN * self.image_seq_length)
                at = s.rfind(IMAGE_TOKEN)
                cut = at + len(IMAGE_TOKEN) if at != -1 else 0
                input_strings.append(f"{s[:cut] + self.tokenizer.bos_token + s[cut:]}\n")
        pixel_values = self.image_processor(images, **output_kwargs["images_kwargs"])["pixel_values"]

        if output_kwargs["text_kwargs"].get("max_length", None) is not None:
            output_kwargs["text_kwargs"]["max_length"] += self.image_seq_length
        inputs = self.tokenizer(input_strings, text_pair=suffix, return_token_type_ids=return_token_type_ids,
                                **output_kwargs["text_kwargs"])
        intrinsic = (self.dataset_intrinsics[unnorm_key] if unnorm_key in self.dataset_intrinsics
                     else self.dataset_intrinsics["default"])
        data = {**inputs, "pixel_values": pixel_values, "intrinsic": intrinsic}
        if return_token_type_ids:
            data["labels"] = inputs["input_ids"].masked_fill(inputs["token_type_ids"] == 0, -100)
        return BatchFeature(data=data)

    def batch_decode(self, *args, **kwargs):
        return self.tokenizer.batch_decode(*args, **kwargs)

    def decode(self, *args, **kwargs):
        return self.tokenizer.decode(*args, **kwargs)

    @property
    def model_input_names(self):
        names = self.tokenizer.model_input_names + self.image_processor.model_input_names
        return list(dict.fromkeys(names))

    def decode_actions(self, generation_outputs: torch.Tensor, unnorm_key: Optional[str] = None
                       ) -> Dict[str, np.ndarray]:
        """Reference :216-254: the first 3 x action_chunk_size generated ids -> {"actions" (chunk, 7) in dataset
        units (q01/q99 un-normalisation on masked dims), "action_ids" (chunk, 3)}; zero-padded when short."""
        n = 3 * self.action_chunk_size
        ids = generation_outputs[0, :n].detach().cpu().long().numpy()
        assert self.tokenizer.eos_token != ids[-1], \
            "[error] actions contain EOS token, please check you truncation settings!"
        if ids.shape[0] < n:
            logger.warning("Padding zero action!")
            ids = np.concatenate([ids, np.zeros(n - ids.shape[0], dtype=np.longlong)])
        ids = ids.reshape(-1, 3)
        normalized = self.action_tokenizer.decode_token_ids_to_actions(ids)
        if unnorm_key is None:
            logger.warning(f"unnorm_key {unnorm_key} is not in statistics, use next one")
            unnorm_key = next(iter(self.statistics.keys()))
        stats = self.statistics[unnorm_key]["action"]
        actions = np.stack([unnormalize_actions(a, stats) for a in normalized])
        return {"actions": actions, "action_ids": ids}
