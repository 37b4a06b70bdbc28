"""SpatialVLA configuration surface.

Mirrors the reference's `SpatialVLAConfig` (reference model/configuration_spatialvla.py:22-118):
same `model_type`, same constructor arguments and defaults, same sub-config kinds
(SigLIP vision, Gemma2 text, ZoeDepth), so a `config.json` written by the reference
loads here unchanged and vice versa.  Sub-configs are plain transformers config
objects (data only — no compute comes from transformers on the hot path).

Canonical presets for the hot path (SURVEY.md §8 "Canonical shapes") live in
`spatialvla_amd.presets`.
"""
import warnings

from transformers import CONFIG_MAPPING, AutoConfig
from transformers.configuration_utils import PretrainedConfig


class SpatialVLAConfig(PretrainedConfig):
    model_type = "spatialvla"
    sub_configs = {"text_config": AutoConfig, "vision_config": AutoConfig, "vision_zoe_config": AutoConfig}

    def __init__(
        self,
        vision_config=None,
        text_config=None,
        ignore_index=-100,
        image_token_index=256000,
        vocab_size=257152,
        projection_dim=2048,
        hidden_size=2048,
        vision_zoe_config=None,
        action_token_begin_idx=None,
        spatial_token_num=259,
        use_spatial_token=False,
        ego3d_patch_reso=4,
        n_freqs=8,
        use_vision_zoe=True,
        **kwargs,
    ):
        # reference configuration_spatialvla.py:43-49
        self._ignore_index = ignore_index
        self.image_token_index = image_token_index
        self._vocab_size = vocab_size
        self.projection_dim = projection_dim
        self.hidden_size = hidden_size
        self.is_encoder_decoder = False

        # vision sub-config (reference :51-66); default is SigLIP-So400m/14 @224
        if isinstance(vision_config, dict):
            vision_config = dict(vision_config)
            vision_config.setdefault("model_type", "siglip_vision_model")
            vision_config = CONFIG_MAPPING[vision_config["model_type"]](**vision_config)
        elif vision_config is None:
            vision_config = CONFIG_MAPPING["siglip_vision_model"](
                intermediate_size=4096, hidden_size=1152, patch_size=14, image_size=224,
                num_hidden_layers=27, num_attention_heads=16, vocab_size=257152, vision_use_head=False,
            )
        self.vision_config = vision_config

        # text sub-config (reference :68-81)
        if isinstance(text_config, dict):
            text_config = dict(text_config)
            text_config.setdefault("model_type", "gemma2")
            text_config = CONFIG_MAPPING[text_config["model_type"]](**text_config)
        elif text_config is None:
            text_config = CONFIG_MAPPING["gemma2"](
                hidden_size=2048, num_hidden_layers=18, intermediate_size=16384, num_attention_heads=8,
                num_key_value_heads=1, is_encoder_decoder=False, vocab_size=vocab_size,
            )
        self.text_config = text_config
        # reference :82-83
        self.text_config.num_image_tokens = (self.vision_config.image_size // self.vision_config.patch_size) ** 2
        self.vision_config.projection_dim = projection_dim

        # ZoeDepth sub-config (reference :86-92)
        if isinstance(vision_zoe_config, dict):
            vision_zoe_config = dict(vision_zoe_config)
            vision_zoe_config.setdefault("model_type", "zoedepth")
            vision_zoe_config = CONFIG_MAPPING[vision_zoe_config["model_type"]](**vision_zoe_config)
        self.vision_zoe_config = vision_zoe_config

        # reference :94-100
        self.action_token_begin_idx = action_token_begin_idx
        self.spatial_token_num = spatial_token_num
        self.use_spatial_token = use_spatial_token
        self.ego3d_patch_reso = ego3d_patch_reso
        self.n_freqs = n_freqs
        self.use_vision_zoe = use_vision_zoe
        super().__init__(**kwargs)

    @property
    def ignore_index(self):
        warnings.warn("The `ignore_index` attribute is deprecated.", FutureWarning)
        return self._ignore_index

    @ignore_index.setter
    def ignore_index(self, value):
        self._ignore_index = value

    def to_dict(self):
        out = super().to_dict()
        out.pop("_ignore_index", None)
        return out
