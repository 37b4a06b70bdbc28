"""Spatial action tokenizer: continuous 7-DoF actions <-> the 8194 spatial action tokens.

Host-side restatement of the reference's model/action_tokenizer.py (classes and call signatures kept so
callers switch by import).  One episode's action chunk becomes 3 tokens per step:

* translation (x, y, z) in [-1, 1]^3 -> spherical (theta, phi, r) -> one token of a theta x phi x r grid
  (reference TranslationTokenizer, action_tokenizer.py:59-139);
* rotation (roll, pitch, yaw) -> one token of a roll x pitch x yaw grid (RotationTokenizer, :141-201);
* gripper -> one of 2 tokens, open iff >= 0.5 (GripperTokenzier, :203-240).

Token ids are laid out [translation | rotation | gripper] starting at the first added token
(`action_token_begin_idx`, 257153 for the PaliGemma2 vocabulary).  Bin edges are uniform in each range or,
given per-axis Gaussian fits (scripts/gs_*.json), equal-probability edges of the fitted Gaussian clipped to
the range (get_bin_policy, :306-336).  All arithmetic is float64 numpy, as in the reference.
"""
from typing import Dict, List, Optional, Sequence

import numpy as np

ACTION_TOKEN = "<ACTION{:05d}>"

# axis ranges of the bin grids (reference SpatialActionTokenizer.range_bins, action_tokenizer.py:243-254)
RANGE_BINS = {
    "translation": {"theta_bins": (0.0, np.pi), "phi_bins": (-np.pi, np.pi), "r_bins": (0.0, np.sqrt(3))},
    "rotation": {"roll_bins": (-1.0, 1.0), "pitch_bins": (-1.0, 1.0), "yaw_bins": (-1.0, 1.0)},
}


def _register(tokenizer, names: Sequence[str]):
    """Add `names` as special tokens (when a tokenizer is given) and return (first id, last id)."""
    tokenizer.add_tokens(list(names), special_tokens=True)
    return tokenizer.convert_tokens_to_ids(names[0]), tokenizer.convert_tokens_to_ids(names[-1])


def _midpoints(edges: np.ndarray, idx: np.ndarray) -> np.ndarray:
    return 0.5 * (edges[idx] + edges[idx + 1])


class ActionTokenizer:
    """Uniform per-dimension binning into `num_bins` tokens (reference :14-56)."""

    def __init__(self, tokenizer, num_bins: int = 256, min_action: int = -1, max_action: int = 1):
        self._vocab_size = num_bins
        self.tokenizer = tokenizer
        self.min_action, self.max_action = min_action, max_action
        self.bin_centers = np.linspace(min_action, max_action, num_bins)
        self.token_array = np.array([ACTION_TOKEN.format(i) for i in range(num_bins)])
        self.token_start_idx, self.token_end_idx = _register(tokenizer, self.token_array)
        self.action_token_begin_idx = self.token_start_idx

    def __call__(self, action: np.ndarray) -> np.ndarray:
        a = np.clip(action, float(self.min_action), float(self.max_action))
        return self.token_array[np.digitize(a, self.bin_centers, right=True)]

    def decode_token_ids_to_actions(self, action_token_id: np.ndarray) -> np.ndarray:
        k = np.clip(action_token_id - self.action_token_begin_idx, 0, self._vocab_size - 1)
        return self.bin_centers[k]

    @property
    def vocab_size(self) -> int:
        return self._vocab_size


class _GridTokenizer:
    """A 3-axis grid of bins whose cell index (i0, i1, i2) maps to token offset (i0 * n1 + i1) * n2 + i2."""

    axes: tuple = ()

    def _init_grid(self, tokenizer, num_bins: Dict, bin_policy: Dict, first_label: int):
        self.tokenizer = tokenizer
        self.n = tuple(int(num_bins[a]) for a in self.axes)
        self._vocab_size = self.n[0] * self.n[1] * self.n[2]
        self.token_array = np.array([ACTION_TOKEN.format(first_label + i) for i in range(self._vocab_size)])
        self.token_start_idx, self.token_end_idx = _register(tokenizer, self.token_array)
        self.set_bins(bin_policy)

    def set_bins(self, bin_policy: Dict):
        self.edges = [np.array(bin_policy[a]) for a in self.axes]
        for a, e in zip(self.axes, self.edges):
            setattr(self, a, e)

    def _flat(self, i0, i1, i2):
        return (i0 * self.n[1] + i1) * self.n[2] + i2

    def _split(self, ids):
        return ids // (self.n[1] * self.n[2]), (ids // self.n[2]) % self.n[1], ids % self.n[2]

    def _cell_centres(self, token_ids):
        ids = np.clip(token_ids, self.token_start_idx, self.token_end_idx) - self.token_start_idx
        return [_midpoints(e, i) for e, i in zip(self.edges, self._split(ids))]

    @property
    def vocab_size(self) -> int:
        return self._vocab_size


class TranslationTokenizer(_GridTokenizer):
    """(x, y, z) -> spherical (theta, phi, r) cell (reference :59-139).  Interior edges only are used for
    digitize, so values outside the range land in the first/last cell."""
    axes = ("theta_bins", "phi_bins", "r_bins")

    def __init__(self, tokenizer, num_bins: Dict, bin_policy: Optional[Dict] = None, use_spherical: bool = True):
        self.use_spherical = use_spherical
        self.num_theta_bins, self.num_phi_bins, self.num_r_bins = (num_bins[a] for a in self.axes)
        self.NP = self.num_phi_bins * self.num_r_bins
        self._init_grid(tokenizer, num_bins, bin_policy, 0)

    @staticmethod
    def cartesian_to_spherical(x, y, z):
        rho = np.sqrt(x ** 2 + y ** 2)
        return np.arctan2(rho, z), np.arctan2(y, x), np.sqrt(x ** 2 + y ** 2 + z ** 2)

    @staticmethod
    def spherical_to_cartesian(theta, phi, r):
        s = r * np.sin(theta)
        return s * np.cos(phi), s * np.sin(phi), r * np.cos(theta)

    def __call__(self, action: np.ndarray) -> np.ndarray:
        c = (self.cartesian_to_spherical(action[:, 0], action[:, 1], action[:, 2]) if self.use_spherical
             else (action[:, 0], action[:, 1], action[:, 2]))
        cell = [np.digitize(v, e[1:-1]) for v, e in zip(c, self.edges)]
        return self.token_array[self._flat(*cell)]

    def decode_token_ids_to_actions(self, action_token_id: np.ndarray) -> np.ndarray:
        t, p, r = self._cell_centres(action_token_id)
        xyz = self.spherical_to_cartesian(t, p, r) if self.use_spherical else (t, p, r)
        # the spherical cells cover the sphere circumscribing the [-1, 1]^3 action cube
        return np.stack(np.clip(np.array(xyz), -1, 1), axis=1)


class RotationTokenizer(_GridTokenizer):
    """(roll, pitch, yaw) cell (reference :141-201); full edge lists, cell = clip(digitize - 1)."""
    axes = ("roll_bins", "pitch_bins", "yaw_bins")

    def __init__(self, tokenizer, num_bins: Dict, bin_policy: Optional[Dict] = None, array_begin_idx=None):
        self.array_begin_idx = array_begin_idx
        self.num_roll_bins, self.num_pitch_bins, self.num_yaw_bins = (num_bins[a] for a in self.axes)
        self.NP = self.num_pitch_bins * self.num_yaw_bins
        self._init_grid(tokenizer, num_bins, bin_policy, array_begin_idx)

    def __call__(self, action: np.ndarray) -> np.ndarray:
        cell = [np.clip(np.digitize(action[:, k], e) - 1, 0, n - 1)
                for k, (e, n) in enumerate(zip(self.edges, self.n))]
        return self.token_array[self._flat(*cell)]

    def decode_token_ids_to_actions(self, action_token_id) -> np.ndarray:
        return np.stack(self._cell_centres(action_token_id), axis=1)


class GripperTokenzier:  # reference spelling (action_tokenizer.py:203), kept for drop-in imports
    """gripper >= 0.5 -> token 1 (open), else token 0 (reference :203-240)."""

    def __init__(self, tokenizer, num_bins: int = 2, array_begin_idx=None) -> None:
        self.tokenizer = tokenizer
        self.num_bins = num_bins
        self.array_begin_idx = array_begin_idx
        self.token_array = np.array([ACTION_TOKEN.format(array_begin_idx + i) for i in range(num_bins)])
        self.token_start_idx, self.token_end_idx = _register(tokenizer, self.token_array)

    def __call__(self, action: np.ndarray) -> np.ndarray:
        return self.token_array[(action >= 0.5).astype(np.int64)]

    def decode_token_ids_to_actions(self, action_token_id: np.ndarray) -> np.ndarray:
        k = np.clip(action_token_id, self.token_start_idx, self.token_end_idx) - self.token_start_idx
        return (k != 0).astype(np.float64)[:, None]

    @property
    def vocab_size(self) -> int:
        return self.num_bins


GripperTokenizer = GripperTokenzier


def bin_policy_from(num_bins: Dict, gs_params: Optional[Dict] = None, min_sigma: float = 0.0) -> Dict:
    """Bin edges per axis (reference get_bin_policy, action_tokenizer.py:306-336): uniform over the axis range,
    or the equal-probability edges of N(mu, max(sigma, min_sigma)) restricted to the range."""
    from scipy.stats import norm
    policy = {}
    for kind, axes in RANGE_BINS.items():
        policy[kind] = {}
        for axis, (lo, hi) in axes.items():
            n = num_bins[kind][axis]
            if gs_params is None:
                policy[kind][axis] = np.linspace(lo, hi, n + 1)
                continue
            g = gs_params[axis.split("_")[0].lower()]
            mu, sigma = g["mu"], max(g["sigma"], min_sigma)
            p = np.linspace(norm.cdf(lo, loc=mu, scale=sigma), norm.cdf(hi, loc=mu, scale=sigma), n + 1)
            policy[kind][axis] = np.clip(norm.ppf(p, loc=mu, scale=sigma), lo, hi).tolist()
    return policy


class SpatialActionTokenizer:
    """[translation, rotation, gripper] tokens per action step (reference :242-430)."""
    range_bins = RANGE_BINS

    def __init__(self, tokenizer, num_bins: Dict, gs_params: Dict = None, bin_policy: Dict = None,
                 use_spherical: bool = True, min_sigma: float = 0.0, min_action: float = -1.0,
                 max_action: float = 1.0):
        self.tokenizer = tokenizer
        self.min_action, self.max_action = min_action, max_action
        self.num_bins = num_bins
        self.min_sigma = min_sigma
        self.bin_policy = bin_policy if bin_policy else self.get_bin_policy(gs_params, min_sigma)
        self.translation_tokenizer = TranslationTokenizer(tokenizer, num_bins["translation"],
                                                          self.bin_policy["translation"], use_spherical=use_spherical)
        self.rotation_tokenizer = RotationTokenizer(tokenizer, num_bins["rotation"], self.bin_policy["rotation"],
                                                    array_begin_idx=self.translation_tokenizer.vocab_size)
        self.gripper_tokenizer = GripperTokenzier(
            tokenizer, num_bins["gripper"],
            array_begin_idx=self.translation_tokenizer.vocab_size + self.rotation_tokenizer.vocab_size)
        self._vocab_size = (self.translation_tokenizer.vocab_size + self.rotation_tokenizer.vocab_size
                            + self.gripper_tokenizer.vocab_size)

    def get_bin_policy(self, gs_params=None, min_sigma=0.0):
        return bin_policy_from(self.num_bins, gs_params, min_sigma)

    def __call__(self, action: np.ndarray) -> np.ndarray:
        """action (n, 7) or (7,) in [-1, 1] -> token strings (n, 3)."""
        a = np.asarray(action)
        if a.ndim == 1:
            assert a.shape[0] == 7, f"action dim mismatch, got action shape: {a.shape}"
            a = a.reshape(1, 7)
        assert a.shape[1] == 7, f"action dim mismatch, got action shape: {a.shape}"
        a = np.clip(a, self.min_action, self.max_action)
        return np.stack((self.translation_tokenizer(a[:, :3]), self.rotation_tokenizer(a[:, 3:6]),
                         self.gripper_tokenizer(a[:, 6])), axis=1)

    def token_ids(self, action: np.ndarray) -> np.ndarray:
        """Like __call__ but returns int64 token ids (n, 3)."""
        toks = self(action)
        flat = [int(self.tokenizer.convert_tokens_to_ids(t)) for t in toks.reshape(-1)]
        return np.array(flat, dtype=np.int64).reshape(toks.shape)

    def decode_token_ids_to_actions(self, action_token_ids: np.ndarray) -> np.ndarray:
        """token ids (n, 3) or (3,) -> normalized actions (n, 7)."""
        ids = np.asarray(action_token_ids)
        if ids.ndim == 1:
            assert ids.shape[0] == 3, f"action token id numbers mismatich, need 3 got {ids.shape[0]}"
            ids = ids.reshape(1, 3)
        assert ids.shape[1] == 3, f"token id numbers mismatich, need 3 got {ids.shape[1]}"
        return np.concatenate((self.translation_tokenizer.decode_token_ids_to_actions(ids[:, 0]),
                               self.rotation_tokenizer.decode_token_ids_to_actions(ids[:, 1]),
                               self.gripper_tokenizer.decode_token_ids_to_actions(ids[:, 2])), axis=1)

    @property
    def vocab_size(self) -> int:
        return self._vocab_size

    @property
    def action_token_begin_idx(self) -> int:
        return self.translation_tokenizer.token_start_idx


def unnormalize_actions(normalized: np.ndarray, action_stats: Dict) -> np.ndarray:
    """[-1, 1] actions -> dataset units with the q01/q99 statistics (reference processing_spatialvla.py:241-253):
    a = 0.5 (x + 1)(q99 - q01) + q01 on masked dims, x elsewhere."""
    dim = len(action_stats["q01"])
    mask = np.array(action_stats.get("mask", np.ones(dim)), dtype=bool)
    hi, lo = np.array(action_stats["q99"]), np.array(action_stats["q01"])
    return np.where(mask, 0.5 * (normalized + 1) * (hi - lo) + lo, normalized)


def decode_actions(generated_ids, action_tokenizer: SpatialActionTokenizer, statistics: Dict, unnorm_key: str,
                   action_chunk_size: int, eos_token_id: Optional[int] = None) -> Dict[str, np.ndarray]:
    """Generated token ids [1, >= 3*chunk] -> {"actions": (chunk, 7), "action_ids": (chunk, 3)}
    (reference SpatialVLAProcessor.decode_actions, processing_spatialvla.py:221-253)."""
    n = 3 * action_chunk_size
    ids = np.asarray(generated_ids)[0, :n].astype(np.int64)
    if eos_token_id is not None:
        assert ids[-1] != eos_token_id, "[error] actions contain EOS token, please check you truncation settings!"
    if ids.shape[0] < n:
        ids = np.concatenate([ids, np.zeros(n - ids.shape[0], dtype=np.int64)])
    ids = ids.reshape(-1, 3)
    normalized = action_tokenizer.decode_token_ids_to_actions(ids)
    actions = np.stack([unnormalize_actions(a, statistics[unnorm_key]["action"]) for a in normalized])
    return {"actions": actions, "action_ids": ids}


def scale_intrinsics(intrinsic_config: Dict, height: int, width: int) -> Dict[str, np.ndarray]:
    """Per-dataset camera matrices rescaled to the model's image size (processing_spatialvla.py:87-95):
    rows 0 and 1 of K scale by width/W and height/H."""
    out = {}
    for key, v in intrinsic_config.items():
        K = np.array(v["intrinsic"], dtype=np.float32)
        K[0] *= np.float32(width / v["width"])
        K[1] *= np.float32(height / v["height"])
        out[key] = K
    return out


def prompt_token_layout(prompt_ids: List[int], image_token_id: int, image_seq_len: int, bos_id: int,
                        newline_ids: List[int], suffix_ids: Optional[List[int]] = None,
                        eos_id: Optional[int] = None) -> Dict[str, np.ndarray]:
    """Token layout the processor builds (processing_spatialvla.py:152-191, PaliGemma's
    build_string_from_input): <image> * image_seq_len + bos + prompt + "\\n" [+ suffix + eos], with
    token_type_ids = 1 on the suffix and labels = ids on the suffix, -100 elsewhere."""
    prefix = [image_token_id] * image_seq_len + [bos_id] + list(prompt_ids) + list(newline_ids)
    suffix = [] if suffix_ids is None else list(suffix_ids) + ([eos_id] if eos_id is not None else [])
    ids = np.array(prefix + suffix, dtype=np.int64)
    tt = np.array([0] * len(prefix) + [1] * len(suffix), dtype=np.int64)
    out = {"input_ids": ids, "attention_mask": np.ones_like(ids)}
    if suffix_ids is not None:
        out["token_type_ids"] = tt
        out["labels"] = np.where(tt == 0, -100, ids)
    return out
