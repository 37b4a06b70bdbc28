"""Shared by tests/test_processor.py and oracle/gen_processor_golden.py: a deterministic small Gemma tokenizer
(character vocabulary; the real 256k-token Gemma model file is not available offline) and image processor, so the
golden (made by the reference's SpatialVLAProcessor) and the test see the same tokenizer."""
import numpy as np

CHARS = list("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789?.,!'-") + ["▁", "\n", " "]
BASE = ["<pad>", "<eos>", "<bos>", "<unk>"]


def build_tokenizer():
    from transformers import GemmaTokenizer
    vocab = {t: i for i, t in enumerate(BASE)}
    for c in CHARS:
        vocab.setdefault(c, len(vocab))
    return GemmaTokenizer(vocab=vocab, merges=[])


def build_image_processor():
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        from transformers import SiglipImageProcessor
        ip = SiglipImageProcessor(size={"height": 224, "width": 224})
    ip.image_seq_length = 256
    return ip


def images(n, seed=0, hw=(180, 260)):
    from PIL import Image
    rng = np.random.default_rng(seed)
    return [Image.fromarray(rng.integers(0, 256, (hw[0], hw[1], 3), dtype=np.uint8)) for _ in range(n)]
