"""Real ImageNet sources on the native reader (csrc/io/imagenet_io.cpp, module `_pddl_io`).

Reference input pipeline (imagenet-resnet50.py:16-49): tfds.load('imagenet2012', split=
['train', 'validation'], as_supervised=True, data_dir=...) -> map(resize_with_crop(224)) ->
batch -> prefetch.  No network on the target machines, so nothing is downloaded: point the
sources at data already on disk.

  * ``tfds:<dir>``   — the TFRecord shards tfds prepared (``imagenet2012-train.tfrecord-*``,
                        ``imagenet2012-validation.tfrecord-*`` anywhere under <dir>), read
                        with CRC checks, tf.Example parsing and libjpeg decoding in C++.
  * ``folder:<dir>`` — untarred ILSVRC class folders (<dir>/<split>/<synset>/*.JPEG), labels
                        = index of the synset in sorted order (the tfds label order).
Both apply tf.image.resize_with_crop_or_pad to image_size x image_size (C6) in the decoder
and hand back uint8 NHWC batches; the in-model Rescaling/RandomCrop/RandomFlip run on the GPU.

``write_tfrecord_imagenet`` writes the same format (tests, small local subsets) and
``scripts/make_records.py`` converts either source into the raw mmap records
(``records:<dir>``) that the fastest loader path consumes.
"""
from __future__ import annotations

import glob
import importlib.machinery
import importlib.util
import os
import struct
from typing import List, Optional, Sequence

import numpy as np
import torch

from .datasets import ImageSource

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_io = None


def io_module():
    global _io
    if _io is None:
        import torch  # noqa: F401  (libc10 first)
        cands = sorted(glob.glob(os.path.join(os.environ.get("PDDL_NATIVE_DIR") or _PKG, "_pddl_io*.so")))
        if not cands:
            raise RuntimeError("native ImageNet reader _pddl_io not built (run `python pddl_build.py`)")
        loader = importlib.machinery.ExtensionFileLoader("_pddl_io", cands[-1])
        spec = importlib.util.spec_from_file_location("_pddl_io", cands[-1], loader=loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        _io = mod
    return _io


_SPLIT = {"train": "train", "val": "validation", "validation": "validation"}


def _host_batch(n: int, S: int):
    pin = torch.cuda.is_available()
    return (torch.empty((n, S, S, 3), dtype=torch.uint8, pin_memory=pin),
            torch.empty((n,), dtype=torch.int64, pin_memory=pin))


class TFDSImageNet(ImageSource):
    def __init__(self, root: str, split: str = "train", image_size: int = 224, num_classes: int = 1000,
                 threads: int = 8, files: Optional[Sequence[str]] = None):
        tag = _SPLIT.get(split, split)
        if files is None:
            files = sorted(glob.glob(os.path.join(root, "**", f"*-{tag}.tfrecord*"), recursive=True))
        if not files:
            raise FileNotFoundError(f"no '*-{tag}.tfrecord*' shards under {root}")
        self.files = list(files)
        self.reader = io_module().TFRecordImageNet(self.files, image_size, threads)
        self.num_examples = len(self.reader)
        self.image_size = image_size
        self.num_classes = num_classes

    host = True

    def fetch_host(self, idx: np.ndarray):
        """Decode into pinned host buffers (native thread pool, GIL released)."""
        n = len(idx)
        img, lab = _host_batch(n, self.image_size)
        self.reader.fetch(torch.from_numpy(np.ascontiguousarray(idx, dtype=np.int64)), img, lab)
        return img, lab


class JpegFolderImageNet(ImageSource):
    def __init__(self, root: str, split: str = "train", image_size: int = 224, num_classes: int = 1000,
                 threads: int = 8):
        base = os.path.join(root, split)
        if not os.path.isdir(base) and split == "val":
            base = os.path.join(root, "validation")
        classes = sorted(d for d in os.listdir(base) if os.path.isdir(os.path.join(base, d)))
        if not classes:
            raise FileNotFoundError(f"no class folders under {base}")
        files: List[str] = []
        labels: List[int] = []
        for ci, c in enumerate(classes):
            for f in sorted(os.listdir(os.path.join(base, c))):
                if f.lower().endswith((".jpeg", ".jpg")):
                    files.append(os.path.join(base, c, f))
                    labels.append(ci)
        self.files = files
        self.labels = np.asarray(labels, dtype=np.int64)
        self.classes = classes
        self.reader = io_module().JpegFiles(image_size, threads)
        self.num_examples = len(files)
        self.image_size = image_size
        self.num_classes = num_classes

    host = True

    def fetch_host(self, idx: np.ndarray):
        n = len(idx)
        img, lab = _host_batch(n, self.image_size)
        self.reader.fetch([self.files[i] for i in idx], img)
        lab.copy_(torch.from_numpy(self.labels[np.asarray(idx)]))
        return img, lab


# ------------------------------------------------------------------ writing (tests, subsets)
def _varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num: int, payload: bytes) -> bytes:
    return _varint((num << 3) | 2) + _varint(len(payload)) + payload


def encode_example(image_jpeg: bytes, label: int, file_name: str = "") -> bytes:
    """tf.Example {"image": bytes, "label": int64, "file_name": bytes} (tfds imagenet2012)."""
    def entry(key: str, feature: bytes) -> bytes:
        return _field(1, _field(1, key.encode()) + _field(2, feature))
    img_f = _field(1, _field(1, image_jpeg))                              # Feature.bytes_list
    lab_f = _field(3, _field(1, _varint(label & 0xFFFFFFFFFFFFFFFF)))    # Feature.int64_list (packed)
    name_f = _field(1, _field(1, file_name.encode()))
    return _field(1, entry("image", img_f) + entry("label", lab_f) + entry("file_name", name_f))


def write_tfrecord_imagenet(path: str, jpegs: Sequence[bytes], labels: Sequence[int]) -> None:
    crc = io_module().masked_crc32c
    with open(path, "wb") as f:
        for i, (jb, lab) in enumerate(zip(jpegs, labels)):
            data = encode_example(jb, int(lab), f"img_{i}.JPEG")
            hdr = struct.pack("<Q", len(data))
            f.write(hdr + struct.pack("<I", crc(hdr)) + data + struct.pack("<I", crc(data)))


def resize_with_crop_or_pad(img: np.ndarray, S: int) -> np.ndarray:
    """NumPy reference of tf.image.resize_with_crop_or_pad (HWC uint8)."""
    H, W = img.shape[:2]
    cy, cx = max((H - S) // 2, 0), max((W - S) // 2, 0)
    crop = img[cy:cy + min(H, S), cx:cx + min(W, S)]
    out = np.zeros((S, S, img.shape[2]), dtype=img.dtype)
    py, px = max((S - H) // 2, 0), max((S - W) // 2, 0)
    out[py:py + crop.shape[0], px:px + crop.shape[1]] = crop
    return out
