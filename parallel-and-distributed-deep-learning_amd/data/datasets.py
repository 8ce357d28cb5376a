"""Input pipeline with the reference's tf.data semantics.

Reference pipeline (imagenet-resnet50.py:28-49): tfds ImageNet2012 -> map(resize_with_crop
to 224) -> batch(B, drop_remainder=True) -> prefetch; Horovod shards AFTER batching
(hvd.py:77-78, each rank takes every size-th batch); MWMS uses AutoShardPolicy.DATA
(multiworkers.py:66-69: element-wise sharding); PS repeats forever (ps.py:118-119).

Sources (no network on the target machines, so no tfds download):
  * SyntheticImageNet — deterministic uint8 [224,224,3] images + labels generated on the
    device (the benchmark data, BASELINE.json "synthetic 3x224x224").
  * RecordsImageNet — a directory of raw uint8 records (`<split>.u8` = N x 224 x 224 x 3,
    `<split>_labels.i64`), memory-mapped and gathered by the native loader thread pool
    (csrc/runtime/loader.cpp) into pinned buffers, then copied asynchronously to the GPU.
  * TFDSImageNet / JpegFolderImageNet (data/imagenet.py) — the reference's tfds TFRecord
    shards or the untarred ILSVRC folders, decoded by the native reader (csrc/io); with
    --cache <dir> behind a DecodedCache (decode once, then mmap gathers).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Iterator, List, Optional, Tuple

import numpy as np
import torch


class ImageSource:
    """A source either generates batches on the device (`fetch`, host = False) or loads them
    into host memory (`fetch_host` -> pinned uint8 images + int64 labels, host = True: decode /
    gather on native thread pools with the GIL released), which the pipeline's prefetch stage
    runs ahead of the training thread and copies to the device asynchronously."""
    num_examples: int
    image_size: int
    num_classes: int
    host = False

    def fetch_host(self, idx: np.ndarray) -> Tuple[torch.Tensor, torch.Tensor]:
        raise NotImplementedError

    def fetch(self, idx: np.ndarray, device) -> Tuple[torch.Tensor, torch.Tensor]:
        if not self.host:
            raise NotImplementedError
        img, lab = self.fetch_host(idx)
        return img.to(device, non_blocking=True), lab.to(device, non_blocking=True)


class SyntheticImageNet(ImageSource):
    """Deterministic synthetic ImageNet: image i depends only on (seed, i)."""

    def __init__(self, num_examples: int, image_size: int = 224, num_classes: int = 1000, seed: int = 0,
                 fixed: bool = False):
        self.num_examples = num_examples
        self.image_size = image_size
        self.num_classes = num_classes
        self.seed = seed
        self.fixed = fixed          # benchmark mode: one device-resident batch reused
        self._cache = {}

    def fetch(self, idx: np.ndarray, device):
        n = len(idx)
        S = self.image_size
        if self.fixed:
            key = (n, str(device))
            if key not in self._cache:
                g = torch.Generator(device=device).manual_seed(self.seed)
                self._cache[key] = (
                    torch.randint(0, 256, (n, S, S, 3), dtype=torch.uint8, device=device, generator=g),
                    torch.randint(0, self.num_classes, (n,), dtype=torch.int64, device=device, generator=g))
            return self._cache[key]
        # per-example deterministic content (counter-based hash of (seed, example, pixel)):
        # the same example has the same pixels whatever batch / shard it is fetched in.
        # On the GPU one native kernel generates the batch (csrc/kernels/eltwise.hip synth).
        if torch.device(device).type == "cuda":
            from ..ops.native import require_native
            ii = torch.as_tensor(np.asarray(idx, dtype=np.int64)).to(device, non_blocking=True)
            img = torch.empty(n, S, S, 3, dtype=torch.uint8, device=device)
            lab = torch.empty(n, dtype=torch.int64, device=device)
            require_native().synth(ii, self.seed, self.num_classes, img, lab)
            return img, lab
        ii = torch.as_tensor(np.asarray(idx, dtype=np.int64), device=device).view(-1, 1)
        p = torch.arange(S * S * 3, dtype=torch.int64, device=device).view(1, -1)
        x = ii * 0x9E3779B1 + p * 0x85EBCA77 + (self.seed + 1) * 0xC2B2AE3D
        x = x ^ (x >> 15)
        x = x * 0x2C1B3C6D
        x = x ^ (x >> 12)
        x = x * 0x297A2D39
        x = x ^ (x >> 15)
        img = (x & 255).to(torch.uint8).view(n, S, S, 3)
        lab = (ii.view(-1) * 2654435761 + self.seed) % self.num_classes
        return img, lab


class RecordsImageNet(ImageSource):
    """Raw uint8 records, memory-mapped; batches gathered by the native loader."""

    def __init__(self, root: str, split: str = "train", image_size: int = 224, num_classes: int = 1000,
                 threads: int = 8):
        self.path = os.path.join(root, f"{split}.u8")
        lab = os.path.join(root, f"{split}_labels.i64")
        self.labels = np.fromfile(lab, dtype=np.int64)
        self.num_examples = len(self.labels)
        self.image_size = image_size
        self.num_classes = num_classes
        self.row = image_size * image_size * 3
        sz = os.path.getsize(self.path)
        if sz != self.row * self.num_examples:
            raise ValueError(f"{self.path}: size {sz} != {self.num_examples} x {self.row}")
        self._loader = None
        self.threads = threads

    def _native(self):
        if self._loader is None:
            from ..ops.native import native_available, require_native
            if native_available() and hasattr(require_native(), "Loader"):
                self._loader = require_native().Loader(self.path, self.row, self.threads)
            else:
                self._loader = np.memmap(self.path, dtype=np.uint8, mode="r").reshape(self.num_examples, -1)
        return self._loader

    host = True

    def fetch_host(self, idx: np.ndarray):
        ld = self._native()
        S = self.image_size
        if isinstance(ld, np.memmap):
            buf = torch.from_numpy(np.ascontiguousarray(ld[idx]))
        else:
            buf = torch.empty((len(idx), self.row), dtype=torch.uint8, pin_memory=torch.cuda.is_available())
            ld.gather(torch.from_numpy(np.asarray(idx, dtype=np.int64)), buf)
        lab = torch.from_numpy(self.labels[idx])
        if torch.cuda.is_available():
            lab = lab.pin_memory()
        return buf.view(len(idx), S, S, 3), lab


class DecodedCache(ImageSource):
    """Decoded-image cache in front of a decoding source (tfds / folder): the reference's C6 map
    (imagenet-resnet50.py:36-41: cast + resize_with_crop_or_pad to 224, all augmentation is
    in-model) is deterministic per image, so its uint8 output can be kept.  The first time an
    example is fetched it is decoded by the wrapped source and written into a memory-mapped
    cache file (`<dir>/<split>-<S>.u8`, one S*S*3 row per example, plus `.i64` labels and a
    `.ok` byte per example, set after the row is written); afterwards it is gathered from the
    cache by the native loader thread pool into pinned memory, and the pipeline's prefetch
    stage copies it to the device asynchronously, like raw records.  Example order stays the
    pipeline's (a fresh permutation per epoch: the reference's shuffle_files=True).  Files are
    sized once (sparse) and may be shared by every rank of a job: ranks write disjoint
    examples, and a row is only read after its `.ok` byte."""
    host = True

    def __init__(self, inner: ImageSource, cache_dir: str, split: str, threads: int = 8):
        import json
        self.inner = inner
        self.num_examples = inner.num_examples
        self.image_size = inner.image_size
        self.num_classes = inner.num_classes
        S, N = self.image_size, self.num_examples
        self.row = S * S * 3
        os.makedirs(cache_dir, exist_ok=True)
        stem = os.path.join(cache_dir, f"{split}-{S}")
        meta = {"examples": N, "image_size": S, "source": type(inner).__name__,
                "files": len(getattr(inner, "files", []) or [])}
        mpath = stem + ".json"
        if os.path.exists(mpath):
            old = json.load(open(mpath))
            if old != meta:
                raise ValueError(f"decoded cache {stem}: made for {old}, not {meta} (use another --cache dir)")
        else:
            tmp = f"{mpath}.{os.getpid()}"
            with open(tmp, "w") as f:
                json.dump(meta, f)
            os.replace(tmp, mpath)
        self.paths = (stem + ".u8", stem + ".i64", stem + ".ok")
        for path, nbytes in zip(self.paths, (N * self.row, N * 8, N)):
            fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o644)
            try:
                if os.fstat(fd).st_size != nbytes:
                    os.ftruncate(fd, nbytes)       # (sparse; same size again keeps the contents)
            finally:
                os.close(fd)
        self.img = np.memmap(self.paths[0], dtype=np.uint8, mode="r+", shape=(N, self.row))
        self.labels = np.memmap(self.paths[1], dtype=np.int64, mode="r+", shape=(N,))
        self.ok = np.memmap(self.paths[2], dtype=np.uint8, mode="r+", shape=(N,))
        self.threads = threads
        self._loader = None
        self.hits = 0
        self.misses = 0

    def _gather(self, idx: np.ndarray, out: torch.Tensor):
        if self._loader is None:
            from ..ops.native import native_available, require_native
            self._loader = (require_native().Loader(self.paths[0], self.row, self.threads)
                            if native_available() and hasattr(require_native(), "Loader") else False)
        if self._loader:
            self._loader.gather(torch.from_numpy(np.ascontiguousarray(idx, dtype=np.int64)), out)
        else:
            out.copy_(torch.from_numpy(np.ascontiguousarray(self.img[idx])))

    def fetch_host(self, idx: np.ndarray):
        idx = np.asarray(idx, dtype=np.int64)
        n, S = len(idx), self.image_size
        hit = self.ok[idx] == 1
        buf = torch.empty((n, self.row), dtype=torch.uint8, pin_memory=torch.cuda.is_available())
        lab = torch.from_numpy(np.asarray(self.labels[idx]).copy())
        if not hit.all():
            miss = np.nonzero(~hit)[0]
            im_m, lab_m = self.inner.fetch_host(idx[miss])
            rows = im_m.reshape(len(miss), self.row)
            buf[torch.from_numpy(miss)] = rows
            lab[torch.from_numpy(miss)] = lab_m.to(torch.int64)
            self.img[idx[miss]] = rows.numpy()
            self.labels[idx[miss]] = lab_m.numpy().astype(np.int64)
            self.ok[idx[miss]] = 1               # (after the row: a reader never sees half a row)
            self.misses += len(miss)
        if hit.any():
            h = np.nonzero(hit)[0]
            if len(h) == n:
                self._gather(idx, buf)
            else:
                part = torch.empty((len(h), self.row), dtype=torch.uint8)
                self._gather(idx[h], part)
                buf[torch.from_numpy(h)] = part
            self.hits += len(h)
        if torch.cuda.is_available():
            lab = lab.pin_memory()
        return buf.view(n, S, S, 3), lab

    def flush(self):
        for m in (self.img, self.labels, self.ok):
            m.flush()


def write_records(root: str, split: str, images: np.ndarray, labels: np.ndarray) -> None:
    """Write a RecordsImageNet split (images uint8 [N,S,S,3], labels int)."""
    os.makedirs(root, exist_ok=True)
    np.ascontiguousarray(images, dtype=np.uint8).tofile(os.path.join(root, f"{split}.u8"))
    np.asarray(labels, dtype=np.int64).tofile(os.path.join(root, f"{split}_labels.i64"))


@dataclass
class Pipeline:
    """batch -> shard -> (repeat) iterator over an ImageSource, tf.data style.

    shard_by="batch"  : Horovod semantics, batch(B) then shard(num_shards, index)
    shard_by="element": MWMS AutoShardPolicy.DATA, shard elements then batch(B)
    """
    source: ImageSource
    batch_size: int
    num_shards: int = 1
    shard_index: int = 0
    shard_by: str = "batch"
    drop_remainder: bool = True
    repeat: bool = False
    shuffle: bool = False
    seed: int = 0

    def num_batches(self) -> int:
        n = self.source.num_examples
        if self.shard_by == "element":
            n_local = len(range(self.shard_index, n, self.num_shards))
            return n_local // self.batch_size if self.drop_remainder else math.ceil(n_local / self.batch_size)
        nb = n // self.batch_size if self.drop_remainder else math.ceil(n / self.batch_size)
        return len(range(self.shard_index, nb, self.num_shards))

    def _order(self, epoch: int) -> np.ndarray:
        n = self.source.num_examples
        if self.shuffle:
            return np.random.default_rng(self.seed + epoch).permutation(n)
        return np.arange(n)

    def batches(self, epoch: int = 0) -> Iterator[np.ndarray]:
        while True:
            order = self._order(epoch)
            B = self.batch_size
            if self.shard_by == "element":
                local = order[self.shard_index::self.num_shards]
                nb = len(local) // B if self.drop_remainder else math.ceil(len(local) / B)
                for i in range(nb):
                    yield local[i * B:(i + 1) * B]
            else:
                nb = len(order) // B if self.drop_remainder else math.ceil(len(order) / B)
                for i in range(self.shard_index, nb, self.num_shards):
                    yield order[i * B:(i + 1) * B]
            if not self.repeat:
                return
            epoch += 1

    def iterate(self, device, epoch: int = 0, prefetch: int = 3):
        """Yields (images, labels) on `device`, tf.data `prefetch` semantics.

        Host sources: a producer thread decodes / gathers up to `prefetch` batches ahead of the
        consumer into pinned memory (native code, GIL released), and the host->device copy of
        batch i+1 is issued on a side stream before batch i is handed out; the consumer's
        stream waits on the copy's event (stream-ordered, the training thread never decodes
        nor blocks on a copy).  Device sources (synthetic) generate on the GPU in order."""
        if getattr(self.source, "host", False):
            yield from _PrefetchIter(self, torch.device(device), epoch, max(1, prefetch))
            return
        it = self.batches(epoch)
        pending = []
        for idx in it:
            pending.append(self.source.fetch(idx, device))
            if len(pending) > prefetch:
                yield pending.pop(0)
        while pending:
            yield pending.pop(0)


class _PrefetchIter:
    """Producer thread (host decode k batches ahead) + async H2D one batch ahead."""

    _END = object()

    def __init__(self, pipe: "Pipeline", device: torch.device, epoch: int, depth: int):
        import queue
        import threading
        self.q = queue.Queue(maxsize=depth)
        self.stop = threading.Event()
        self.device = device
        self.cuda = device.type == "cuda"
        self.copy_stream = torch.cuda.Stream(device=device) if self.cuda else None
        self.th = threading.Thread(target=self._produce, args=(pipe, epoch), daemon=True,
                                   name="pddl-prefetch")
        self.th.start()

    def _put(self, item) -> bool:
        import queue
        while not self.stop.is_set():
            try:
                self.q.put(item, timeout=0.1)
                return True
            except queue.Full:
                continue
        return False

    def _produce(self, pipe, epoch):
        try:
            for idx in pipe.batches(epoch):
                if self.stop.is_set() or not self._put(pipe.source.fetch_host(idx)):
                    return
            self._put(self._END)
        except BaseException as e:   # surfaced on the consumer thread
            self._put(e)

    def _to_device(self, hb):
        img, lab = hb
        if not self.cuda:
            return img, lab, None
        with torch.cuda.stream(self.copy_stream):
            di = img.to(self.device, non_blocking=True)
            dl = lab.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
        return di, dl, ev

    def _hand_out(self, item):
        di, dl, ev = item
        if ev is not None:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            di.record_stream(cur)     # the copy stream's allocation is used on the compute stream
            dl.record_stream(cur)
        return di, dl

    def __iter__(self):
        pending = None
        try:
            while True:
                item = self.q.get()
                if item is self._END:
                    break
                if isinstance(item, BaseException):
                    raise item
                nxt = self._to_device(item)       # batch i+1's copy starts before batch i is used
                if pending is not None:
                    yield self._hand_out(pending)
                pending = nxt
            if pending is not None:
                yield self._hand_out(pending)
        finally:
            self.stop.set()
            while not self.q.empty():
                try:
                    self.q.get_nowait()
                except Exception:
                    break
            self.th.join(timeout=5)


def make_source(spec: str, split: str, cfg) -> ImageSource:
    if spec == "synthetic" or spec == "synthetic_fixed":
        n = cfg.train_images if split == "train" else cfg.val_images
        return SyntheticImageNet(n, cfg.image_size, cfg.num_classes, seed=cfg.seed + (0 if split == "train" else 1),
                                 fixed=spec == "synthetic_fixed")
    if spec.startswith("records:"):
        return RecordsImageNet(spec.split(":", 1)[1], split, cfg.image_size, cfg.num_classes)
    cache = getattr(cfg, "data_cache", None)
    if spec.startswith("tfds:"):
        from .imagenet import TFDSImageNet
        src = TFDSImageNet(spec.split(":", 1)[1], split, cfg.image_size, cfg.num_classes)
        return DecodedCache(src, cache, split) if cache else src
    if spec.startswith("folder:"):
        from .imagenet import JpegFolderImageNet
        src = JpegFolderImageNet(spec.split(":", 1)[1], split, cfg.image_size, cfg.num_classes)
        return DecodedCache(src, cache, split) if cache else src
    raise ValueError(f"unknown data spec {spec!r} (synthetic | records:<dir> | tfds:<dir> | folder:<dir>)")
