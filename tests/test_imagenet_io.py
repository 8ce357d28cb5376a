"""Native ImageNet reader (csrc/io/imagenet_io.cpp): tfds TFRecord framing + tf.Example parsing
+ libjpeg decode + tf.image.resize_with_crop_or_pad (reference imagenet-resnet50.py:28-41),
checked against PIL decoding of the same JPEG bytes and a NumPy resize_with_crop_or_pad."""
import io
import os

import numpy as np
import pytest
import torch

PIL = pytest.importorskip("PIL.Image")


def _jpeg(arr, mode="RGB", quality=92):
    from PIL import Image
    im = Image.fromarray(arr, mode=mode) if mode != "CMYK" else Image.fromarray(arr, mode="RGB").convert("CMYK")
    b = io.BytesIO()
    im.save(b, format="JPEG", quality=quality)
    return b.getvalue()


def _pil_rgb(jb):
    from PIL import Image
    return np.asarray(Image.open(io.BytesIO(jb)).convert("RGB"))


def _images(rng):
    sizes = [(300, 260), (180, 400), (224, 224), (100, 150), (500, 375)]
    out = []
    # smooth, photo-like content: decoders (libjpeg 9 here, libjpeg-turbo in PIL / TF) differ
    # mostly in chroma upsampling at sharp colour edges, which natural images rarely have
    for h, w in sizes:
        y, x = np.mgrid[0:h, 0:w].astype(np.float32)
        ph = rng.uniform(0, 6.28, 3)
        arr = np.stack([127 + 100 * np.sin(x / (17 + 9 * c) + y / (23 + 5 * c) + ph[c]) for c in range(3)], -1)
        arr += rng.normal(0, 3, arr.shape)
        out.append(_jpeg(np.ascontiguousarray(arr.clip(0, 255).astype(np.uint8))))
    y, x = np.mgrid[0:250, 0:300].astype(np.float32)
    gray = (127 + 120 * np.cos(x / 31) * np.sin(y / 19)).astype(np.uint8)
    out.append(_jpeg(np.ascontiguousarray(gray), mode="L"))
    return out


def test_tfrecord_reader_matches_pil(tmp_path):
    from pddl.data.imagenet import TFDSImageNet, resize_with_crop_or_pad, write_tfrecord_imagenet
    rng = np.random.default_rng(0)
    jpegs = _images(rng)
    labels = [3, 999, 0, 17, 512, 7]
    d = tmp_path / "imagenet2012" / "5.1.0"
    d.mkdir(parents=True)
    write_tfrecord_imagenet(str(d / "imagenet2012-train.tfrecord-00000-of-00002"), jpegs[:4], labels[:4])
    write_tfrecord_imagenet(str(d / "imagenet2012-train.tfrecord-00001-of-00002"), jpegs[4:], labels[4:])
    src = TFDSImageNet(str(tmp_path), "train", image_size=224, threads=3)
    assert src.num_examples == 6
    idx = np.array([5, 0, 3, 1, 4, 2])
    img, lab = src.fetch(idx, "cpu")
    assert lab.tolist() == [labels[i] for i in idx]
    for k, i in enumerate(idx):
        want = resize_with_crop_or_pad(_pil_rgb(jpegs[i]), 224).astype(np.int16)
        got = img[k].numpy().astype(np.int16)
        assert np.abs(got - want).mean() < 1.5, (i, np.abs(got - want).mean())
        pad_rows = want.sum(axis=(1, 2)) == 0
        assert (got[pad_rows] == 0).all()            # zero padding exactly where TF pads


def test_tfrecord_crc_detects_corruption(tmp_path):
    from pddl.data.imagenet import TFDSImageNet, write_tfrecord_imagenet
    rng = np.random.default_rng(1)
    path = tmp_path / "x-train.tfrecord-00000-of-00001"
    write_tfrecord_imagenet(str(path), _images(rng)[:2], [1, 2])
    raw = bytearray(path.read_bytes())
    raw[40] ^= 0xFF                                   # flip a byte inside the first record's data
    path.write_bytes(bytes(raw))
    src = TFDSImageNet(str(tmp_path), "train", image_size=64)
    with pytest.raises(RuntimeError, match="corrupt"):
        src.fetch(np.array([0]), "cpu")
    img, lab = src.fetch(np.array([1]), "cpu")        # the intact record still reads
    assert lab.tolist() == [2]


def test_folder_reader_and_pipeline(tmp_path):
    from pddl.data.datasets import Pipeline
    from pddl.data.imagenet import JpegFolderImageNet, resize_with_crop_or_pad
    rng = np.random.default_rng(2)
    jpegs = _images(rng)
    for ci, syn in enumerate(["n01440764", "n01443537"]):
        os.makedirs(tmp_path / "train" / syn)
        for j in range(3):
            (tmp_path / "train" / syn / f"img{j}.JPEG").write_bytes(jpegs[ci * 3 + j])
    src = JpegFolderImageNet(str(tmp_path), "train", image_size=96, threads=2)
    assert src.num_examples == 6 and src.classes == ["n01440764", "n01443537"]
    pipe = Pipeline(src, 2, num_shards=2, shard_index=1, shard_by="element")
    batches = list(pipe.iterate("cpu"))
    assert len(batches) == 1
    img, lab = batches[0]
    assert img.shape == (2, 96, 96, 3) and img.dtype == torch.uint8
    # element shard 1 of 2 = examples 1, 3 -> class 0, class 1
    assert lab.tolist() == [0, 1]
    want = resize_with_crop_or_pad(_pil_rgb(jpegs[1]), 96).astype(np.int16)
    assert np.abs(img[0].numpy().astype(np.int16) - want).mean() < 1.5


def test_decoded_cache_is_bitwise_the_decoded_batches(tmp_path):
    """--cache <dir>: the first fetch of an example decodes it (native reader + C6 crop-or-pad)
    and writes it to the memory-mapped cache; later fetches gather it from the cache.  Cached,
    half-cached and decoded batches are bitwise equal, labels included, and a second cache object
    on the same directory (another rank / a later run) starts warm."""
    from pddl.config import make_config
    from pddl.data.datasets import DecodedCache, Pipeline, make_source
    from pddl.data.imagenet import TFDSImageNet, write_tfrecord_imagenet
    rng = np.random.default_rng(1)
    jpegs = _images(rng) * 2
    labels = list(range(100, 100 + len(jpegs)))
    d = tmp_path / "tfds"
    d.mkdir()
    write_tfrecord_imagenet(str(d / "imagenet2012-train.tfrecord-00000-of-00001"), jpegs, labels)
    ref = TFDSImageNet(str(d), "train", image_size=224, threads=2)
    cfg = make_config("single", data=f"tfds:{d}", image_size=224, crop=224, device="cpu")
    cfg = cfg.replace(data_cache=str(tmp_path / "cache"))
    src = make_source(cfg.data, "train", cfg)
    assert isinstance(src, DecodedCache) and src.num_examples == len(jpegs)
    want_i, want_l = ref.fetch_host(np.arange(len(jpegs)))
    a = np.array([3, 1, 7])
    i1, l1 = src.fetch_host(a)                         # all misses: decode + write
    assert src.misses == 3 and src.hits == 0
    assert torch.equal(i1, want_i[a]) and torch.equal(l1, want_l[a])
    b = np.array([7, 0, 3, 11])                        # mixed: 2 hits, 2 misses
    i2, l2 = src.fetch_host(b)
    assert src.hits == 2 and src.misses == 5
    assert torch.equal(i2, want_i[b]) and torch.equal(l2, want_l[b])
    src.flush()
    warm = DecodedCache(TFDSImageNet(str(d), "train", image_size=224, threads=2), str(tmp_path / "cache"), "train")
    i3, l3 = warm.fetch_host(b)                        # all hits, gathered by the native loader
    assert warm.hits == 4 and warm.misses == 0
    assert torch.equal(i3, want_i[b]) and torch.equal(l3, want_l[b])
    # through the prefetching pipeline: two epochs, identical batches whatever the cache state
    p = Pipeline(src, 4, shuffle=True, seed=3)
    for ep in range(2):
        for (im, lb), idx in zip(p.iterate("cpu", epoch=ep), p.batches(ep)):
            assert torch.equal(im, want_i[idx]) and torch.equal(lb, want_l[idx])
    assert src.ok.all()
