"""Convert ImageNet (tfds TFRecord shards or ILSVRC class folders) into the raw uint8 records
the mmap loader reads (`--data records:<out>`): decode + resize_with_crop_or_pad once, offline.

    python scripts/make_records.py tfds:/data/tensorflow_datasets /data/imagenet_u8 --split train
    python scripts/make_records.py folder:/data/ILSVRC2012 /data/imagenet_u8 --split val --limit 50000
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src", help="tfds:<dir> or folder:<dir>")
    ap.add_argument("out")
    ap.add_argument("--split", default="train")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--limit", type=int, default=0)
    ap.add_argument("--chunk", type=int, default=1024)
    args = ap.parse_args()
    import pddl  # noqa: F401
    from pddl.data.datasets import make_source

    class _Cfg:
        image_size = args.image_size
        num_classes = 1000
    src = make_source(args.src, args.split, _Cfg())
    n = src.num_examples if not args.limit else min(args.limit, src.num_examples)
    os.makedirs(args.out, exist_ok=True)
    split = "train" if args.split == "train" else "val"
    S = args.image_size
    img_path = os.path.join(args.out, f"{split}.u8")
    labels = np.empty(n, dtype=np.int64)
    with open(img_path, "wb") as f:
        for s in range(0, n, args.chunk):
            idx = np.arange(s, min(n, s + args.chunk))
            img, lab = src.fetch(idx, "cpu")
            f.write(img.numpy().reshape(len(idx), S * S * 3).tobytes())
            labels[s:s + len(idx)] = lab.numpy()
            print(f"{s + len(idx)}/{n}", flush=True)
    labels.tofile(os.path.join(args.out, f"{split}_labels.i64"))
    print(f"wrote {n} x {S}x{S}x3 records to {args.out}")


if __name__ == "__main__":
    main()
