"""Input-pipeline throughput: native JPEG decode per thread count, mmap records gather, and
whether a training step fed by the prefetching pipeline runs as fast as one fed by a
device-resident synthetic batch (the reference's map(AUTOTUNE) -> batch -> prefetch(AUTOTUNE),
imagenet-resnet50.py:44-49).

    python scripts/decode_bench.py --images 2048 --threads 1,2,4,8,16 --json gpurun_out/decode.json
    python scripts/decode_bench.py --train-steps 20 --batch 256          # + the GPU step comparison
    python scripts/decode_bench.py --train-steps 30 --batch 256 --crop 244 --cache-threads 8
        # + a decoded-image cache (data/datasets.py DecodedCache) warmed once, then fed to the step

Data: photo-like synthetic JPEGs (smooth gradients + noise, ImageNet-typical 500x375, quality 90)
written as tfds-style TFRecord shards into a temp dir (no dataset download is possible), then
converted to raw records for the mmap loader.
"""
import argparse
import io
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_jpegs(n, w, h, seed=0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    out = []
    for i in range(n):
        a, b, c = rng.uniform(0.2, 1.0, 3)
        base = np.stack([128 + 100 * np.sin(xx * a / 40 + i), 128 + 100 * np.cos(yy * b / 35),
                         128 + 80 * np.sin((xx + yy) * c / 50)], -1)
        img = (base + rng.normal(0, 12, base.shape)).clip(0, 255).astype(np.uint8)
        buf = io.BytesIO()
        Image.fromarray(img).save(buf, format="JPEG", quality=90)
        out.append(buf.getvalue())
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=2048)
    ap.add_argument("--size", default="500x375")
    ap.add_argument("--threads", default="1,2,4,8,16")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--train-steps", type=int, default=0, help="GPU: also compare step time vs synthetic")
    ap.add_argument("--crop", type=int, default=224, help="network input of the step comparison (244: the presets)")
    ap.add_argument("--cache-threads", type=int, default=0,
                    help="also feed the step from a warm decoded-image cache gathered by this many threads")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import torch
    import pddl  # noqa: F401
    from pddl.data.datasets import Pipeline, RecordsImageNet, write_records
    from pddl.data.imagenet import TFDSImageNet, write_tfrecord_imagenet
    rows = []

    def emit(r):
        rows.append(r)
        print(json.dumps(r), flush=True)

    w, h = (int(v) for v in a.size.split("x"))
    tmp = tempfile.mkdtemp(prefix="pddl_decode_")
    t0 = time.perf_counter()
    jp = make_jpegs(a.images, w, h)
    labels = np.arange(a.images) % 1000
    half = a.images // 2
    write_tfrecord_imagenet(os.path.join(tmp, "imagenet2012-train.tfrecord-00000-of-00002"), jp[:half], labels[:half])
    write_tfrecord_imagenet(os.path.join(tmp, "imagenet2012-train.tfrecord-00001-of-00002"), jp[half:], labels[half:])
    emit({"kind": "setup", "images": a.images, "jpeg_kib_avg": round(sum(map(len, jp)) / len(jp) / 1024, 1),
          "seconds": round(time.perf_counter() - t0, 1), "host_cpus": os.cpu_count()})
    B = a.batch
    n_b = a.images // B
    for t in [int(x) for x in a.threads.split(",")]:
        src = TFDSImageNet(tmp, "train", 224, threads=t)
        idx = np.arange(a.images)
        src.fetch_host(idx[:B])                      # warm the page cache / pools
        t0 = time.perf_counter()
        for i in range(n_b):
            src.fetch_host(idx[i * B:(i + 1) * B])
        dt = time.perf_counter() - t0
        emit({"kind": "jpeg_decode", "threads": t, "images_per_sec": round(n_b * B / dt, 1)})
    # raw records (decoded + resized once, offline: scripts/make_records.py)
    src = TFDSImageNet(tmp, "train", 224, threads=max(int(x) for x in a.threads.split(",")))
    recdir = os.path.join(tmp, "records")
    imgs, labs = src.fetch_host(np.arange(a.images))
    write_records(recdir, "train", imgs.numpy(), labs.numpy())
    del imgs
    rec = RecordsImageNet(recdir, "train", 224)
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    for name, s in (("records", rec), ("jpeg", src)):
        p = Pipeline(s, B, shuffle=True, seed=1)
        t0 = time.perf_counter()
        n = 0
        for im, lb in p.iterate(dev):
            n += im.shape[0]
        if dev.type == "cuda":
            torch.cuda.synchronize()
        emit({"kind": "pipeline", "source": name, "device": dev.type,
              "images_per_sec": round(n / (time.perf_counter() - t0), 1)})
    if a.train_steps and dev.type == "cuda":
        from pddl.config import make_config
        from pddl.parallel.strategies import make_strategy
        from pddl.train.trainer import Trainer
        cfg = make_config("single", device="cuda", batch_size=B, crop=a.crop, image_size=224, save=False, verbose=0,
                          data=f"records:{recdir}", train_images=a.images)
        st = make_strategy(cfg)
        Trainer(cfg, st)
        syn = (torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device="cuda"),
               torch.randint(0, 1000, (B,), device="cuda"))

        def run(feed):
            for _ in range(3):
                st.train_step(*next(feed))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.train_steps):
                st.train_step(*next(feed))
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / a.train_steps * 1e3

        def synthetic():
            while True:
                yield syn

        def records():
            ep = 0
            while True:
                for b in st.train_pipeline().iterate(st.device, epoch=ep):
                    yield b
                ep += 1
        ms_syn = run(synthetic())
        ms_rec = run(records())
        row = {"kind": "train_step", "batch": B, "crop": a.crop, "synthetic_ms": round(ms_syn, 2),
               "records_ms": round(ms_rec, 2), "ratio": round(ms_rec / ms_syn, 3)}
        if a.cache_threads:
            from pddl.data.datasets import DecodedCache
            cache = DecodedCache(TFDSImageNet(tmp, "train", 224, threads=a.cache_threads),
                                 os.path.join(tmp, "cache"), "train", threads=a.cache_threads)
            t0 = time.perf_counter()
            for i in range(n_b):                          # first epoch: decode + write the cache
                cache.fetch_host(np.arange(i * B, (i + 1) * B))
            row["cache_fill_images_per_sec"] = round(n_b * B / (time.perf_counter() - t0), 1)

            def cached():
                ep = 0
                while True:
                    for b in Pipeline(cache, B, shuffle=True, seed=5).iterate(st.device, epoch=ep):
                        yield b
                    ep += 1
            ms_c = run(cached())
            row.update(cache_ms=round(ms_c, 2), cache_ratio=round(ms_c / ms_syn, 3), cache_threads=a.cache_threads,
                       cache_hits=cache.hits, cache_misses=cache.misses)
        emit(row)
    if a.json:
        json.dump(rows, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
