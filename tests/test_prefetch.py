"""The input pipeline's prefetch stage (C7 batch->prefetch, N12 tf.data runtime): host sources
are decoded / gathered by a producer thread k batches ahead of the training thread, in order,
with errors surfaced to the consumer and no thread left behind when the consumer stops early."""
import threading
import time

import numpy as np
import pytest
import torch

from pddl.data.datasets import ImageSource, Pipeline, RecordsImageNet, write_records


class SlowHost(ImageSource):
    """Host source whose load takes `delay` s (sleep releases the GIL like the native decoders)."""
    host = True

    def __init__(self, n=64, delay=0.0, fail_at=None):
        self.num_examples, self.image_size, self.num_classes = n, 4, 10
        self.delay, self.fail_at, self.calls = delay, fail_at, 0
        self.threads = set()

    def fetch_host(self, idx):
        self.calls += 1
        self.threads.add(threading.current_thread().name)
        if self.fail_at is not None and self.calls > self.fail_at:
            raise ValueError("corrupt record")
        time.sleep(self.delay)
        img = torch.tensor(idx, dtype=torch.uint8).view(-1, 1, 1, 1).expand(-1, 4, 4, 3).contiguous()
        return img, torch.tensor(idx, dtype=torch.int64)


def test_prefetch_order_and_content_match_sync(tmp_path):
    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, (40, 8, 8, 3), dtype=np.uint8)
    write_records(str(tmp_path), "train", imgs, np.arange(40) % 7)
    src = RecordsImageNet(str(tmp_path), "train", image_size=8, num_classes=7)
    p = Pipeline(src, 6, shuffle=True, seed=3)
    got = list(p.iterate("cpu", epoch=1))
    want = [src.fetch(idx, "cpu") for idx in p.batches(1)]
    assert len(got) == len(want) == 40 // 6
    for (a, la), (b, lb) in zip(got, want):
        assert torch.equal(a, b) and torch.equal(la, lb)


def test_prefetch_runs_ahead_on_its_own_thread():
    src = SlowHost(n=64, delay=0.05)
    p = Pipeline(src, 8)                                    # 8 batches of 50 ms loading
    t0 = time.perf_counter()
    n = 0
    for im, lb in p.iterate("cpu", prefetch=3):
        time.sleep(0.05)                                    # 50 ms of "training" per batch
        n += 1
    dt = time.perf_counter() - t0
    assert n == 8
    assert dt < 0.65, dt                                    # overlapped: ~0.45 s, serial would be 0.8 s
    assert src.threads == {"pddl-prefetch"}                 # never decoded on the training thread


def test_prefetch_surfaces_errors_and_stops_cleanly():
    p = Pipeline(SlowHost(n=64, fail_at=2), 8)
    it = p.iterate("cpu")
    with pytest.raises(ValueError, match="corrupt"):
        for _ in it:
            pass
    before = {t.name for t in threading.enumerate()}
    p2 = Pipeline(SlowHost(n=640, delay=0.01), 8)
    for i, _ in enumerate(p2.iterate("cpu")):
        if i == 2:
            break                                           # consumer stops early
    time.sleep(0.3)
    alive = [t for t in threading.enumerate() if t.name == "pddl-prefetch"]
    assert not alive, alive
    assert "pddl-prefetch" not in before
