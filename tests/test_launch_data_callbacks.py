"""Launch resolution, tf.data-style sharding, Keras/Horovod callback semantics (CPU)."""
import argparse

import numpy as np
import pytest
import torch


# ------------------------------------------------------------------ launch
def test_hostlist_and_tasks_expansion():
    from pddl.parallel.launch import expand_hostlist, expand_tasks_per_node
    assert expand_hostlist("n[01-03,07],gpu5") == ["n01", "n02", "n03", "n07", "gpu5"]
    assert expand_hostlist("node1") == ["node1"]
    assert expand_tasks_per_node("2(x3),1") == [2, 2, 2, 1]


def test_slurm_resolver_port_base():
    from pddl.parallel.launch import SlurmClusterResolver
    env = {"SLURM_PROCID": "3", "SLURM_NTASKS": "4", "SLURM_STEP_NUM_TASKS": "4",
           "SLURM_STEP_NODELIST": "g[1-2]", "SLURM_STEP_TASKS_PER_NODE": "2(x2)", "SLURM_LOCALID": "1",
           "SLURM_NODEID": "1"}
    info = SlurmClusterResolver(12345, env).resolve()
    assert (info.rank, info.world_size, info.local_rank, info.local_world_size) == (3, 4, 1, 2)
    assert info.task_addresses == ["g1:12345", "g1:12346", "g2:12345", "g2:12346"]
    assert info.master_addr == "g1" and info.master_port == 12345


def test_resolve_cluster_sources():
    from pddl.parallel.launch import resolve_cluster
    i = resolve_cluster({"RANK": "2", "WORLD_SIZE": "8", "LOCAL_RANK": "2", "MASTER_PORT": "29511"})
    assert (i.source, i.rank, i.world_size, i.local_rank, i.master_port) == ("torchrun", 2, 8, 2, 29511)
    i = resolve_cluster({"OMPI_COMM_WORLD_RANK": "1", "OMPI_COMM_WORLD_SIZE": "2",
                         "OMPI_COMM_WORLD_LOCAL_RANK": "1"})
    assert (i.source, i.rank, i.world_size) == ("mpi", 1, 2)
    i = resolve_cluster({})
    assert (i.source, i.world_size, i.master_addr) == ("single", 1, "127.0.0.1")


def test_ps_cli_q6_forms():
    from pddl.parallel.parameter_server import add_ps_args, parse_ps_counts
    ap = argparse.ArgumentParser()
    add_ps_args(ap)
    assert parse_ps_counts(ap.parse_args(["--ps", "2", "--worker", "6"])) == (2, 6)
    assert parse_ps_counts(ap.parse_args(["2", "6"])) == (2, 6)
    assert parse_ps_counts(ap.parse_args([])) == (1, 1)


def test_in_process_cluster_spec():
    from pddl.parallel.launch import create_in_process_cluster
    spec = create_in_process_cluster(3, 2)
    assert len(spec["worker"]) == 3 and len(spec["ps"]) == 2
    assert len(set(spec["worker"] + spec["ps"])) == 5


def test_min_size_partitioner():
    from pddl.models.resnet50 import ParamLayout
    from pddl.parallel.parameter_server import min_size_partitions, partition_variables, ps_ranges
    assert min_size_partitions((2048, 1000), 4, 256 << 10, 2) == 2     # 8 MB -> max_shards
    assert min_size_partitions((64,), 4, 256 << 10, 2) == 1           # tiny -> 1 shard
    assert min_size_partitions((1, 1, 64, 256), 4, 256 << 10, 4) == 1  # axis-0 length 1
    L = ParamLayout()
    sh = partition_variables(L, 2)
    covered = sorted((s.offset, s.offset + s.size) for s in sh)
    tot = sum(e - s for s, e in covered)
    assert tot == L.count(True)
    for (s0, e0), (s1, e1) in zip(covered, covered[1:]):
        assert e0 <= s1
    r = ps_ranges(sh, 2)
    assert abs(sum(n for _, n in r[0]) - sum(n for _, n in r[1])) < 0.25 * L.count(True)


# ------------------------------------------------------------------ data
class _Src:
    num_examples = 23
    image_size = 4
    num_classes = 10

    def fetch(self, idx, device):
        idx = torch.as_tensor(np.asarray(idx))
        return idx.view(-1, 1, 1, 1).expand(-1, 4, 4, 3).to(torch.uint8), idx


def test_pipeline_horovod_shards_batches():
    from pddl.data.datasets import Pipeline
    p0 = Pipeline(_Src(), 4, num_shards=2, shard_index=0, shard_by="batch")
    p1 = Pipeline(_Src(), 4, num_shards=2, shard_index=1, shard_by="batch")
    b0 = [list(b) for b in p0.batches()]
    b1 = [list(b) for b in p1.batches()]
    assert b0 == [[0, 1, 2, 3], [8, 9, 10, 11], [16, 17, 18, 19]]
    assert b1 == [[4, 5, 6, 7], [12, 13, 14, 15]]
    assert p0.num_batches() == 3 and p1.num_batches() == 2


def test_pipeline_mwms_shards_elements():
    from pddl.data.datasets import Pipeline
    p = Pipeline(_Src(), 3, num_shards=2, shard_index=1, shard_by="element")
    assert [list(b) for b in p.batches()] == [[1, 3, 5], [7, 9, 11], [13, 15, 17], [19, 21, 23][:3]][:3]
    assert p.num_batches() == 3


def test_pipeline_repeat_and_iterate():
    from pddl.data.datasets import Pipeline
    p = Pipeline(_Src(), 10, repeat=True)
    it = p.batches()
    got = [next(it)[0] for _ in range(5)]
    assert got == [0, 10, 0, 10, 0]
    ims = list(Pipeline(_Src(), 5).iterate("cpu"))
    assert len(ims) == 4 and ims[0][0].shape == (5, 4, 4, 3)


def test_records_native_loader(tmp_path):
    from pddl.data.datasets import RecordsImageNet, write_records
    imgs = np.random.default_rng(0).integers(0, 256, (7, 8, 8, 3), dtype=np.uint8)
    write_records(str(tmp_path), "train", imgs, np.arange(7))
    src = RecordsImageNet(str(tmp_path), "train", image_size=8)
    im, lb = src.fetch(np.array([5, 1, 6]), "cpu")
    assert np.array_equal(im.numpy(), imgs[[5, 1, 6]]) and lb.tolist() == [5, 1, 6]
    from pddl.ops.native import native_available
    if native_available():
        assert type(src._loader).__name__ == "Loader"


def test_synthetic_is_deterministic():
    from pddl.data.datasets import SyntheticImageNet
    s = SyntheticImageNet(100, 16, 1000, seed=3)
    a, la = s.fetch(np.arange(4), "cpu")
    b, lb = s.fetch(np.arange(4), "cpu")
    assert torch.equal(a, b) and torch.equal(la, lb)


# ------------------------------------------------------------------ callbacks
class _T:
    def __init__(self):
        self.lr = 0.1
        self.stop_training = False
        self.steps_per_epoch = 10
        self.logs = []

    def set_lr(self, lr):
        self.lr = lr

    def log(self, m):
        self.logs.append(m)


def test_reduce_lr_on_plateau_keras_semantics():
    from pddl.train.callbacks import ReduceLROnPlateau
    t = _T()
    cb = ReduceLROnPlateau(monitor="val_loss", factor=0.1, patience=2, min_lr=1e-3)
    cb.set_trainer(t)
    cb.on_train_begin()
    for e, v in enumerate([1.0, 0.9, 0.9, 0.9, 0.9, 0.9, 0.9]):
        cb.on_epoch_end(e, {"val_loss": v})
    # improvement at e1; plateau e2,e3 -> reduce to 0.01 at e3; e4,e5 -> reduce to 1e-3 at e5
    assert abs(t.lr - 1e-3) < 1e-12


def test_early_stopping_min_delta():
    from pddl.train.callbacks import EarlyStopping
    t = _T()
    cb = EarlyStopping(monitor="val_loss", min_delta=0.001, patience=2)
    cb.set_trainer(t)
    cb.on_train_begin()
    for e, v in enumerate([1.0, 0.9995, 0.9993]):   # improvements smaller than min_delta
        cb.on_epoch_end(e, {"val_loss": v})
    assert t.stop_training and cb.stopped_epoch == 2


def test_horovod_lr_warmup_schedule():
    from pddl.train.callbacks import LearningRateWarmupCallback
    t = _T()
    size = 8
    cb = LearningRateWarmupCallback(0.1 * size, warmup_epochs=3, size=size)
    cb.set_trainer(t)
    cb.on_epoch_begin(0)
    cb.on_batch_begin(0)
    assert abs(t.lr - 0.1) < 1e-12                       # initial_lr / size
    cb.on_epoch_begin(1)
    cb.on_batch_begin(5)                                  # epoch 1.5
    assert abs(t.lr - 0.1 * (1.5 * 7 / 3 + 1)) < 1e-9
    cb.on_epoch_begin(3)
    t.lr = 0.8
    cb.on_batch_begin(0)
    assert t.lr == 0.8


def test_config_presets_reproduce_reference_constants():
    from pddl.config import make_config
    c = make_config("single")
    assert (c.batch_size, c.crop, c.optimizer, c.lr, c.epochs) == (32, 244, "adam", 1e-3, 50)
    assert c.checkpoint_name() == "ImageNet-ResNet50_ImageNet-reuse.h5"
    h = make_config("horovod")
    assert (h.crop, h.lr, h.lr_scale_by_size, h.warmup_epochs) == (160, 0.1, True, 3)
    assert h.checkpoint_name(8) == "ImageNet-ResNet50_ImageNet-8GPUs-reuse.h5"    # Q7 fixed
    w = make_config("multiworker")
    assert (w.batch_size, w.val_batch_size, w.shard_by, w.port_base) == (128, 256, "element", 12345)
    p = make_config("ps")
    assert (p.steps_per_epoch, p.min_shard_bytes) == (312500, 256 << 10)
    assert make_config("mirrored").checkpoint_name() == "ImageNet-ResNet50_ImageNet_mirror-reuse.h5"
    assert make_config("single_pretrained").weights == "imagenet"


def test_throughput_meter_times_training_steps_only():
    """img/s covers the epoch's training steps after the warm-up steps; the validation pass
    that follows (before on_epoch_end) is not timed."""
    import time
    from pddl.train.callbacks import ThroughputMeter
    t = _T()
    t.global_batch = 64
    t.sync = lambda: None
    cb = ThroughputMeter(skip=2)
    cb.set_trainer(t)
    cb.on_epoch_begin(0)
    for b in range(6):
        cb.on_batch_end(b)
        time.sleep(0.01)
    cb.on_train_batches_end(0)
    time.sleep(0.3)                                       # "validation"
    logs = {}
    cb.on_epoch_end(0, logs)
    # 4 timed steps of 64 images in ~0.04-0.05 s: far above what timing the 0.3 s pass would give
    assert logs["images_per_sec"] > 4 * 64 / 0.2, logs
