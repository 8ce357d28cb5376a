"""Keras-layout HDF5 checkpoints through the native `_pddl_h5` module.

Reference: `model.save('ImageNet-' + model.name + '-reuse.h5')` at the end of every script
(imagenet-resnet50.py:69-72; Horovod rank-0 only, imagenet-resnet50-hvd.py:125-129) writes
the Keras HDF5 full-model format:
  /                      attrs keras_version, backend, model_config (JSON), training_config
  /model_weights         attrs layer_names, backend, keras_version
  /model_weights/<layer> attr weight_names; datasets <layer>/<weight name>, e.g.
                         model_weights/resnet50/conv1_conv/kernel:0 (HWIO), .../conv1_bn/gamma:0
  /optimizer_weights     attr weight_names: Adam/iter:0, Adam/<var>/m:0 ..., Adam/<var>/v:0 ...
`weights='imagenet'` (imagenet-pretrained-resnet50.py:56) loads Keras'
resnet50_weights_tf_dim_ordering_tf_kernels_notop.h5 (weights-only layout: root layer_names);
with no network it must already be on disk (~/.keras/models or PDDL_KERAS_WEIGHTS).
Extra, additive: `--resume` restores parameters, BN statistics and optimizer slots.
"""
from __future__ import annotations

import glob
import importlib.machinery
import importlib.util
import json
import os
from typing import Dict, List, Optional

import numpy as np
import torch

from ..models.resnet50 import BN_EPS, BN_MOMENTUM, ParamLayout

KERAS_VERSION = "2.8.0"
_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_h5 = None


def h5():
    global _h5
    if _h5 is None:
        import torch  # noqa: F401  (libc10 first)
        cands = sorted(glob.glob(os.path.join(_PKG, "_pddl_h5*.so")))
        if not cands:
            raise RuntimeError("native HDF5 module _pddl_h5 not built (run `python pddl_build.py`)")
        loader = importlib.machinery.ExtensionFileLoader("_pddl_h5", cands[-1])
        spec = importlib.util.spec_from_file_location("_pddl_h5", cands[-1], loader=loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        _h5 = mod
    return _h5


# ------------------------------------------------------------------ Keras layer order
def keras_resnet50_layers(L: ParamLayout) -> List[dict]:
    """Layer list of keras.applications.ResNet50(include_top=False, pooling='avg') in the
    Keras functional order, with configs and inbound nodes (model_config)."""
    layers = []

    def add(cls, name, cfg, inbound):
        layers.append({"class_name": cls, "config": dict(name=name, trainable=True, dtype="float32", **cfg),
                       "name": name, "inbound_nodes": [[[i, 0, 0, {}] for i in inbound]] if inbound else []})

    def conv_cfg(c):
        return dict(filters=c.cout, kernel_size=[c.k, c.k], strides=[c.stride, c.stride],
                    padding="same" if c.k == 3 else "valid", data_format="channels_last", dilation_rate=[1, 1],
                    groups=1, activation="linear", use_bias=True,
                    kernel_initializer={"class_name": "GlorotUniform", "config": {"seed": None}},
                    bias_initializer={"class_name": "Zeros", "config": {}}, kernel_regularizer=None,
                    bias_regularizer=None, activity_regularizer=None, kernel_constraint=None, bias_constraint=None)

    bn_cfg = dict(axis=[3], momentum=BN_MOMENTUM, epsilon=BN_EPS, center=True, scale=True,
                  beta_initializer={"class_name": "Zeros", "config": {}},
                  gamma_initializer={"class_name": "Ones", "config": {}},
                  moving_mean_initializer={"class_name": "Zeros", "config": {}},
                  moving_variance_initializer={"class_name": "Ones", "config": {}},
                  beta_regularizer=None, gamma_regularizer=None, beta_constraint=None, gamma_constraint=None)
    layers.append({"class_name": "InputLayer", "config": {"batch_input_shape": [None, None, None, 3],
                                                            "dtype": "float32", "sparse": False, "ragged": False,
                                                            "name": "input_2"}, "name": "input_2",
                   "inbound_nodes": []})
    add("ZeroPadding2D", "conv1_pad", dict(padding=[[3, 3], [3, 3]], data_format="channels_last"), ["input_2"])
    add("Conv2D", "conv1_conv", conv_cfg(L.stem), ["conv1_pad"])
    add("BatchNormalization", "conv1_bn", bn_cfg, ["conv1_conv"])
    add("Activation", "conv1_relu", dict(activation="relu"), ["conv1_bn"])
    add("ZeroPadding2D", "pool1_pad", dict(padding=[[1, 1], [1, 1]], data_format="channels_last"), ["conv1_relu"])
    add("MaxPooling2D", "pool1_pool", dict(pool_size=[3, 3], padding="valid", strides=[2, 2],
                                           data_format="channels_last"), ["pool1_pad"])
    prev = "pool1_pool"
    for b in L.blocks:
        n = b.name
        c = b.convs
        add("Conv2D", f"{n}_1_conv", conv_cfg(c["1"]), [prev])
        add("BatchNormalization", f"{n}_1_bn", bn_cfg, [f"{n}_1_conv"])
        add("Activation", f"{n}_1_relu", dict(activation="relu"), [f"{n}_1_bn"])
        add("Conv2D", f"{n}_2_conv", conv_cfg(c["2"]), [f"{n}_1_relu"])
        add("BatchNormalization", f"{n}_2_bn", bn_cfg, [f"{n}_2_conv"])
        add("Activation", f"{n}_2_relu", dict(activation="relu"), [f"{n}_2_bn"])
        if b.proj:
            add("Conv2D", f"{n}_0_conv", conv_cfg(c["0"]), [prev])
        add("Conv2D", f"{n}_3_conv", conv_cfg(c["3"]), [f"{n}_2_relu"])
        if b.proj:
            add("BatchNormalization", f"{n}_0_bn", bn_cfg, [f"{n}_0_conv"])
        add("BatchNormalization", f"{n}_3_bn", bn_cfg, [f"{n}_3_conv"])
        add("Add", f"{n}_add", {}, [f"{n}_0_bn" if b.proj else prev, f"{n}_3_bn"])
        add("Activation", f"{n}_out", dict(activation="relu"), [f"{n}_add"])
        prev = f"{n}_out"
    add("GlobalAveragePooling2D", "avg_pool", dict(data_format="channels_last", keepdims=False), [prev])
    return layers


def keras_weight_names(L: ParamLayout, layer_order: List[dict]) -> List[str]:
    names = []
    for ly in layer_order:
        nm = ly["name"]
        if ly["class_name"] == "Conv2D":
            names += [f"{nm}/kernel:0", f"{nm}/bias:0"]
        elif ly["class_name"] == "BatchNormalization":
            names += [f"{nm}/gamma:0", f"{nm}/beta:0", f"{nm}/moving_mean:0", f"{nm}/moving_variance:0"]
    return names


def model_config(L: ParamLayout, cfg) -> dict:
    inner = keras_resnet50_layers(L)
    resnet = {"class_name": "Functional", "config": {"name": "resnet50", "layers": inner,
                                                     "input_layers": [["input_2", 0, 0]],
                                                     "output_layers": [["avg_pool", 0, 0]]},
              "name": "resnet50", "inbound_nodes": [[["random_flip", 0, 0, {"training": False}]]]}
    S = cfg.image_size if cfg is not None else 224
    crop = cfg.crop if cfg is not None else 224
    outer = [
        {"class_name": "InputLayer", "config": {"batch_input_shape": [None, S, S, 3], "dtype": "float32",
                                                "sparse": False, "ragged": False, "name": "input_1"},
         "name": "input_1", "inbound_nodes": []},
        {"class_name": "Rescaling", "config": {"name": "rescaling", "trainable": True, "dtype": "float32",
                                               "scale": 1.0 / 255, "offset": 0.0},
         "name": "rescaling", "inbound_nodes": [[["input_1", 0, 0, {}]]]},
        {"class_name": "RandomCrop", "config": {"name": "random_crop", "trainable": True, "dtype": "float32",
                                                "height": crop, "width": crop, "seed": None},
         "name": "random_crop", "inbound_nodes": [[["rescaling", 0, 0, {}]]]},
        {"class_name": "RandomFlip", "config": {"name": "random_flip", "trainable": True, "dtype": "float32",
                                                "mode": "horizontal", "seed": None},
         "name": "random_flip", "inbound_nodes": [[["random_crop", 0, 0, {}]]]},
        resnet,
        {"class_name": "Dense", "config": {"name": "dense", "trainable": True, "dtype": "float32",
                                           "units": L.num_classes, "activation": "softmax", "use_bias": True,
                                           "kernel_initializer": {"class_name": "GlorotUniform",
                                                                  "config": {"seed": None}},
                                           "bias_initializer": {"class_name": "Zeros", "config": {}},
                                           "kernel_regularizer": None, "bias_regularizer": None,
                                           "activity_regularizer": None, "kernel_constraint": None,
                                           "bias_constraint": None},
         "name": "dense", "inbound_nodes": [[["resnet50", 1, 0, {}]]]},
    ]
    name = cfg.model_name if cfg is not None else "ResNet50_ImageNet"
    return {"class_name": "Functional", "config": {"name": name, "layers": outer,
                                                   "input_layers": [["input_1", 0, 0]],
                                                   "output_layers": [["dense", 0, 0]]},
            "keras_version": KERAS_VERSION, "backend": "tensorflow"}


# ------------------------------------------------------------------ tensor conversion
def _to_keras(e, t: torch.Tensor) -> np.ndarray:
    a = t.detach().float().cpu().view(e.shape)
    if e.kind == "kernel":
        a = a.permute(1, 2, 3, 0) if len(e.shape) == 4 else a.t()   # OHWI -> HWIO ; [out,in] -> [in,out]
    return np.ascontiguousarray(a.numpy().astype(np.float32))


def _from_keras(e, arr: np.ndarray) -> torch.Tensor:
    a = torch.from_numpy(np.asarray(arr, dtype=np.float32))
    if tuple(a.shape) != tuple(e.keras_shape):
        raise ValueError(f"{e.name}: shape {tuple(a.shape)} != Keras {e.keras_shape}")
    if e.kind == "kernel":
        a = a.permute(3, 0, 1, 2) if a.dim() == 4 else a.t()
    return a.contiguous().view(-1)


def save_keras_h5(path: str, engine, optimizer=None, cfg=None, progress: Optional[dict] = None) -> None:
    """Keras HDF5 full-model layout.  `progress` (additive, for --resume): completed epochs,
    current learning rate and LR/stop callback state, stored as the root attr `pddl_resume`
    (JSON; Keras ignores unknown root attributes)."""
    L: ParamLayout = engine.L
    params = engine.params.detach().cpu()
    inner = keras_resnet50_layers(L)
    wnames = keras_weight_names(L, inner)
    datasets, attrs = [], []
    outer_layers = ["input_1", "rescaling", "random_crop", "random_flip", "resnet50", "dense"]
    for wn in wnames:
        e = L.entries[wn]
        datasets.append((f"model_weights/resnet50/{wn}", _to_keras(e, params[e.offset:e.offset + e.size])))
    for wn in ("dense/kernel:0", "dense/bias:0"):
        e = L.entries[wn]
        datasets.append((f"model_weights/dense/{wn}", _to_keras(e, params[e.offset:e.offset + e.size])))
    attrs += [("", "backend", "tensorflow"), ("", "keras_version", KERAS_VERSION),
              ("", "model_config", json.dumps(model_config(L, cfg)))]
    attrs += [("model_weights", "layer_names", outer_layers), ("model_weights", "backend", "tensorflow"),
              ("model_weights", "keras_version", KERAS_VERSION)]
    for ln in outer_layers:
        w = wnames if ln == "resnet50" else (["dense/kernel:0", "dense/bias:0"] if ln == "dense" else [])
        attrs.append((f"model_weights/{ln}", "weight_names", w))
    if optimizer is not None:
        oname = "Adam" if type(optimizer).__name__ == "Adam" else "SGD"
        train_vars = [wn for wn in wnames if L.entries[wn].trainable] + ["dense/kernel:0", "dense/bias:0"]
        onames = [f"{oname}/iter:0"]
        datasets.append((f"optimizer_weights/{oname}/iter:0", np.array(optimizer.iterations, dtype=np.int64)))
        st = {k: v.detach().cpu() for k, v in optimizer.state_tensors().items()}
        slot_names = {"m": "m", "v": "v", "momentum": "momentum"}
        for sk in st:
            for wn in train_vars:
                e = L.entries[wn]
                nm = f"{oname}/{wn[:-2]}/{slot_names[sk]}:0"
                onames.append(nm)
                datasets.append((f"optimizer_weights/{nm}", _to_keras(e, st[sk][e.offset:e.offset + e.size])))
        attrs.append(("optimizer_weights", "weight_names", onames))
        lr = float(getattr(optimizer, "lr", 1e-3))
        ocfg = ({"name": "Adam", "learning_rate": lr, "decay": 0.0, "beta_1": optimizer.b1, "beta_2": optimizer.b2,
                 "epsilon": optimizer.eps, "amsgrad": False} if oname == "Adam"
                else {"name": "SGD", "learning_rate": lr, "decay": 0.0, "momentum": optimizer.mu,
                      "nesterov": optimizer.nesterov})
        attrs.append(("", "training_config", json.dumps({
            "loss": "sparse_categorical_crossentropy", "metrics": [["accuracy"]], "weighted_metrics": None,
            "loss_weights": None, "optimizer_config": {"class_name": oname, "config": ocfg}})))
    if progress is not None:
        attrs.append(("", "pddl_resume", json.dumps(progress)))
    tmp = path + ".tmp"
    h5().write(tmp, datasets, attrs)
    os.replace(tmp, path)   # atomic: a crashed writer never leaves a torn checkpoint


def _weights_group(path: str):
    """(group prefix, layer names) for a full-model file or a weights-only file."""
    m = h5()
    ln = m.read_attr(path, "model_weights", "layer_names")
    if ln is not None:
        return "model_weights", ln
    ln = m.read_attr(path, "", "layer_names")
    if ln is None:
        raise ValueError(f"{path}: not a Keras HDF5 weights file")
    return "", ln


def read_keras_weights(path: str) -> Dict[str, np.ndarray]:
    m = h5()
    grp, layers = _weights_group(path)
    out = {}
    for ln in layers:
        base = f"{grp}/{ln}" if grp else ln
        for wn in m.read_attr(path, base, "weight_names") or []:
            out[wn] = m.read_dataset(path, f"{base}/{wn}")
    return out


def load_weights_into(engine, weights: Dict[str, np.ndarray], strict_head: bool = False) -> int:
    L: ParamLayout = engine.L
    host = engine.params.detach().cpu().clone()
    n = 0
    for wn, arr in weights.items():
        if wn not in L.entries:
            continue
        e = L.entries[wn]
        host[e.offset:e.offset + e.size] = _from_keras(e, arr)
        n += 1
    engine.params.copy_(host.to(engine.params.device))
    return n


def load_pretrained(spec: str, engine) -> int:
    """weights='imagenet' (offline Keras notop file) or a path to any Keras .h5."""
    if spec == "imagenet":
        cands = [os.environ.get("PDDL_KERAS_WEIGHTS", ""),
                 os.path.expanduser("~/.keras/models/resnet50_weights_tf_dim_ordering_tf_kernels_notop.h5")]
        path = next((c for c in cands if c and os.path.exists(c)), None)
        if path is None:
            raise FileNotFoundError("weights='imagenet' needs resnet50_weights_tf_dim_ordering_tf_kernels_notop.h5 "
                                    "in ~/.keras/models or PDDL_KERAS_WEIGHTS (no network access)")
    else:
        path = spec
    n = load_weights_into(engine, read_keras_weights(path))
    if n == 0:
        raise ValueError(f"{path}: no ResNet-50 weights matched")
    return n


def load_checkpoint(path: str, engine, optimizer=None) -> int:
    """--resume: parameters + BN statistics + optimizer slots / iteration count."""
    n = load_weights_into(engine, read_keras_weights(path))
    if optimizer is not None:
        m = h5()
        names = m.read_attr(path, "optimizer_weights", "weight_names") or []
        st = optimizer.state_tensors()
        L = engine.L
        host = {k: v.detach().cpu().clone() for k, v in st.items()}
        for nm in names:
            parts = nm.split("/")
            if parts[-1] == "iter:0":
                optimizer.iterations = int(m.read_dataset(path, f"optimizer_weights/{nm}"))
                continue
            slot = parts[-1][:-2]
            wn = "/".join(parts[1:-1]) + ":0"
            if slot in host and wn in L.entries:
                e = L.entries[wn]
                host[slot][e.offset:e.offset + e.size] = _from_keras(e, m.read_dataset(path, f"optimizer_weights/{nm}"))
        for k, v in st.items():
            v.copy_(host[k].to(v.device))
    return n


def read_resume_state(path: str) -> Optional[dict]:
    """The `progress` a periodic checkpoint was saved with (None for a plain Keras file)."""
    raw = h5().read_attr(path, "", "pddl_resume")
    if not raw:
        return None
    return json.loads(raw if isinstance(raw, str) else raw[0])
