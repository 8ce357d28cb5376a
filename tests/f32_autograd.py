"""PyTorch-autograd form of the fp32 ResNet-50 over the fp32 HIP conv op (ops/conv_f32.py): an
independent test oracle for the explicit fp32 engines (models/engine_f32.py) -- PyTorch autograd
differentiates the same model instead of the hand-written backward schedule.  Not used by any
strategy."""
import torch
import torch.nn.functional as F

from pddl.models.reference import ReferenceResNet50, TorchEngine, preprocess
from pddl.models.resnet50 import ParamLayout
from pddl.ops.conv_f32 import conv2d_f32


class HipF32ResNet50(ReferenceResNet50):
    """ReferenceResNet50 with fp32 HIP convolutions (the explicit stem pad becomes the
    kernel's zero padding: same values, no padded copy of the input)."""

    def __init__(self, layout: ParamLayout, bn_mode: str = "frozen"):
        super().__init__(layout, bn_mode, bf16_points=False)

    def _conv(self, params, x, c, pad_explicit=False):
        w = self._w(params, c.name, "kernel")          # OHWI
        b = self._w(params, c.name, "bias")
        return conv2d_f32(x, w, b, c.stride, 0 if pad_explicit else c.pad)

    def features(self, params, x, training=True):
        # the stem's explicit (3, 3, 3, 3) pad folded into the conv's padding
        L = self.L
        s = L.stem
        x = F.relu(self._bn(params, conv2d_f32(x, self._w(params, s.name, "kernel"), self._w(params, s.name, "bias"),
                                               s.stride, 3), s, training))
        x = F.pad(x, (1, 1, 1, 1))
        x = F.max_pool2d(x, 3, 2)
        for b in L.blocks:
            c = b.convs
            sc = self._bn(params, self._conv(params, x, c["0"]), c["0"], training) if b.proj else x
            y = F.relu(self._bn(params, self._conv(params, x, c["1"]), c["1"], training))
            y = F.relu(self._bn(params, self._conv(params, y, c["2"]), c["2"], training))
            y = self._bn(params, self._conv(params, y, c["3"]), c["3"], training)
            x = F.relu(y + sc)
        return x.mean(dim=(2, 3))

    def logits(self, params, x, training=True):
        f = self.features(params, x, training)
        w = self._w(params, "dense", "kernel")        # [classes, 2048]
        out = conv2d_f32(f.view(f.shape[0], -1, 1, 1), w.view(w.shape[0], 1, 1, -1), self._w(params, "dense", "bias"))
        return out.reshape(f.shape[0], -1)


class HipF32AutogradEngine(TorchEngine):
    """TorchEngine interface (flat fp32 params / grads, forward_backward, evaluate) over
    HipF32ResNet50 on the GPU: the autograd form, kept for --bn-mode train in fp32 (batch
    statistics); the frozen-BN reference configuration runs HipF32Engine below."""

    def __init__(self, layout: ParamLayout, batch: int, crop: int = 224, device="cuda", bn_mode="frozen",
                 num_classes: int = 1000):
        super().__init__(layout, batch, crop=crop, device=device, bn_mode=bn_mode, num_classes=num_classes)
        self.model = HipF32ResNet50(layout, bn_mode)

    def forward_backward(self, images, labels, gscale, flip=None, crop_offset=(0, 0), bucket_cb=None, buckets=None):
        with torch.backends.cudnn.flags(enabled=False):
            return super().forward_backward(images, labels, gscale, flip, crop_offset, bucket_cb, buckets)

    @torch.no_grad()
    def evaluate(self, images, labels):
        with torch.backends.cudnn.flags(enabled=False):
            x = preprocess(images.to(self.device), self.crop, False)
            self.model.stats = self.params
            logits = self.model.logits(self.params, x, training=False)
            lab = labels.to(self.device)
            loss_sum = F.cross_entropy(logits, lab, reduction="sum")
            return torch.stack([loss_sum, (logits.argmax(1) == lab).sum().float()])
