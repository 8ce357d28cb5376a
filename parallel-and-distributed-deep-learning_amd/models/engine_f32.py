"""Reference-precision (fp32) GPU engines (`--precision fp32`; the reference trains in float32
with no mixed-precision policy, imagenet-resnet50.py:56-62).

HipF32Engine (frozen BN, the reference's `training=False`, Q3): the bf16 engine's explicit
schedule (models/engine.py) in fp32 end to end -- no autograd, no PyTorch kernel in the step;
up to batch 1024 the weight gradients (and each block's finalize) run on a side stream while the
data-gradient chain continues, over 5-deep gradient rings (b256: 61.9 -> 58.1-58.3 ms):
  forward  : stem_s2d (fp32 space-to-depth image) -> conv_f32 (4x4 window stem) -> maxpool_f32
             -> 16 bottleneck blocks of conv_f32 launches whose epilogues fold frozen BN + bias
             + residual + ReLU -> gap_f32 -> conv_f32 (Dense, bias epilogue)
  backward : softmax_xent_f32 -> per layer wgrad_f32 (raw dW, fp32 atomics) + a conv_f32 dgrad
             whose epilogue adds the residual gradient, applies the ReLU mask of the layer
             below, scatters the stride-2 grid and writes per-m-tile column sums; the
             projection block's two dgrad sources are two launches (the second adds the
             first); then the bf16 engine's wgrad_finalize / colsum_reduce / bn_grad kernels
             (dW *= BN scale, dgamma / dbeta / dbias).
HipF32EngineBNTrain (`--bn-mode train`): the same explicit schedule with batch-statistics BN
(bn.hip's kernels in fp32) -- no PyTorch op in the step either.
(tests/f32_autograd.py keeps a PyTorch-autograd form over the fp32 conv op as an independent
test oracle.)
"""
from __future__ import annotations

import struct
from typing import Callable, Dict, Optional

import torch

from ..ops.native import require_native
from ..utils import profiling as prof
from ..utils.envopts import opt
from .engine import _BNG_FMT, _CRED_FMT, _FIN_FMT, _PREP_FMT, STEM_K
from .resnet50 import BN_EPS, BN_MOMENTUM, ParamLayout


EPI_PLAIN, EPI_FWD, EPI_DGRAD = 0, 1, 2


def _rows64(m: int) -> int:
    return (m + 63) // 64


class HipF32Engine:
    """Explicit-schedule fp32 engine (frozen BN).  Interface of HipEngine / TorchEngine: flat
    fp32 `params` / `grads`, `init`, `after_update`, `forward_backward`, `evaluate`."""
    BN_MODES = ("frozen",)

    def __init__(self, layout: ParamLayout, batch: int, crop: int = 224, image_size: Optional[int] = None,
                 device="cuda", bn_mode: str = "frozen", num_classes: int = 1000):
        if bn_mode not in self.BN_MODES:
            raise ValueError(f"{type(self).__name__} runs bn_mode {self.BN_MODES[0]!r} "
                             "(HipF32Engine: frozen, the reference's training=False; HipF32EngineBNTrain: train)")
        self.N = require_native()
        self.L = L = layout
        self.device = dev = torch.device(device)
        self.batch, self.crop = batch, crop
        self.image_size = image_size if image_size is not None else crop
        self.num_classes = num_classes
        self.bn_mode = bn_mode
        f32 = dict(dtype=torch.float32, device=dev)
        self.params = torch.zeros(L.total, **f32)
        # per-channel bookkeeping, identical to the bf16 engine's (shared finalize / bn_grad kernels)
        self.ch: Dict[str, int] = {}
        off = 0
        for c in L.convs:
            self.ch[c.name] = off
            off += c.cout
        self.ch["dense"] = off
        off += (num_classes + 7) // 8 * 8
        self.nch = (off + 63) // 64 * 64
        n_tr = L.n_trainable
        nst = 64 * STEM_K
        self.ws = torch.zeros(n_tr + 2 * self.nch + 64 + nst, **f32)   # zeroed every step
        self.grads = self.ws[:n_tr]
        self.colsum = self.ws[n_tr:n_tr + self.nch]
        self.dgr = self.ws[n_tr + self.nch:n_tr + 2 * self.nch]
        self.stats = self.ws[n_tr + 2 * self.nch:n_tr + 2 * self.nch + 2]
        o = n_tr + 2 * self.nch + 64
        self.stem_dw2 = self.ws[o:o + nst].view(64, STEM_K)
        self.scale = torch.ones(self.nch, **f32)
        self.shift = torch.zeros(self.nch, **f32)
        self._tables()
        self._alloc(batch)

    # ------------------------------------------------------------------ tables
    def _dev_table(self, rows):
        return torch.frombuffer(bytearray(b"".join(rows)), dtype=torch.uint8).clone().to(self.device)

    def _tables(self):
        L = self.L
        # fp32 prepared weights: the stem in the 4x4x16 space-to-depth layout, then every layer's
        # dgrad weights [cin][R][S][cout] (flipped, transposed, scaled by the folded BN)
        self.wd: Dict[str, int] = {}
        off = 64 * STEM_K
        for c in L.convs[1:]:
            self.wd[c.name] = off
            off += c.cin * c.k * c.k * c.cout
        self.wd["dense"] = off
        off += 2048 * self.num_classes
        self.wf32 = torch.zeros(off, dtype=torch.float32, device=self.device)
        rows = []
        for c in L.convs:
            stem = c is L.stem
            g, b, m, v = L.off(c.bn, "gamma"), L.off(c.bn, "beta"), L.off(c.bn, "moving_mean"), \
                L.off(c.bn, "moving_variance")
            rows.append(struct.pack(_PREP_FMT, L.off(c.name, "kernel"), c.cout, c.k, c.k, c.cin,
                                    STEM_K if stem else c.k * c.k * c.cin, 0, -1 if stem else self.wd[c.name],
                                    c.cout, L.off(c.name, "bias"), g, b, m, v, self.ch[c.name], 1 if stem else 0))
        rows.append(struct.pack(_PREP_FMT, L.off("dense", "kernel"), self.num_classes, 1, 1, 2048, 2048, 0,
                                self.wd["dense"], self.num_classes, L.off("dense", "bias"), -1, -1, -1, -1,
                                self.ch["dense"], 0))
        self._prep_tab, self._prep_n = self._dev_table(rows), len(rows)
        fin = {c.name: struct.pack(_FIN_FMT, L.off(c.name, "kernel"), c.cout, c.k * c.k * c.cin, self.ch[c.name],
                                   self.ch[c.name]) for c in L.convs}
        self._fin = {b.name: self._dev_table([fin[b.convs[k].name] for k in (["3", "2", "1", "0"] if b.proj
                                                                              else ["3", "2", "1"])])
                     for b in L.blocks}
        self._fin["stem"] = self._dev_table([fin[L.stem.name]])
        bg = []
        for c in L.convs:
            cs = self.ch[c.name]
            for b in L.blocks:   # a projection block's conv0 BN sees conv3's output gradient
                if b.proj and b.convs["0"].name == c.name:
                    cs = self.ch[b.convs["3"].name]
            bg.append(struct.pack(_BNG_FMT, c.cout, self.ch[c.name], L.off(c.name, "bias"), L.off(c.bn, "gamma"),
                                  L.off(c.bn, "beta"), L.off(c.bn, "moving_mean"), L.off(c.bn, "moving_variance"),
                                  cs, self.ch[c.name]))
        bg.append(struct.pack(_BNG_FMT, self.num_classes, self.ch["dense"], L.off("dense", "bias"), -1, -1, -1, -1,
                              self.ch["dense"], -1))
        self._bng_tab, self._bng_n = self._dev_table(bg), len(bg)

    def _w(self, name, rows, k):           # forward weights: the fp32 master itself ([cout][R*S*cin])
        o = self.L.off(name, "kernel")
        return self.params[o:o + rows * k].view(rows, k)

    def _wd(self, name, cin, k):           # dgrad weights [cin][R*S*cout]
        o = self.wd[name]
        return self.wf32[o:o + cin * k].view(cin, k)

    def _gv(self, name, rows, k):
        o = self.L.off(name, "kernel")
        return self.grads[o:o + rows * k].view(rows, k)

    # ------------------------------------------------------------------ buffers
    def _alloc(self, B):
        L, dev = self.L, self.device
        f32 = dict(dtype=torch.float32, device=dev)
        crop = self.crop
        assert crop % 2 == 0, "crop must be even (space-to-depth stem)"
        self.H1 = H1 = (crop + 6 - 7) // 2 + 1
        self.H2 = H2 = (H1 + 2 - 3) // 2 + 1
        self.Hs = (crop + 6) // 2
        self.x2 = torch.empty(B, self.Hs, self.Hs, 16, **f32)
        self.c1 = torch.empty(B, H1, H1, 64, **f32)
        self.pool = torch.empty(B, H2, H2, 64, **f32)
        self.pidx = torch.empty(B, H2, H2, 64, dtype=torch.uint8, device=dev)
        self.acts, self.geo = {}, {}
        H, inner, outer, tmp = H2, 0, B * H1 * H1 * 64, 1
        for b in L.blocks:
            f = b.filters
            Ho = (H - 1) // b.stride + 1
            a = {"y1": torch.empty(B, Ho, Ho, f, **f32), "y2": torch.empty(B, Ho, Ho, f, **f32),
                 "out": torch.empty(B, Ho, Ho, 4 * f, **f32)}
            if b.proj:
                a["sc"] = torch.empty(B, Ho, Ho, 4 * f, **f32)
                tmp = max(tmp, B * Ho * Ho * b.cin)
            self.acts[b.name] = a
            self.geo[b.name] = (H, Ho)
            inner = max(inner, B * Ho * Ho * f)
            outer = max(outer, B * H * H * b.cin, B * Ho * Ho * 4 * f)
            H = Ho
        self.H5 = H
        # two-stream backward (weight gradients on a side stream, HipF32Engine._side_run): the
        # gradient buffers are rings deep enough for the data-gradient chain to run a few
        # blocks ahead of the weight gradients still reading older ones
        self.two_stream = self._two_stream_wanted(B)
        D = opt("PDDL_ENGINE", "grad_ring", self.RING) if self.two_stream else 1
        self.gbuf = [torch.empty(outer, **f32) for _ in range(max(2, D))]
        self.g1bufs = [torch.empty(inner, **f32) for _ in range(D)]
        self.g2bufs = [torch.empty(inner, **f32) for _ in range(D)]
        self.g1buf, self.g2buf = self.g1bufs[0], self.g2bufs[0]
        self.side = torch.cuda.Stream(dev) if self.two_stream and dev.type == "cuda" else None
        self._evpool, self._evi = [], 0
        self.tmp = torch.empty(tmp, **f32)
        # split-K workspace of the underfilled conv / dgrad problems (conv_f32.hip: small batches),
        # this engine's own (N.splitk_use makes it current for the launching thread)
        self.splitk_ws = torch.empty(self.N.splitk_default_floats(dev.index or 0), **f32) if dev.type == "cuda" else None
        # blocks feeding a stride-2 projection block: their output gradient is written on the
        # stride-2 grid only (dgrad up2 scatter) into a buffer zeroed once here
        bl = L.blocks
        self.s2 = {bi for bi in range(len(bl) - 1) if bl[bi + 1].proj and bl[bi + 1].stride == 2}
        self.s2full = {bi: torch.zeros(B * self.geo[bl[bi].name][1] ** 2 * 4 * bl[bi].filters, **f32)
                       for bi in self.s2}
        self.pooled = torch.empty(B, 2048, **f32)
        self.logits = torch.empty(B, self.num_classes, **f32)
        self.dlogits = torch.empty(B, self.num_classes, **f32)
        self.dpooled = torch.empty(B, 2048, **f32)
        self.labels_dev = torch.zeros(B, dtype=torch.int64, device=dev)
        self.cap = B
        self._cred = {}
        self.colpart = torch.empty(self._colred(B)[2], **f32)

    def _colred(self, B):
        """Partial column-sum regions of the fused producers: (offsets by layer, table, floats, n)."""
        if B in self._cred:
            return self._cred[B]
        offs, rows, off = {}, [], 0

        def add(layer, nrows, C):
            nonlocal off
            offs[layer] = off
            rows.append(struct.pack(_CRED_FMT, off, nrows, C, self.ch[layer], 0))
            off += nrows * C
        bl = self.L.blocks
        add(bl[-1].convs["3"].name, B, 2048)                        # gap_bwd: one row per image
        for bi in range(len(bl) - 1, -1, -1):
            b = bl[bi]
            H, Ho = self.geo[b.name]
            M = B * Ho * Ho
            add(b.convs["2"].name, _rows64(M), b.filters)            # c3 dgrad -> g2
            add(b.convs["1"].name, _rows64(M), b.filters)            # c2 dgrad -> g1
            if bi > 0:                                               # c1 dgrad -> previous output
                add(bl[bi - 1].convs["3"].name, _rows64(M if b.stride == 2 else B * H * H), b.cin)
        res = (offs, self._dev_table(rows), off, len(rows))
        self._cred[B] = res
        return res

    # ------------------------------------------------------------------ two-stream backward
    TWO_STREAM_MAX_BATCH = 1024
    RING = 5   # (fp32 b256: ring 2 / 3 / 5 / 8 -> 59.9 / 59.3 / 58.4 / 58.5 ms; one stream 61.9)

    def _two_stream_wanted(self, batch) -> bool:
        ts = opt("PDDL_ENGINE", "two_stream", "auto")
        if ts != "auto":
            return ts == "1"
        return batch <= self.TWO_STREAM_MAX_BATCH

    def _event(self):
        """The i-th fork / join event of every step reuses one pooled event (a wait binds to the
        record made before it), so a step creates no HIP events."""
        i = self._evi
        self._evi += 1
        if i == len(self._evpool):
            self._evpool.append(torch.cuda.Event())
        return self._evpool[i]

    def _side_run(self, fn, *args, reads=()):
        """fn(*args) on the side stream after everything enqueued on the compute stream so far;
        `reads`: the gradient buffers it reads, which the compute stream must not overwrite
        before it is done (_before_write)."""
        if self.side is None:
            fn(*args)
            return
        ev = self._event()
        ev.record(torch.cuda.current_stream(self.device))
        self.side.wait_event(ev)
        with torch.cuda.stream(self.side):
            fn(*args)
        done = self._event()
        done.record(self.side)
        for r in reads:
            self._pending[r] = done
        self._last_side = done

    def _before_write(self, *bufs):
        if self.side is None:
            return
        main = torch.cuda.current_stream(self.device)
        for b in bufs:
            ev = self._pending.pop(b, None)
            if ev is not None:
                main.wait_event(ev)

    def _join_side(self):
        if self.side is not None and self._last_side is not None:
            torch.cuda.current_stream(self.device).wait_event(self._last_side)
            self._pending.clear()
            self._last_side = None

    # ------------------------------------------------------------------ params
    def init(self, seed=0):
        self.L.init_params(self.params, seed)
        self.after_update()

    def after_update(self):
        """Folded BN affine + fp32 stem / dgrad weights from the master (one launch pair)."""
        self.N.prep_f32(self.params, self._prep_tab, self._prep_n, self.wf32, self.scale, self.shift, BN_EPS)

    # ------------------------------------------------------------------ forward
    def _stem_mode(self, training, crop_offset):
        if self.crop == self.image_size:
            return 0, 0, 0
        if self.crop > self.image_size or not training:
            return 1, 0, 0
        return 2, crop_offset[0], crop_offset[1]

    def _conv(self, x, R, stride, pad, Ho, w, out, scale=None, shift=None, res=None, relu=0, epi=EPI_FWD,
              add=None, mask=None, up2=0, colsum=None):
        self.N.conv_f32_epi(x, R, R, stride, pad, Ho, Ho, w, epi, scale, shift, res, relu, add, mask, up2, out,
                            colsum)

    def _fwd_conv(self, c, x, out, res=None, relu=1):
        ch = self.ch[c.name]
        self._conv(x, c.k, c.stride, c.pad, out.shape[1], self._w(c.name, c.cout, c.k * c.k * c.cin), out,
                   self.scale[ch:], self.shift[ch:], res, relu)

    def _forward(self, images, B, training, flip, crop_offset):
        self.N.splitk_use(self.splitk_ws)   # this engine's split-K workspace, for this thread's launches
        N, L = self.N, self.L
        mode, oy, ox = self._stem_mode(training, crop_offset)
        x2 = self.x2[:B]
        N.stem_s2d(images, flip if training else None, mode, self.crop, self.crop, oy, ox, x2, None)
        s = L.stem
        c1 = self.c1[:B]
        ch = self.ch[s.name]
        self._conv(x2, 4, 1, 0, self.H1, self.wf32[:64 * STEM_K].view(64, STEM_K), c1, self.scale[ch:],
                   self.shift[ch:], None, 1)
        pool = self.pool[:B]
        N.maxpool_fwd_f32(c1, pool, self.pidx[:B])
        x = pool
        for b in L.blocks:
            a = {k: v[:B] for k, v in self.acts[b.name].items()}
            if b.proj:
                self._fwd_conv(b.convs["1"], x, a["y1"])
                self._fwd_conv(b.convs["0"], x, a["sc"], relu=0)
                res = a["sc"]
            else:
                self._fwd_conv(b.convs["1"], x, a["y1"])
                res = x
            self._fwd_conv(b.convs["2"], a["y1"], a["y2"])
            self._fwd_conv(b.convs["3"], a["y2"], a["out"], res=res)
            x = a["out"]
        pooled = self.pooled[:B]
        N.gap_fwd_f32(x, pooled)
        chd = self.ch["dense"]
        self._conv(pooled.view(B, 1, 1, 2048), 1, 1, 0, 1, self._w("dense", self.num_classes, 2048),
                   self.logits[:B].view(B, 1, 1, self.num_classes), self.scale[chd:], self.shift[chd:], None, 0)
        return x

    def _labels(self, labels, B):
        lab = self.labels_dev[:B]
        lab.copy_(labels, non_blocking=True)
        return lab

    # ------------------------------------------------------------------ train step
    def forward_backward(self, images, labels, gscale, flip=None, crop_offset=(0, 0),
                         bucket_cb: Optional[Callable[[int], None]] = None, buckets=None):
        N, L = self.N, self.L
        B = images.shape[0]
        assert B <= self.cap, "batch larger than the engine's buffers"
        self.ws.zero_()
        lab = self._labels(labels, B)
        prof.push("step/forward")
        x5 = self._forward(images, B, True, flip, crop_offset)
        prof.pop()
        prof.push("step/backward")
        ncls = self.num_classes
        dl = self.dlogits[:B]
        N.softmax_xent_f32(self.logits[:B], lab, ncls, float(gscale), dl, self.stats[0:1], self.stats[1:2])
        bks = buckets if buckets is not None else []
        nb = [0]

        def done_upto(off):
            while bucket_cb is not None and nb[0] < len(bks) - 1 and bks[nb[0]][1] <= off:
                bucket_cb(nb[0])
                nb[0] += 1

        # ---- head
        self._pending, self._last_side, self._evi = {}, None, 0
        pooled = self.pooled[:B]
        chd = self.ch["dense"]
        N.wgrad_f32(pooled.view(B, 1, 1, 2048), 1, 1, 1, 0, dl.view(B, 1, 1, ncls), self._gv("dense", ncls, 2048))
        N.colsum_f32(dl, ncls, self.colsum[chd:])
        dpooled = self.dpooled[:B]
        self._conv(dl.view(B, 1, 1, ncls), 1, 1, 0, 1, self._wd("dense", 2048, ncls), dpooled.view(B, 1, 1, 2048),
                   epi=EPI_PLAIN)
        e = L.entry("dense", "kernel")
        done_upto(e.offset + e.size)
        H5, bl = self.H5, L.blocks
        coffs, ctab, _, cn = self._colred(B)
        cp = self.colpart
        D = len(self.g1bufs)
        nbuf = len(self.gbuf)

        def part(layer):
            return cp[coffs[layer]:]
        # weight gradients (+ each block's finalize) on the side stream, data gradients on the
        # compute stream; ("g", i) / ("g1", j) / ("g2", j) / ("s2", bi): gradient buffers a side
        # launch reads, which the compute stream waits for before overwriting
        cur = 0
        gout = self.gbuf[cur][: B * H5 * H5 * 2048].view(B, H5, H5, 2048)
        N.gap_bwd_f32(dpooled, x5, gout, part(bl[-1].convs["3"].name))
        for bi in range(len(bl) - 1, -1, -1):
            b = bl[bi]
            a = {k: v[:B] for k, v in self.acts[b.name].items()}
            H, Ho = self.geo[b.name]
            f, cin = b.filters, b.cin
            x_in = self.acts[bl[bi - 1].name]["out"][:B] if bi > 0 else self.pool[:B]
            c1n, c2n, c3n = b.convs["1"].name, b.convs["2"].name, b.convs["3"].name
            gkey = ("s2", bi) if bi in self.s2 else ("g", cur)
            gsrc = self.s2full[bi] if bi in self.s2 else self.gbuf[cur]
            gout = gsrc[: B * Ho * Ho * 4 * f].view(B, Ho, Ho, 4 * f)
            j = bi % D
            g2 = self.g2bufs[j][: B * Ho * Ho * f].view(B, Ho, Ho, f)
            g1 = self.g1bufs[j][: B * Ho * Ho * f].view(B, Ho, Ho, f)
            # conv3 (1x1) and conv2 (3x3): raw dW, then dgrad with the ReLU mask of their input
            self._side_run(N.wgrad_f32, a["y2"], 1, 1, 1, 0, gout, self._gv(c3n, 4 * f, f), reads=(gkey,))
            self._before_write(("g2", j))
            self._conv(gout, 1, 1, 0, Ho, self._wd(c3n, f, 4 * f), g2, epi=EPI_DGRAD, mask=a["y2"],
                       colsum=part(c2n))
            self._side_run(N.wgrad_f32, a["y1"], 3, 3, 1, 1, g2, self._gv(c2n, f, 9 * f), reads=(("g2", j),))
            self._before_write(("g1", j))
            self._conv(g2, 3, 1, 1, Ho, self._wd(c2n, f, 9 * f), g1, epi=EPI_DGRAD, mask=a["y1"],
                       colsum=part(c1n))
            # conv1 (+ conv0): input gradient of the block
            nxt = (cur + 1) % nbuf
            cs_in = part(bl[bi - 1].convs["3"].name) if bi > 0 else None
            if b.proj:
                c0n = b.convs["0"].name
                self._side_run(N.wgrad_f32, x_in, 1, 1, b.stride, 0, g1, self._gv(c1n, f, cin), reads=(("g1", j),))
                self._side_run(N.wgrad_f32, x_in, 1, 1, b.stride, 0, gout, self._gv(c0n, 4 * f, cin), reads=(gkey,))
                self._side_run(N.wgrad_finalize, self.params, self.grads, self._fin[b.name], 4, self.scale, self.dgr)
                # dx = (W1'.g1 + W0'.gout) * mask: the first source into `tmp`, added by the second
                tmp = self.tmp[: B * Ho * Ho * cin].view(B, Ho, Ho, cin)
                self._conv(g1, 1, 1, 0, Ho, self._wd(c1n, cin, f), tmp, epi=EPI_PLAIN)
                if b.stride == 2:
                    gx = self.s2full[bi - 1][: B * H * H * cin].view(B, H, H, cin)   # grid positions only
                    self._before_write(("s2", bi - 1))
                    self._conv(gout, 1, 1, 0, Ho, self._wd(c0n, cin, 4 * f), gx, epi=EPI_DGRAD, add=tmp,
                               mask=x_in, up2=1, colsum=cs_in)
                else:
                    gx = self.gbuf[nxt][: B * H * H * cin].view(B, H, H, cin)
                    self._before_write(("g", nxt))
                    self._conv(gout, 1, 1, 0, Ho, self._wd(c0n, cin, 4 * f), gx, epi=EPI_DGRAD, add=tmp,
                               mask=x_in, colsum=cs_in)
                last = L.entry(c0n, "kernel")
            else:
                self._side_run(N.wgrad_f32, x_in, 1, 1, 1, 0, g1, self._gv(c1n, f, cin), reads=(("g1", j),))
                self._side_run(N.wgrad_finalize, self.params, self.grads, self._fin[b.name], 3, self.scale, self.dgr)
                gx = self.gbuf[nxt][: B * H * H * cin].view(B, H, H, cin)
                self._before_write(("g", nxt))
                self._conv(g1, 1, 1, 0, H, self._wd(c1n, cin, f), gx, epi=EPI_DGRAD, add=gout, mask=x_in,
                           colsum=cs_in)
                last = L.entry(c1n, "kernel")
            if bucket_cb is not None:
                self._join_side()   # (a bucket's weight gradients come from the side stream)
            done_upto(last.offset + last.size)
            cur = nxt
        # ---- stem: max-pool backward (with conv1's ReLU mask), s2d-domain wgrad folded to 7x7x3
        H1, H2 = self.H1, self.H2
        gpool = self.gbuf[cur][: B * H2 * H2 * 64].view(B, H2, H2, 64)
        gi = (cur + 1) % nbuf
        gc1 = self.gbuf[gi][: B * H1 * H1 * 64].view(B, H1, H1, 64)
        s = L.stem
        self._before_write(("g", gi))
        N.maxpool_bwd_f32(gpool, self.pidx[:B], self.c1[:B], gc1)
        N.colsum_f32(gc1.view(-1, 64), 64, self.colsum[self.ch[s.name]:])
        self._side_run(N.wgrad_f32, self.x2[:B], 4, 4, 1, 0, gc1, self.stem_dw2, reads=(("g", gi),))
        self._side_run(N.stem_wgrad_fold, self.stem_dw2, self._gv(s.name, 64, 147), 64)
        self._side_run(N.wgrad_finalize, self.params, self.grads, self._fin["stem"], 1, self.scale, self.dgr)
        N.colsum_reduce(cp, ctab, cn, self.colsum)   # (compute-stream data only: under the side stream's tail)
        self._join_side()
        done_upto(L.kernels_end)
        N.bn_grad(self.params, self.grads, self._bng_tab, self._bng_n, self.colsum, self.dgr, self.scale, BN_EPS)
        prof.pop()
        if bucket_cb is not None:
            while nb[0] < len(bks):
                bucket_cb(nb[0])
                nb[0] += 1
        return self.stats

    @torch.no_grad()
    def evaluate(self, images, labels):
        B = images.shape[0]
        assert B <= self.cap
        self.stats.zero_()
        lab = self._labels(labels, B)
        self._forward(images, B, False, None, (0, 0))
        self.N.softmax_xent_f32(self.logits[:B], lab, self.num_classes, 0.0, self.dlogits[:B], self.stats[0:1],
                                self.stats[1:2])
        return self.stats


_STAT_FMT = "<8if i"   # BnStatLayer (csrc/kernels/kernels.h)


class HipF32EngineBNTrain(HipF32Engine):
    """fp32 engine with train-mode BatchNormalization (Keras `training=True`: batch mean / biased
    variance normalise, Bessel-corrected variance into the moving statistics, momentum 0.99,
    epsilon 1.001e-5) -- the explicit schedule of HipF32Engine with nothing folded into the
    convolutions and the bf16 train engine's BN kernels (csrc/kernels/bn.hip, templated on the
    activation type) in fp32.  No PyTorch op in the step:

      forward, per conv  : conv_f32 -> z = conv + bias (fp32)
                           -> bn_bwd_reduce(z, z, mean 0) = per-channel (sum z, sum z^2)
                           -> bn_stats (mean, 1/sigma, BN scale / shift, moving statistics)
                           -> bn_apply: y = relu(bn(z) [+ x | + bn0(z0)])
      backward, per conv : (the next conv's dgrad applies the ReLU mask of y and adds the
                           residual gradient) -> bn_bwd_reduce (sum g, sum g*(z - mean))
                           -> bn_bwd_apply (dz; dgamma, dbeta, dbias = 0) -> wgrad_f32(x, dz)
                           (on the side stream, as in HipF32Engine) and the conv_f32 dgrad of dz;
                           a projection block's BN3 and BN0 share one reduce and one apply.
    The reference itself freezes BN (imagenet-resnet50.py:57): this is the `--bn-mode train`
    variant at the reference's precision (tests/test_gpu_f32.py bounds it against the PyTorch
    reference model in float64)."""
    BN_MODES = ("train",)
    RING = 12   # (fp32 b256: ring 3 / 5 / 8 / 12 / 16 -> 73.4 / 73.1 / 72.3-72.6 / 71.9 / 71.8 ms)

    def __init__(self, layout: ParamLayout, batch: int, crop: int = 224, image_size: Optional[int] = None,
                 device="cuda", bn_mode: str = "train", num_classes: int = 1000):
        super().__init__(layout, batch, crop=crop, image_size=image_size, device=device, bn_mode=bn_mode,
                         num_classes=num_classes)
        assert struct.calcsize(_STAT_FMT) == self.N.BNSTAT_LAYER_BYTES
        f32 = dict(dtype=torch.float32, device=self.device)
        n = self.nch
        self.bn_mean, self.bn_inv = torch.zeros(n, **f32), torch.ones(n, **f32)
        self.bn_scale, self.bn_shift = torch.ones(n, **f32), torch.zeros(n, **f32)
        self.bws = torch.zeros(4 * n, **f32)          # zeroed every step: acc S | acc Q | sum g | sum g(z-mean)
        self.acc = self.bws[:2 * n]
        self.bsg, self.bsgx = self.bws[2 * n:3 * n], self.bws[3 * n:]
        self.bcoef = torch.zeros(3 * n, **f32)
        self.zero_c = torch.zeros(2048, **f32)
        L = self.L
        self._bng_dense = self._dev_table([struct.pack(_BNG_FMT, self.num_classes, self.ch["dense"],
                                                       L.off("dense", "bias"), -1, -1, -1, -1, self.ch["dense"], -1)])
        self._stat_tabs: Dict[tuple, torch.Tensor] = {}
        self._eval_tab = self._stat_table(L.convs, 1.0, training=False)

    # ------------------------------------------------------------------ tables
    def _tables(self):
        super()._tables()
        # nothing folded: the conv epilogue adds only the bias (scale 1), the dgrad weights are
        # W^T unscaled; the batch statistics drive bn_apply / bn_bwd_apply instead
        L, rows = self.L, []
        for c in L.convs:
            stem = c is L.stem
            rows.append(struct.pack(_PREP_FMT, L.off(c.name, "kernel"), c.cout, c.k, c.k, c.cin,
                                    STEM_K if stem else c.k * c.k * c.cin, 0, -1 if stem else self.wd[c.name],
                                    c.cout, L.off(c.name, "bias"), -1, -1, -1, -1, self.ch[c.name], 1 if stem else 0))
        rows.append(struct.pack(_PREP_FMT, L.off("dense", "kernel"), self.num_classes, 1, 1, 2048, 2048, 0,
                                self.wd["dense"], self.num_classes, L.off("dense", "bias"), -1, -1, -1, -1,
                                self.ch["dense"], 0))
        self._prep_tab, self._prep_n = self._dev_table(rows), len(rows)

    def _stat_table(self, convs, count: float, training: bool = True):
        n, L = self.nch, self.L
        rows = [struct.pack(_STAT_FMT, c.cout, self.ch[c.name], n + self.ch[c.name], self.ch[c.name],
                            L.off(c.bn, "gamma"), L.off(c.bn, "beta"), L.off(c.bn, "moving_mean"),
                            L.off(c.bn, "moving_variance"), float(count), 0) for c in convs]
        return self._dev_table(rows)

    def _stats(self, c, M):
        key = (c.name, M)
        t = self._stat_tabs.get(key)
        if t is None:
            t = self._stat_tabs[key] = self._stat_table([c], float(M))
        return t

    def _alloc(self, B):
        super()._alloc(B)
        f32 = dict(dtype=torch.float32, device=self.device)
        self.zs = torch.empty(B, self.H1, self.H1, 64, **f32)
        self.z: Dict[str, Dict[str, torch.Tensor]] = {}
        for b in self.L.blocks:
            H, Ho = self.geo[b.name]
            f = b.filters
            z = {"1": torch.empty(B, Ho, Ho, f, **f32), "2": torch.empty(B, Ho, Ho, f, **f32),
                 "3": torch.empty(B, Ho, Ho, 4 * f, **f32)}
            if b.proj:
                z["0"] = torch.empty(B, Ho, Ho, 4 * f, **f32)
            self.z[b.name] = z
        # dz3 of each block: a ring like the other gradient buffers (the side stream's conv3
        # weight gradient reads it while the compute stream runs ahead)
        self.gbuf3s = [torch.empty_like(self.gbuf[0]) for _ in range(len(self.g1bufs))]

    # ------------------------------------------------------------------ forward
    def _chs(self, arr, c):
        o = self.ch[c.name]
        return arr[o:o + c.cout]

    def _z(self, c, x, R, stride, pad, Ho, w, z, training):
        """z = conv(x) + bias; when training, its batch statistics -> BN scale / shift."""
        ch = self.ch[c.name]
        self._conv(x, R, stride, pad, Ho, w, z, self.scale[ch:], self.shift[ch:], None, 0)
        if training:
            M = z.numel() // c.cout
            self.N.bn_bwd_reduce(z, z, None, self.zero_c[:c.cout], None, self.acc[ch:ch + c.cout],
                                 self.acc[self.nch + ch:self.nch + ch + c.cout], None, None)
            self.N.bn_stats(self.acc, self._stats(c, M), 1, c.cout, True, self.params, self.bn_mean, self.bn_inv,
                            self.bn_scale, self.bn_shift, BN_EPS, BN_MOMENTUM)

    def _forward(self, images, B, training, flip, crop_offset):
        self.N.splitk_use(self.splitk_ws)   # this engine's split-K workspace, for this thread's launches
        N, L = self.N, self.L
        if not training:   # the moving statistics for every layer at once
            N.bn_stats(self.acc, self._eval_tab, len(L.convs), 2048, False, self.params, self.bn_mean, self.bn_inv,
                       self.bn_scale, self.bn_shift, BN_EPS, BN_MOMENTUM)
        mode, oy, ox = self._stem_mode(training, crop_offset)
        x2 = self.x2[:B]
        N.stem_s2d(images, flip if training else None, mode, self.crop, self.crop, oy, ox, x2, None)
        s = L.stem
        zs, c1 = self.zs[:B], self.c1[:B]
        self._z(s, x2, 4, 1, 0, self.H1, self.wf32[:64 * STEM_K].view(64, STEM_K), zs, training)
        N.bn_apply(zs, self._chs(self.bn_scale, s), self._chs(self.bn_shift, s), None, None, None, True, c1, None)
        pool = self.pool[:B]
        N.maxpool_fwd_f32(c1, pool, self.pidx[:B])
        x = pool
        for b in L.blocks:
            a = {k: v[:B] for k, v in self.acts[b.name].items()}
            z = {k: v[:B] for k, v in self.z[b.name].items()}
            Ho = self.geo[b.name][1]
            f = b.filters
            c = b.convs
            self._z(c["1"], x, 1, b.stride, 0, Ho, self._w(c["1"].name, f, b.cin), z["1"], training)
            if b.proj:
                self._z(c["0"], x, 1, b.stride, 0, Ho, self._w(c["0"].name, 4 * f, b.cin), z["0"], training)
            N.bn_apply(z["1"], self._chs(self.bn_scale, c["1"]), self._chs(self.bn_shift, c["1"]), None, None, None,
                       True, a["y1"], None)
            self._z(c["2"], a["y1"], 3, 1, 1, Ho, self._w(c["2"].name, f, 9 * f), z["2"], training)
            N.bn_apply(z["2"], self._chs(self.bn_scale, c["2"]), self._chs(self.bn_shift, c["2"]), None, None, None,
                       True, a["y2"], None)
            self._z(c["3"], a["y2"], 1, 1, 0, Ho, self._w(c["3"].name, 4 * f, f), z["3"], training)
            if b.proj:
                N.bn_apply(z["3"], self._chs(self.bn_scale, c["3"]), self._chs(self.bn_shift, c["3"]), z["0"],
                           self._chs(self.bn_scale, c["0"]), self._chs(self.bn_shift, c["0"]), True, a["out"], None)
            else:
                N.bn_apply(z["3"], self._chs(self.bn_scale, c["3"]), self._chs(self.bn_shift, c["3"]), x, None, None,
                           True, a["out"], None)
            x = a["out"]
        pooled = self.pooled[:B]
        N.gap_fwd_f32(x, pooled)
        chd = self.ch["dense"]
        self._conv(pooled.view(B, 1, 1, 2048), 1, 1, 0, 1, self._w("dense", self.num_classes, 2048),
                   self.logits[:B].view(B, 1, 1, self.num_classes), self.scale[chd:], self.shift[chd:], None, 0)
        return x

    # ------------------------------------------------------------------ backward
    def _bn_layer(self, c, M):
        L = self.L
        return [float(c.cout), float(self.ch[c.name]), float(L.off(c.bn, "gamma")), float(L.off(c.bn, "beta")),
                float(L.off(c.name, "bias")), float(M)]

    def _bn_bwd(self, g, z, c, M, out, z2=None, c2=None, out2=None):
        """dz (into `out`, may alias g) from g = dL/dy of conv `c`'s BN; with z2 / c2 the second BN
        fed by the same gradient (a projection block's shortcut)."""
        N = self.N
        if z2 is None:
            N.bn_bwd_reduce(g, z, None, self._chs(self.bn_mean, c), None, self._chs(self.bsg, c),
                            self._chs(self.bsgx, c), None, None)
            N.bn_bwd_apply(g, z, None, self._bn_layer(c, M), [], self.params, self.bn_mean, self.bn_inv, self.bsg,
                           self.bsgx, out, None, self.grads, self.bcoef)
        else:
            N.bn_bwd_reduce(g, z, z2, self._chs(self.bn_mean, c), self._chs(self.bn_mean, c2), self._chs(self.bsg, c),
                            self._chs(self.bsgx, c), self._chs(self.bsg, c2), self._chs(self.bsgx, c2))
            N.bn_bwd_apply(g, z, z2, self._bn_layer(c, M), self._bn_layer(c2, M), self.params, self.bn_mean,
                           self.bn_inv, self.bsg, self.bsgx, out, out2, self.grads, self.bcoef)

    def forward_backward(self, images, labels, gscale, flip=None, crop_offset=(0, 0),
                         bucket_cb: Optional[Callable[[int], None]] = None, buckets=None):
        N, L = self.N, self.L
        B = images.shape[0]
        assert B <= self.cap, "batch larger than the engine's buffers"
        self.ws.zero_()
        self.bws.zero_()
        lab = self._labels(labels, B)
        prof.push("step/forward")
        x5 = self._forward(images, B, True, flip, crop_offset)
        prof.pop()
        prof.push("step/backward")
        ncls = self.num_classes
        dl = self.dlogits[:B]
        N.softmax_xent_f32(self.logits[:B], lab, ncls, float(gscale), dl, self.stats[0:1], self.stats[1:2])
        bks = buckets if buckets is not None else []
        nb = [0]

        def done_upto(off):
            while bucket_cb is not None and nb[0] < len(bks) - 1 and bks[nb[0]][1] <= off:
                bucket_cb(nb[0])
                nb[0] += 1

        # ---- head: Dense wgrad, bias gradient (column sums), dgrad into the pooled features
        self._pending, self._last_side, self._evi = {}, None, 0
        pooled = self.pooled[:B]
        chd = self.ch["dense"]
        N.wgrad_f32(pooled.view(B, 1, 1, 2048), 1, 1, 1, 0, dl.view(B, 1, 1, ncls), self._gv("dense", ncls, 2048))
        N.colsum_f32(dl, ncls, self.colsum[chd:])
        N.bn_grad(self.params, self.grads, self._bng_dense, 1, self.colsum, self.dgr, self.scale, BN_EPS)
        dpooled = self.dpooled[:B]
        self._conv(dl.view(B, 1, 1, ncls), 1, 1, 0, 1, self._wd("dense", 2048, ncls), dpooled.view(B, 1, 1, 2048),
                   epi=EPI_PLAIN)
        e = L.entry("dense", "kernel")
        done_upto(e.offset + e.size)
        cur = 0
        H5, bl = self.H5, L.blocks
        D, nbuf = len(self.g1bufs), len(self.gbuf)
        W = self._side_run
        gout = self.gbuf[cur][: B * H5 * H5 * 2048].view(B, H5, H5, 2048)
        N.gap_bwd_f32(dpooled, x5, gout, None)
        # weight gradients on the side stream (HipF32Engine._side_run), BN backward and data
        # gradients on the compute stream; ("g", i) / ("s2", bi) / ("z3", j) / ("g2", j) / ("g1", j):
        # gradient buffers a side launch reads, waited for before the compute stream rewrites them
        for bi in range(len(bl) - 1, -1, -1):
            b = bl[bi]
            a = {k: v[:B] for k, v in self.acts[b.name].items()}
            z = {k: v[:B] for k, v in self.z[b.name].items()}
            H, Ho = self.geo[b.name]
            M = B * Ho * Ho
            f, cin = b.filters, b.cin
            x_in = self.acts[bl[bi - 1].name]["out"][:B] if bi > 0 else self.pool[:B]
            c1c, c2c, c3c = b.convs["1"], b.convs["2"], b.convs["3"]
            gkey = ("s2", bi) if bi in self.s2 else ("g", cur)
            gsrc = self.s2full[bi] if bi in self.s2 else self.gbuf[cur]
            gout = gsrc[: M * 4 * f].view(B, Ho, Ho, 4 * f)
            j = bi % D
            dz3 = self.gbuf3s[j][: M * 4 * f].view(B, Ho, Ho, 4 * f)
            self._before_write(("z3", j))
            if b.proj:   # BN3 and the shortcut's BN0 share gout; dz0 overwrites gout in place
                self._bn_bwd(gout, z["3"], c3c, M, dz3, z["0"], b.convs["0"], gout)
            else:
                self._bn_bwd(gout, z["3"], c3c, M, dz3)
            g2 = self.g2bufs[j][: M * f].view(B, Ho, Ho, f)
            g1 = self.g1bufs[j][: M * f].view(B, Ho, Ho, f)
            W(N.wgrad_f32, a["y2"], 1, 1, 1, 0, dz3, self._gv(c3c.name, 4 * f, f), reads=(("z3", j),))
            self._before_write(("g2", j))
            self._conv(dz3, 1, 1, 0, Ho, self._wd(c3c.name, f, 4 * f), g2, epi=EPI_DGRAD, mask=a["y2"])
            self._bn_bwd(g2, z["2"], c2c, M, g2)
            W(N.wgrad_f32, a["y1"], 3, 3, 1, 1, g2, self._gv(c2c.name, f, 9 * f), reads=(("g2", j),))
            self._before_write(("g1", j))
            self._conv(g2, 3, 1, 1, Ho, self._wd(c2c.name, f, 9 * f), g1, epi=EPI_DGRAD, mask=a["y1"])
            self._bn_bwd(g1, z["1"], c1c, M, g1)
            nxt = (cur + 1) % nbuf
            if b.proj:
                c0n = b.convs["0"].name
                W(N.wgrad_f32, x_in, 1, 1, b.stride, 0, g1, self._gv(c1c.name, f, cin), reads=(("g1", j),))
                W(N.wgrad_f32, x_in, 1, 1, b.stride, 0, gout, self._gv(c0n, 4 * f, cin), reads=(gkey,))
                tmp = self.tmp[: B * Ho * Ho * cin].view(B, Ho, Ho, cin)
                self._conv(g1, 1, 1, 0, Ho, self._wd(c1c.name, cin, f), tmp, epi=EPI_PLAIN)
                if b.stride == 2:
                    gx = self.s2full[bi - 1][: B * H * H * cin].view(B, H, H, cin)   # grid positions only
                    self._before_write(("s2", bi - 1))
                    self._conv(gout, 1, 1, 0, Ho, self._wd(c0n, cin, 4 * f), gx, epi=EPI_DGRAD, add=tmp,
                               mask=x_in, up2=1)
                else:
                    gx = self.gbuf[nxt][: B * H * H * cin].view(B, H, H, cin)
                    self._before_write(("g", nxt))
                    self._conv(gout, 1, 1, 0, Ho, self._wd(c0n, cin, 4 * f), gx, epi=EPI_DGRAD, add=tmp,
                               mask=x_in)
                last = L.entry(c0n, "kernel")
            else:
                W(N.wgrad_f32, x_in, 1, 1, 1, 0, g1, self._gv(c1c.name, f, cin), reads=(("g1", j),))
                gx = self.gbuf[nxt][: B * H * H * cin].view(B, H, H, cin)
                self._before_write(("g", nxt))
                self._conv(g1, 1, 1, 0, H, self._wd(c1c.name, cin, f), gx, epi=EPI_DGRAD, add=gout, mask=x_in)
                last = L.entry(c1c.name, "kernel")
            if bucket_cb is not None:
                self._join_side()   # (a bucket's weight gradients come from the side stream)
            done_upto(last.offset + last.size)
            cur = nxt
        # ---- stem: max-pool backward with conv1's ReLU mask, the stem BN, s2d-domain wgrad
        H1, H2 = self.H1, self.H2
        gpool = self.gbuf[cur][: B * H2 * H2 * 64].view(B, H2, H2, 64)
        gi = (cur + 1) % nbuf
        gc1 = self.gbuf[gi][: B * H1 * H1 * 64].view(B, H1, H1, 64)
        s = L.stem
        self._before_write(("g", gi))
        N.maxpool_bwd_f32(gpool, self.pidx[:B], self.c1[:B], gc1)
        self._bn_bwd(gc1, self.zs[:B], s, B * H1 * H1, gc1)
        W(N.wgrad_f32, self.x2[:B], 4, 4, 1, 0, gc1, self.stem_dw2, reads=(("g", gi),))
        W(N.stem_wgrad_fold, self.stem_dw2, self._gv(s.name, 64, 147), 64)
        self._join_side()
        done_upto(L.kernels_end)
        prof.pop()
        if bucket_cb is not None:
            while nb[0] < len(bks):
                bucket_cb(nb[0])
                nb[0] += 1
        return self.stats
