"""HIP engine with train-mode BatchNormalization (batch statistics), `bn_mode="train"`.

The reference runs every BN layer in inference mode during training (`base_model(x,
training=False)`, imagenet-resnet50.py:57), which the default HipEngine folds
into the conv epilogues.  This engine is the Keras `training=True` variant (FusedBatchNormV3:
batch mean / biased variance for normalisation, Bessel-corrected variance into the moving
statistics, momentum 0.99, epsilon 1.001e-5) on the same MFMA kernels plus csrc/kernels/bn.hip:

  forward, per conv : igemm -> z = conv + bias (bf16) with fused per-wave (sum, sum^2) partials
                      -> colsum_reduce -> bn_stats (mean, 1/sigma, moving stats)
                      -> bn_apply: y = relu(bn(z) [+ x | + bn0(z0)]) + ReLU bitmask
  backward, per conv: (dgrad of the next conv applies the ReLU bitmask, adds the residual
                      gradient) -> bn_bwd_reduce (sum g, sum g*(z - mean)) -> bn_bwd_apply
                      (dz; dgamma, dbeta, dbias) -> wgrad(x, dz) and dgrad(dz, W^T);
                      for BN1 / BN2 (fed by the conv2 / conv3 dgrads) the two sums are fused
                      into the dgrad epilogue (it reads z instead of a separate pass over g, z)
  A projection block's BN3 and shortcut BN0 share one reduce and one apply pass (same g).

Parity: tests/test_gpu_bn_train.py compares against models/reference.py (bn_mode="train") and
plain PyTorch fp32 references of every BN kernel.
"""
from __future__ import annotations

import struct
from typing import Callable, Dict, Optional

import torch

from .engine import STEM_K, HipEngine
from ..utils import profiling as prof
from .resnet50 import BN_EPS, BN_MOMENTUM, ParamLayout

_STAT_FMT = "<8if i"   # BnStatLayer: C, sum_off, sq_off, ch, gamma, beta, mm, mv, count, pad


class HipEngineBNTrain(HipEngine):
    BN_MODES = ("train",)
    FUSE_BWD_OK = False    # (its conv3 dgrad carries the fused BN-backward sums)
    FUSE_PROJ_OK = False   # (batch statistics: the shortcut's BN cannot be folded into weights)
    FUSE_STEM_OK = False   # (conv1's batch statistics need its raw output)
    # weight gradients on the side stream up to TWO_STREAM_MAX_BATCH (eager steps; its graphed
    # steps keep one stream: no deferred side graphs for this schedule)
    DEFER_OK = False
    C64_OK = False         # (train-mode BN needs the batch statistics from the conv epilogue)
    C3C1_OK = False
    S2C_OK = False

    def __init__(self, layout: ParamLayout, batch: int, **kw):
        kw.setdefault("bn_mode", "train")
        # deeper gradient rings up to b256 (b256 ring 3 / 5 / 8 / 12 / 16: 20.70 / 20.64 / 20.52 /
        # 20.45 / 20.45 ms, round 6); larger batches keep GRAD_RING (12 x 1.6 GB of ring at b1024)
        if kw.get("grad_ring") is None and batch <= 256:
            kw["grad_ring"] = 12
        # (needed by _alloc_acts, which the base constructor calls)
        self.L = layout
        self._launch_nn = self._fwd_launches()
        self._acc_off: Dict[str, int] = {}
        off = 0
        for key, nn in self._launch_nn.items():
            self._acc_off[key] = off
            off += 2 * nn
        self._stat_cache = {}
        super().__init__(layout, batch, **kw)
        assert struct.calcsize(_STAT_FMT) == self.N.BNSTAT_LAYER_BYTES
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        self.bn_mean = torch.zeros(self.nch, **f32)
        self.bn_inv = torch.ones(self.nch, **f32)
        self.bn_scale = torch.ones(self.nch, **f32)
        self.bn_shift = torch.zeros(self.nch, **f32)
        self.bcoef = torch.zeros(3 * self.nch, **f32)   # backward (A, B, C) per channel
        # zeroed per step: forward (sum, sum^2) of every igemm launch | backward sum g | sum g*(z-mean)
        self.bws = torch.zeros(off + 2 * self.nch, **f32)
        self._bws_off = off
        self._bwd_tabs = {}
        self.acc = self.bws[:off]
        self.bsg = self.bws[off:off + self.nch]
        self.bsgx = self.bws[off + self.nch:off + 2 * self.nch]
        self._eval_tab = self._stat_table([(c, 0, 0) for c in layout.convs], count=1.0)
        # dense bias gradient (the only bn_grad row left in this mode)
        L = layout
        self._bng_dense = self._dev_table([struct.pack("<9i", self.num_classes, self.ch["dense"],
                                                       L.off("dense", "bias"), -1, -1, -1, -1, self.ch["dense"], -1)])

    # ------------------------------------------------------------------ tables
    def _fold_offsets(self, c):
        # nothing folded: forward weights are W, dgrad weights W^T, epilogue z = acc + bias
        return -1, -1, -1, -1

    def _fwd_launches(self):
        """igemm launches that produce BN inputs: key -> GEMM N (conv1+conv0 share one)."""
        L = self.L
        out = {L.stem.name: 64}
        for b in L.blocks:
            f = b.filters
            out[b.convs["1"].name] = 5 * f if b.proj else f
            out[b.convs["2"].name] = f
            out[b.convs["3"].name] = 4 * f
        return out

    def _stat_table(self, items, count: float) -> torch.Tensor:
        """items: (conv, acc offset of its launch, column offset within the launch's N)."""
        L = self.L
        rows = []
        for c, aoff, col in items:
            nn = self._launch_nn.get(c.name, None)
            if nn is None:   # conv0 shares conv1's launch
                nn = self._launch_nn[c.name.replace("_0_conv", "_1_conv")]
            rows.append(struct.pack(_STAT_FMT, c.cout, aoff + col, aoff + nn + col, self.ch[c.name],
                                    L.off(c.bn, "gamma"), L.off(c.bn, "beta"), L.off(c.bn, "moving_mean"),
                                    L.off(c.bn, "moving_variance"), float(count), 0))
        return self._dev_table(rows)

    def _launch_tables(self, B):
        """Per forward igemm launch: (partial rows, colsum_reduce table, bn_stats table, #BN, max C)."""
        if B in self._stat_cache:
            return self._stat_cache[B]
        N, L = self.N, self.L
        res = {}
        geo = {L.stem.name: (B * self.H1 * self.H1, 64, STEM_K)}
        convs = {L.stem.name: [L.stem]}
        for b in L.blocks:
            H, Ho = self.geo[b.name]
            M = B * Ho * Ho
            f = b.filters
            geo[b.convs["1"].name] = (M, 5 * f if b.proj else f, b.cin)
            convs[b.convs["1"].name] = [b.convs["1"], b.convs["0"]] if b.proj else [b.convs["1"]]
            geo[b.convs["2"].name] = (M, f, 9 * f)
            convs[b.convs["2"].name] = [b.convs["2"]]
            geo[b.convs["3"].name] = (M, 4 * f, f)
            convs[b.convs["3"].name] = [b.convs["3"]]
        max_part = 0
        for key, (M, nn, K) in geo.items():
            rows = N.igemm_partial_rows(M, nn, K)
            max_part = max(max_part, rows * 2 * nn)
            aoff = self._acc_off[key]
            cred = self._dev_table([struct.pack("<q4i", 0, rows, 2 * nn, aoff, 0)])
            items, col = [], 0
            for c in convs[key]:
                items.append((c, aoff, col))
                col += c.cout
            st = self._stat_table(items, count=float(M))
            res[key] = (cred, st, len(items), max(c.cout for c in convs[key]), M)
        for b in L.blocks:   # fused BN-backward dgrads (c3 -> g2, c2 -> g1): [rows][2 * f]
            H, Ho = self.geo[b.name]
            M, f = B * Ho * Ho, b.filters
            for K in (4 * f, 9 * f):
                max_part = max(max_part, N.igemm_partial_rows(M, f, K, True) * 2 * f)
        res["_max_part"] = max_part
        self._stat_cache[B] = res
        return res

    # ------------------------------------------------------------------ buffers
    def _alloc_acts(self, B):
        super()._alloc_acts(B)
        self.s2g2full = {}   # (the frozen engine's compact conv2-gradient path is not used here; s2full is:
        #                    the downsampling blocks' dgrads write only the stride-2 grid into it)
        L, dev = self.L, self.device
        bf = dict(dtype=torch.bfloat16, device=dev)
        self.zs = torch.empty(B, self.H1, self.H1, 64, **bf)
        self.z: Dict[str, Dict[str, torch.Tensor]] = {}
        for b in L.blocks:
            H, Ho = self.geo[b.name]
            f = b.filters
            z = {"1": torch.empty(B, Ho, Ho, f, **bf), "2": torch.empty(B, Ho, Ho, f, **bf),
                 "3": torch.empty(B, Ho, Ho, 4 * f, **bf)}
            if b.proj:
                z["0"] = torch.empty(B, Ho, Ho, 4 * f, **bf)
            self.z[b.name] = z
        # dz3 of each block, a ring like the other gradient buffers (two-stream backward)
        self.gbuf3s = [torch.empty_like(self.gbuf[0]) for _ in range(len(self.g1bufs))]
        self._stat_cache = {}
        self.partial = torch.empty(self._launch_tables(B)["_max_part"], dtype=torch.float32, device=dev)

    # ------------------------------------------------------------------ forward
    def _chs(self, arr, c):
        o = self.ch[c.name]
        return arr[o:o + c.cout]

    def _conv_bn(self, key, training, tabs, x, H, W, R, S, stride, pad, Ho, Wo, nn, K, out, out2=None, n_split=0):
        """z = conv(x) + bias (+ batch statistics of z when training)."""
        N = self.N
        ch = self.ch[key]
        N.igemm_bn(x, None, H, W, R, S, stride, pad, Ho, Wo, self._wf(key, nn, K), 0, self.scale[ch:], self.shift[ch:],
                   None, None, None, out, 0, out2, 0, n_split, 0, 0, 0, None, None,
                   self.partial if training else None, None, None)
        if training:
            cred, st, nst, maxc, _ = tabs[key]
            N.colsum_reduce(self.partial, cred, 1, self.acc)
            N.bn_stats(self.acc, st, nst, maxc, True, self.params, self.bn_mean, self.bn_inv, self.bn_scale,
                       self.bn_shift, BN_EPS, BN_MOMENTUM)

    def _forward(self, images, B, training, flip, crop_offset):
        self.N.splitk_use(self.splitk_ws)   # this engine's split-K workspace, for this thread's launches
        N, L = self.N, self.L
        tabs = self._launch_tables(B) if training else None
        if not training:   # inference: every BN layer from its moving statistics, one launch
            N.bn_stats(self.acc, self._eval_tab, len(L.convs), 2048, False, self.params, self.bn_mean, self.bn_inv,
                       self.bn_scale, self.bn_shift, BN_EPS, BN_MOMENTUM)
        mode, oy, ox = self._stem_mode(training, crop_offset)
        x2 = self.stem_x2[:B]
        crop_dev = None
        if mode == 2 and isinstance(crop_offset, torch.Tensor):
            crop_dev, oy, ox = crop_offset, 0, 0
        N.stem_s2d(images, flip if training else None, mode, self.crop, self.crop, oy, ox, x2, crop_dev)
        H1, Hs = self.H1, self.Hs
        s = L.stem
        zs = self.zs[:B]
        self._conv_bn(s.name, training, tabs, x2, Hs, Hs, 4, 4, 1, 0, H1, H1, 64, STEM_K, zs)
        c1 = self.c1[:B]
        N.bn_apply(zs, self._chs(self.bn_scale, s), self._chs(self.bn_shift, s), None, None, None, True, c1, None)
        pool = self.pool[:B]
        use_bits = training and self.bitmask
        N.maxpool_fwd(c1, pool, self.pidx[:B], self.pool_bits[:B] if use_bits else None)
        x = pool
        for b in L.blocks:
            a = self.acts[b.name]
            z = {k: v[:B] for k, v in self.z[b.name].items()}
            bt = {k: v[:B] for k, v in self.bits[b.name].items()} if use_bits else {}
            H, Ho = self.geo[b.name]
            f, cin = b.filters, b.cin
            y1, y2, out = a["y1"][:B], a["y2"][:B], a["out"][:B]
            c1c, c2c, c3c = b.convs["1"], b.convs["2"], b.convs["3"]
            if b.proj:
                self._conv_bn(c1c.name, training, tabs, x, H, H, 1, 1, b.stride, 0, Ho, Ho, 5 * f, cin, z["1"],
                              z["0"], f)
            else:
                self._conv_bn(c1c.name, training, tabs, x, H, H, 1, 1, 1, 0, Ho, Ho, f, cin, z["1"])
            N.bn_apply(z["1"], self._chs(self.bn_scale, c1c), self._chs(self.bn_shift, c1c), None, None, None, True,
                       y1, bt.get("y1"))
            self._conv_bn(c2c.name, training, tabs, y1, Ho, Ho, 3, 3, 1, 1, Ho, Ho, f, 9 * f, z["2"])
            N.bn_apply(z["2"], self._chs(self.bn_scale, c2c), self._chs(self.bn_shift, c2c), None, None, None, True,
                       y2, bt.get("y2"))
            self._conv_bn(c3c.name, training, tabs, y2, Ho, Ho, 1, 1, 1, 0, Ho, Ho, 4 * f, f, z["3"])
            if b.proj:
                c0c = b.convs["0"]
                N.bn_apply(z["3"], self._chs(self.bn_scale, c3c), self._chs(self.bn_shift, c3c), z["0"],
                           self._chs(self.bn_scale, c0c), self._chs(self.bn_shift, c0c), True, out, bt.get("out"))
            else:
                N.bn_apply(z["3"], self._chs(self.bn_scale, c3c), self._chs(self.bn_shift, c3c), x, None, None, True,
                           out, bt.get("out"))
            x = out
        pooled = self.pooled[:B]
        N.gap_fwd(x, pooled)
        logits = self.logits[:B]
        chd = self.ch["dense"]
        N.igemm(pooled.view(B, 1, 1, 2048), None, 1, 1, 1, 1, 1, 0, 1, 1, self._wf("dense", self.num_classes, 2048), 2,
                self.scale[chd:], self.shift[chd:], None, None, None, logits, 0, None, 0, 0, 0, 0, 0, None, None)
        return x

    # ------------------------------------------------------------------ backward
    def _bn_layer(self, c, M):
        L = self.L
        return [float(c.cout), float(self.ch[c.name]), float(L.off(c.bn, "gamma")), float(L.off(c.bn, "beta")),
                float(L.off(c.name, "bias")), float(M)]

    def _bn_bwd(self, g, z, c, M, out, z2=None, c2=None, out2=None):
        """dz (and dz2 of the shortcut BN fed by the same g) from g = dL/d(BN output)."""
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

    def _dgrad_bn_bwd(self, g_in, Ho, R, pad, w, mask, g, z, c, M):
        """g = dgrad(g_in) * mask with the BN-backward sums (sum g, sum g*(z - mean)) of conv `c`'s
        BN fused into the dgrad epilogue (stats rows folded into bsg / bsgx: no bn_bwd_reduce
        pass over g and z), then dz = bn_bwd_apply(g, z) in place."""
        N = self.N
        f = c.cout
        N.igemm_bn(g_in, None, Ho, Ho, R, R, 1, pad, Ho, Ho, w, 1, None, None, None, mask, None, g, 0, None, 0, 0,
                   0, 0, 0, None, None, self.partial, z, self._chs(self.bn_mean, c))
        key = (c.name, M)
        tab = self._bwd_tabs.get(key)
        if tab is None:
            rows = N.igemm_partial_rows(M, f, w.shape[1], True)
            o = self._bws_off + self.ch[c.name]
            tab = self._dev_table([struct.pack("<q4i", 0, rows, f, o, 2 * f),
                                   struct.pack("<q4i", f, rows, f, o + self.nch, 2 * f)])
            self._bwd_tabs[key] = tab
        N.colsum_reduce(self.partial, tab, 2, self.bws)
        self._bn_bwd_apply(g, z, c, M, g)

    def _bn_bwd_apply(self, g, z, c, M, out):
        """dz from g once bsg / bsgx of conv `c`'s BN hold (sum g, sum g*(z - mean))."""
        self.N.bn_bwd_apply(g, z, None, self._bn_layer(c, M), [], self.params, self.bn_mean, self.bn_inv, self.bsg,
                            self.bsgx, out, None, self.grads, self.bcoef)

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
        logits = self.logits[:B]
        dl = self.dlogits[:B]
        N.softmax_xent(logits, lab, self.num_classes, float(gscale), dl, self.stats[0:1], self.stats[1:2])
        if self._dgrad_ready is not None:   # the dgrad weights after_update prepared on the side stream
            torch.cuda.current_stream(self.device).wait_event(self._dgrad_ready)
            self._dgrad_ready = None
        self._pending, self._last_side = {}, None
        self._evi = 0
        bks = buckets if buckets is not None else []
        nb = [0]

        def done_upto(off):
            while bucket_cb is not None and nb[0] < len(bks) - 1 and bks[nb[0]][1] <= off:
                self._bucket_ready(bucket_cb, nb[0])
                nb[0] += 1

        # ---- head (as the frozen engine)
        pooled = self.pooled[:B]
        chd = self.ch["dense"]
        N.wgrad(pooled.view(B, 1, 1, 2048), 1, 1, 1, 1, 1, 0, 1, 1, dl, None, 0,
                self._gview("dense", self.num_classes, 2048), 2048, 0)
        N.colsum(dl, self.num_classes, self.colsum[chd:])
        dpooled = self.dpooled[:B]
        N.igemm(dl.view(B, 1, 1, self.ncls_pad), None, 1, 1, 1, 1, 1, 0, 1, 1,
                self._wdv("dense", 2048, self.ncls_pad), 1, None, None, None, None, None, dpooled, 0,
                None, 0, 0, 0, 0, 0, None, None)
        N.bn_grad(self.params, self.grads, self._bng_dense, 1, self.colsum, self.dgr, self.scale, BN_EPS)
        e = L.entry("dense", "kernel")
        done_upto(e.offset + e.size)
        cur = 0
        H5 = self.H5
        blocks = L.blocks
        D, nbuf = len(self.g1bufs), len(self.gbuf)
        W = self._side_run
        gout = self.gbuf[cur][: B * H5 * H5 * 2048].view(B, H5, H5, 2048)
        N.gap_bwd(dpooled, x5, gout, None)
        s2 = self._s2_fed()
        # weight gradients on the side stream (HipEngine._side_run), BN backward and data gradients
        # on the compute stream; ("g", i) / ("s2", bi) / ("z3", j) / ("g2", j) / ("g1", j): gradient
        # buffers a side launch reads, waited for before the compute stream rewrites them
        for bi in range(len(blocks) - 1, -1, -1):
            b = blocks[bi]
            a = self.acts[b.name]
            z = {k: v[:B] for k, v in self.z[b.name].items()}
            H, Ho = self.geo[b.name]
            M = B * Ho * Ho
            f, cin = b.filters, b.cin
            x_in = self.acts[blocks[bi - 1].name]["out"][:B] if bi > 0 else self.pool[:B]
            mask_in = x_in
            y1m, y2m = a["y1"][:B], a["y2"][:B]
            if self.bitmask:
                mask_in = self.bits[blocks[bi - 1].name]["out"][:B] if bi > 0 else self.pool_bits[:B]
                y1m, y2m = self.bits[b.name]["y1"][:B], self.bits[b.name]["y2"][:B]
            y1, y2 = a["y1"][:B], a["y2"][:B]
            gkey = ("s2", bi) if bi in s2 else ("g", cur)
            gout = (self.s2full[bi] if bi in s2 else self.gbuf[cur])[: M * 4 * f].view(B, Ho, Ho, 4 * f)
            j = bi % D
            dz3 = self.gbuf3s[j][: M * 4 * f].view(B, Ho, Ho, 4 * f)
            c1c, c2c, c3c = b.convs["1"], b.convs["2"], b.convs["3"]
            self._before_write(("z3", j))
            if b.proj:   # BN3 and the shortcut BN0 share gout; dz0 overwrites gout in place
                self._bn_bwd(gout, z["3"], c3c, M, dz3, z["0"], b.convs["0"], gout)
            else:
                self._bn_bwd(gout, z["3"], c3c, M, dz3)
            # conv3
            W(N.wgrad, y2, Ho, Ho, 1, 1, 1, 0, Ho, Ho, dz3, None, 0, self._gview(c3c.name, 4 * f, f), f, 0,
              reads=(("z3", j),))
            g2 = self.g2bufs[j][: M * f].view(B, Ho, Ho, f)
            self._before_write(("g2", j))
            self._dgrad_bn_bwd(dz3, Ho, 1, 0, self._wdv(c3c.name, f, 4 * f), y2m, g2, z["2"], c2c, M)
            # conv2 (3x3)
            W(N.wgrad, y1, Ho, Ho, 3, 3, 1, 1, Ho, Ho, g2, None, 0, self._gview(c2c.name, f, 9 * f), 9 * f, 0,
              reads=(("g2", j),))
            g1 = self.g1bufs[j][: M * f].view(B, Ho, Ho, f)
            self._before_write(("g1", j))
            self._dgrad_bn_bwd(g2, Ho, 3, 1, self._wdv(c2c.name, f, 9 * f), y1m, g1, z["1"], c1c, M)
            # conv1 (+ conv0)
            nxt = (cur + 1) % nbuf
            gx = self.gbuf[nxt][: B * H * H * cin].view(B, H, H, cin)
            gx_key = ("g", nxt)
            if b.proj:
                W(N.wgrad, x_in, H, H, 1, 1, b.stride, 0, Ho, Ho, g1, gout, f, self._gview(c1c.name, 5 * f, cin), cin, 0,
                  reads=(("g1", j), gkey))
                up2 = 1 if b.stride == 2 else 0
                if bi - 1 in s2:   # grid positions only, into the pre-zeroed full-resolution buffer
                    gx, up2 = self.s2full[bi - 1][: B * H * H * cin].view(B, H, H, cin), 2
                    gx_key = ("s2", bi - 1)
                self._before_write(gx_key)
                N.igemm(g1, gout, Ho, Ho, 1, 1, 1, 0, Ho, Ho, self._wdv(c1c.name, cin, 5 * f), 1, None, None, None,
                        mask_in, None, gx, 0, None, 0, 0, up2, H, H, None, None)
                last = L.entry(b.convs["0"].name, "kernel")
            else:
                W(N.wgrad, x_in, H, H, 1, 1, 1, 0, Ho, Ho, g1, None, 0, self._gview(c1c.name, f, cin), cin, 0,
                  reads=(("g1", j),))
                self._before_write(gx_key)
                N.igemm(g1, None, Ho, Ho, 1, 1, 1, 0, Ho, Ho, self._wdv(c1c.name, cin, f), 1, None, None, None,
                        mask_in, gout, gx, 0, None, 0, 0, 0, 0, 0, None, None)
                last = L.entry(c1c.name, "kernel")
            done_upto(last.offset + last.size)
            cur = nxt
        # ---- stem
        H1, H2, Hs = self.H1, self.H2, self.Hs
        gpool = self.gbuf[cur][: B * H2 * H2 * 64].view(B, H2, H2, 64)
        gi = (cur + 1) % nbuf
        gc1 = self.gbuf[gi][: B * H1 * H1 * 64].view(B, H1, H1, 64)
        s = L.stem
        self._before_write(("g", gi))
        N.maxpool_bwd(gpool, self.pidx[:B], None, gc1, None)
        self._bn_bwd(gc1, self.zs[:B], s, B * H1 * H1, gc1)
        W(N.wgrad, self.stem_x2[:B], Hs, Hs, 4, 4, 1, 0, H1, H1, gc1, None, 0, self.stem_dw2, STEM_K, 0,
          reads=(("g", gi),))
        W(N.stem_wgrad_fold, self.stem_dw2, self._gview(s.name, 64, 147), 64)
        self._join_side()
        done_upto(L.kernels_end)
        prof.pop()
        if bucket_cb is not None:
            while nb[0] < len(bks):
                self._bucket_ready(bucket_cb, nb[0])
                nb[0] += 1
        return self.stats
