"""HIP execution engine for ResNet-50 on MI355X: explicit forward/backward schedule.

No autograd tape on the GPU path.  The whole training step is a fixed sequence of native
kernel launches over preallocated NHWC bf16 activation buffers (sized once for the batch),
with fp32 master parameters, gradients and optimizer state in flat buffers:

  forward  : stem_im2col (preprocess fused) -> igemm(stem) -> maxpool -> 16 bottleneck
             blocks (3 or 4 igemm launches each; frozen BN + bias + residual + ReLU folded
             into epilogues; conv1 and the projection conv0 share one launch) -> GAP ->
             igemm(dense, fp32) -> softmax-xent (fwd+bwd fused)
  backward : per layer wgrad (fp32 atomics into the flat gradient buffer) + colsum +
             dgrad igemm whose epilogue applies the ReLU mask of the layer below and adds
             the residual gradient; conv1+conv0 dgrad is ONE GEMM over a K-concatenation;
             then wgrad_finalize (dW *= BN scale, dgamma partials) and bn_grad (per-channel).
  buckets  : `bucket_cb(i)` fires as soon as gradient bucket i (a contiguous slice of the
             flat buffer) has been fully produced on the compute stream, so a DP strategy
             can all-reduce it while backward continues.

Reference parity: the Keras graph of imagenet-resnet50.py:51-67 (see models/reference.py
for the fp32 oracle and tests/test_gpu_engine.py for the parity checks).
"""
from __future__ import annotations

import os
import struct
from typing import Callable, Dict, List, Optional

import torch

from ..ops.native import require_native
from ..utils import profiling as prof
from ..utils.envopts import opt
from .resnet50 import BN_EPS, ParamLayout

_PREP_FMT = "<6i2q8i"
STEM_K = 256   # 4x4 taps x 16 channels of the space-to-depth stem
_FIN_FMT = "<5i"
_CRED_FMT = "<q4i"
_BNG_FMT = "<9i"
_FUSE_FMT = "<16iq"   # FuseLayer (csrc/kernels/kernels.h)
E = "PDDL_ENGINE"     # the engine's fusion / schedule switches (utils/envopts.py KEYS)


def _ceil(a, b):
    return (a + b - 1) // b * b


class HipEngine:
    BN_MODES = ("frozen",)   # HipEngineBNTrain (models/engine_bn.py) runs bn_mode="train"
    FUSE_PROJ_OK = True     # projection blocks: conv3 + shortcut conv as one dual-source GEMM
    FUSE_BWD_OK = True      # stage-2/3 conv3 backward: dgrad + wgrad in one launch (bwd1x1.hip)
    FUSE_STEM_OK = True     # stem conv + BN + ReLU + max-pool forward in one launch (stem.hip)
    TWO_STREAM_OK = True
    DEFER_OK = True         # segmented graphs may defer the side work into side graphs (_side_run)
    C64_OK = True           # stage-2 3x3 convs on the row-tile kernels (conv3x3c64.hip)
    C64_MIN_M = 262144      # ... from 4 x 256 CUs x 256-pixel tiles up (b >= 84 at 56 x 56)
    C3C1_OK = True          # stage-2 boundaries: conv3 + next conv1 fused (c3c1.hip)
    S2C_OK = True           # blocks feeding a downsampling block store only their stride-2 grid
    TWO_STREAM_MAX_BATCH = 1024
    # Engines whose steps replay from HIP graphs run ONE stream (two_stream=1 forces the side
    # stream into their graphs).  The runtime launches a single-stream graph from pre-built
    # packets (~0.5 us per kernel; R = 8 b32 host loop 1.6 ms) but a multi-branch one node by node
    # (~3.5 us; 6.2 ms) through its parallel-stream table -- and that path faults (a freed stream
    # in the table, SIGSEGV at +0xaee41) on the first launch of a fresh multi-branch executable
    # once the process has created, replayed and destroyed replica graphs: deterministic in-process
    # repro in profiles/r6_graph_repro.txt.  Cost where the branches paid: segmented Mirrored
    # b256 12.95 vs 12.2 ms (b32: 4.45 one stream vs 4.85-5.00 two, eager 4.36).  The segmented
    # replica graphs (graphed="segmented") get the overlap back without branches: each segment's
    # weight gradients become a single-stream SIDE graph replayed on the side stream after the
    # segment, concurrently with the next one (b32 -15.5 % -> -4 % of eager, b256 -3 %:
    # profiles/r6_mirror_seg_side.txt).
    GRAD_RING = 5           # two-stream: gradient buffers per kind, so the data-gradient chain can run
                            # up to four blocks ahead of the weight gradients still reading older ones
                            # (b32: 3 -> 5 buffers 4.21 -> 4.17 ms eager, 4.17 -> 4.05 ms graphed)
    GRAD_RING_SMALL = 16    # ... and at batches <= 64, where a whole stage's data gradients outrun
                            # its weight gradients: b32 eager 3.90 (5) -> 3.82 (8) -> 3.77 (12) ->
                            # 3.75 ms (16), 24 / 32 no better; b256 within noise from 5 to 24
                            # (round 5, gpurun_out/gr_*); 16 x 51 MB of ring at b32.  Engines whose
                            # step replays from HIP graphs keep GRAD_RING (build_engine graphed=True):
                            # b32 graph 3.90 -> 4.08 ms, PS workers 6.72k -> 6.50k img/s with 16

    def __init__(self, layout: ParamLayout, batch: int, crop: int = 224, image_size: int = 224,
                 device="cuda", bn_mode: str = "frozen", num_classes: int = 1000, bitmask: Optional[bool] = None,
                 grad_ring: Optional[int] = None, graphed=False):
        self._grad_ring = grad_ring   # None: GRAD_RING_SMALL at batches <= 64, else GRAD_RING
        # graphed: steps replay from HIP graphs -- True: one stream (see TWO_STREAM_MAX_BATCH);
        # "segmented": bucket-segmented graphs (train/graph.py SegmentedStepGraphs) with the weight
        # gradients deferred into a single-stream SIDE graph per segment (see _side_run)
        self.graphed = bool(graphed)
        self.defer_side = (graphed == "segmented" and bool(opt(E, "seg_side", True)) and self.TWO_STREAM_OK
                           and self.DEFER_OK)
        self._defer = None            # capture-time list of deferred side-stream closures
        if bn_mode not in self.BN_MODES:
            raise ValueError(f"{type(self).__name__} runs bn_mode in {self.BN_MODES}, not {bn_mode!r} "
                             "(use make_hip_engine)")
        self.bn_mode = bn_mode
        self.N = require_native()
        self.L = layout
        self.device = torch.device(device)
        self.batch = batch
        self.crop = crop
        self.image_size = image_size
        self.num_classes = num_classes
        self.ncls_pad = _ceil(num_classes, 64)
        if bitmask is None:
            bitmask = opt(E, "bitmask", True)
        self.bitmask = bool(bitmask)
        assert struct.calcsize(_PREP_FMT) == self.N.PREP_LAYER_BYTES
        assert struct.calcsize(_FIN_FMT) == self.N.FIN_LAYER_BYTES
        assert struct.calcsize(_BNG_FMT) == self.N.BNGRAD_LAYER_BYTES
        assert struct.calcsize(_FUSE_FMT) == self.N.FUSE_LAYER_BYTES
        assert struct.calcsize(_CRED_FMT) == self.N.COLRED_LAYER_BYTES
        dev = self.device
        L = layout
        self.params = torch.zeros(L.total, dtype=torch.float32, device=dev)
        # ---- per-channel bookkeeping (folded scale / shift, colsum, dgamma partials)
        self.ch: Dict[str, int] = {}
        off = 0
        for c in L.convs:
            self.ch[c.name] = off
            off += c.cout
        self.ch["dense"] = off
        off += _ceil(num_classes, 8)
        # fused projection blocks (conv3 + shortcut conv as one dual-source GEMM, no shortcut
        # activation in HBM): their own folded affine slots (scale 1, shift b3 + b0)
        self.fuse_proj = self.FUSE_PROJ_OK and opt(E, "fuse_proj", True)
        # stage-2/3 conv3 backward as one launch (bwd1x1.hip: data + weight gradient from one read
        # of the 256 / 512-channel gradient; needs the ReLU bitmasks)
        fb = opt(E, "fuse_bwd", 1)
        self.fuse_bwd = self.FUSE_BWD_OK and self.bitmask and fb != 0
        self._fuse_bwd3 = fb != 2
        self._fuse_bwd_s2 = opt(E, "fuse_bwd_s2", True)
        # stem conv + max-pool forward as one launch (stem.hip): conv1's output never reaches HBM
        self.fuse_stem = self.FUSE_STEM_OK and opt(E, "fuse_stem", True) and crop <= 250
        # stage-2 3x3 convs (64 -> 64) on the persistent row-tile kernels (conv3x3c64.hip) at
        # batches where every CU streams several row tiles through its windows
        self.c64 = self.C64_OK and opt(E, "c64", True)
        self.c64w = self.c64 and opt(E, "c64w", True)
        self.c64_min_m = opt(E, "c64_min_m", self.C64_MIN_M)
        # stage-2 block boundaries: conv3 + the next block's conv1 in one launch (c3c1.hip)
        self.c3c1 = opt(E, "c3c1", 1) if self.C3C1_OK else 0
        # stage-2 backward boundaries: the next block's conv1 data gradient computed inside this
        # block's fused conv3 backward (bwd1x1 pre form), its 256-channel result never re-read
        self.c1pre = self.C3C1_OK and opt(E, "c1pre", True)
        # blocks whose output feeds a downsampling block (conv2_block3, conv3_block4, conv4_block6):
        # every consumer of that output (the next block's stride-2 conv1 and shortcut, forward and
        # weight gradient, and its ReLU mask) reads only the even rows / columns, so conv3 runs on
        # the compact quarter and stores only it (3/4 fewer conv3 rows and output bytes)
        self.s2c = self.S2C_OK and self.bitmask and opt(E, "s2c", True)
        for b in L.blocks:
            if b.proj:
                self.ch["fuse:" + b.name] = off
                off += 4 * b.filters
        self.nch = _ceil(off, 64)
        # ---- one zeroed-per-step workspace: grads | colsum | dgamma_raw | stats
        n_tr = L.n_trainable
        nst = 64 * STEM_K
        self.ws = torch.zeros(n_tr + 2 * self.nch + 64 + nst, dtype=torch.float32, device=dev)
        self.grads = self.ws[:n_tr]
        self.colsum = self.ws[n_tr:n_tr + self.nch]
        self.dgr = self.ws[n_tr + self.nch:n_tr + 2 * self.nch]
        self.stats = self.ws[n_tr + 2 * self.nch:n_tr + 2 * self.nch + 2]
        o = n_tr + 2 * self.nch + 64
        self.stem_dw2 = self.ws[o:o + nst].view(64, STEM_K)   # s2d-domain stem weight grad
        self.scale = torch.ones(self.nch, dtype=torch.float32, device=dev)
        self.shift = torch.zeros(self.nch, dtype=torch.float32, device=dev)
        self._build_weight_tables()
        self._alloc_acts(batch)
        # split-K workspace of the small-M layers (igemm.hip: stage 5 at small batches, the Dense
        # head), this engine's own (N.splitk_use makes it current for the launching thread)
        self.splitk_ws = torch.empty(self.N.splitk_default_floats(self.device.index or 0), dtype=torch.float32,
                                     device=dev)
        # two-stream backward (small batches, where single kernels underfill the chip): the weight
        # gradients run on a side stream concurrently with the data-gradient chain.
        # PDDL_ENGINE two_stream=1 / 0 forces it; default on up to TWO_STREAM_MAX_BATCH images.
        self.two_stream = self._two_stream_wanted(batch)
        self.side = torch.cuda.Stream(dev) if self.two_stream and dev.type == "cuda" else None
        self._pending, self._last_side = {}, None
        self._evpool, self._evi = [], 0   # fork/join events (see _event)
        self._prep_evs, self._dgrad_ready = None, None   # (after_update's dgrad-weight fork)

    # ------------------------------------------------------------------ tables
    def _build_weight_tables(self):
        L = self.L
        wf: Dict[str, int] = {}
        off = 0
        for c in L.convs:
            kpad = STEM_K if c is L.stem else _ceil(c.k * c.k * c.cin, 64)
            wf[c.name] = off
            off += c.cout * kpad
        wf["dense"] = off
        off += self.num_classes * 2048
        fuse_rows, fuse_max = [], 0
        for b in L.blocks:   # fused projection forward weights [4f][f + cin]
            if b.proj:
                c3, c0 = b.convs["3"], b.convs["0"]
                wf["fuse:" + b.name] = off
                off += c3.cout * (c3.cin + c0.cin)
                g3, be3, m3, v3 = self._fold_offsets(c3)
                g0, be0, m0, v0 = self._fold_offsets(c0)
                fuse_rows.append(struct.pack(_FUSE_FMT, c3.cout, c3.cin, c0.cin, L.off(c3.name, "kernel"),
                                             L.off(c0.name, "kernel"), L.off(c3.name, "bias"), g3, be3, m3, v3,
                                             L.off(c0.name, "bias"), g0, be0, m0, v0, self.ch["fuse:" + b.name],
                                             wf["fuse:" + b.name]))
                fuse_max = max(fuse_max, c3.cout * (c3.cin + c0.cin))
        # dgrad weights: [cin][R][S][ld]; a projection block's conv1 and conv0 share rows
        wd: Dict[str, int] = {}
        wd_ld: Dict[str, int] = {}
        for b in L.blocks:
            if b.proj:
                c1, c0 = b.convs["1"], b.convs["0"]
                ld = c1.cout + c0.cout
                wd[c1.name], wd[c0.name] = off, off + c1.cout
                wd_ld[c1.name] = wd_ld[c0.name] = ld
                off += c1.cin * ld
            else:
                c1 = b.convs["1"]
                wd[c1.name], wd_ld[c1.name] = off, c1.cout
                off += c1.cin * c1.cout
            for k in ("2", "3"):
                c = b.convs[k]
                wd[c.name], wd_ld[c.name] = off, c.cout
                off += c.cin * c.k * c.k * c.cout
        wd["dense"], wd_ld["dense"] = off, self.ncls_pad
        off += 2048 * self.ncls_pad
        self.wbf = torch.zeros(off, dtype=torch.bfloat16, device=self.device)
        self.wf, self.wd, self.wd_ld = wf, wd, wd_ld
        # prep table
        rows = []
        max_el = 0
        for c in L.convs + ["dense"]:
            if c == "dense":
                name, cout, R, cin = "dense", self.num_classes, 1, 2048
                kpad = 2048
                bias, gam, bet, mu, var = L.off("dense", "bias"), -1, -1, -1, -1
                wd_off, ld = wd["dense"], wd_ld["dense"]
            else:
                name, cout, R, cin = c.name, c.cout, c.k, c.cin
                kpad = STEM_K if c is L.stem else _ceil(R * R * cin, 64)
                bias = L.off(c.name, "bias")
                gam, bet, mu, var = self._fold_offsets(c)
                wd_off, ld = wd.get(c.name, -1), wd_ld.get(c.name, 0)
            mode = 1 if c is L.stem else 0
            rows.append(struct.pack(_PREP_FMT, L.off(name, "kernel"), cout, R, R, cin, kpad, wf[name], wd_off, ld,
                                    bias, gam, bet, mu, var, self.ch[name], mode))
            max_el = max(max_el, cout * kpad)
        self._prep_tab = self._dev_table(rows)
        self._prep_n = len(rows)
        self._prep_max = max_el
        self._fuse_tab = self._dev_table(fuse_rows)
        self._fuse_n, self._fuse_max = len(fuse_rows), fuse_max
        # finalize table rows per layer, bn-grad table
        self._fin_rows: Dict[str, bytes] = {}
        for c in L.convs:
            self._fin_rows[c.name] = struct.pack(_FIN_FMT, L.off(c.name, "kernel"), c.cout, c.k * c.k * c.cin,
                                                 self.ch[c.name], self.ch[c.name])
        self._fin_tabs: Dict[str, torch.Tensor] = {}
        self._fin_rows_n: Dict[str, int] = {}   # widest layer of each table (finalize grid rows)
        for b in L.blocks:
            keys = ["3", "2", "1", "0"] if b.proj else ["3", "2", "1"]
            self._fin_tabs[b.name] = self._dev_table([self._fin_rows[b.convs[k].name] for k in keys])
            self._fin_rows_n[b.name] = max(b.convs[k].cout for k in keys)
        self._fin_tabs["stem"] = self._dev_table([self._fin_rows[L.stem.name]])
        self._fin_rows_n["stem"] = L.stem.cout
        bg = []
        for c in L.convs:
            cs = self.ch[c.name]
            for b in L.blocks:   # conv0 of a projection block shares conv3's gradient
                if b.proj and b.convs["0"].name == c.name:
                    cs = self.ch[b.convs["3"].name]
            bg.append(struct.pack(_BNG_FMT, c.cout, self.ch[c.name], L.off(c.name, "bias"), L.off(c.bn, "gamma"),
                                  L.off(c.bn, "beta"), L.off(c.bn, "moving_mean"), L.off(c.bn, "moving_variance"),
                                  cs, self.ch[c.name]))
        bg.append(struct.pack(_BNG_FMT, self.num_classes, self.ch["dense"], L.off("dense", "bias"), -1, -1, -1, -1,
                              self.ch["dense"], -1))
        self._bng_tab = self._dev_table(bg)
        self._bng_n = len(bg)

    def _fold_offsets(self, c):
        """BN parameters folded into a conv's forward epilogue / dgrad weights (frozen BN)."""
        L = self.L
        return (L.off(c.bn, "gamma"), L.off(c.bn, "beta"), L.off(c.bn, "moving_mean"),
                L.off(c.bn, "moving_variance"))

    def _dev_table(self, rows: List[bytes]) -> torch.Tensor:
        buf = bytearray(b"".join(rows))
        return torch.frombuffer(buf, dtype=torch.uint8).clone().to(self.device)

    # ------------------------------------------------------------------ buffers
    def _alloc_acts(self, B):
        L, dev = self.L, self.device
        bf = dict(dtype=torch.bfloat16, device=dev)
        crop = self.crop
        H1 = (crop + 6 - 7) // 2 + 1
        H2 = (H1 + 2 - 3) // 2 + 1
        self.H1, self.H2 = H1, H2
        self.Hs = (crop + 6) // 2
        assert crop % 2 == 0, "crop must be even (space-to-depth stem)"
        self.stem_x2 = torch.empty(B, self.Hs, self.Hs, 16, **bf)
        # (the fused stem never materialises conv1's output)
        self.c1 = None if self.fuse_stem else torch.empty(B, H1, H1, 64, **bf)
        self.pool = torch.empty(B, H2, H2, 64, **bf)
        self.pidx = torch.empty(B, H2, H2, 64, dtype=torch.uint8, device=dev)
        u8 = dict(dtype=torch.uint8, device=dev)
        # ReLU masks of every masked dgrad as bitmasks (1 bit per element instead of re-reading
        # the 16-bit activation): written by the forward epilogues, read by the dgrad epilogues
        self.bits: Dict[str, Dict[str, torch.Tensor]] = {}
        self.pool_bits = torch.empty(B, H2, H2, 8, **u8) if self.bitmask else None
        self.acts: Dict[str, Dict[str, torch.Tensor]] = {}
        H = H2
        inner = 0
        outer = B * H1 * H1 * 64
        self.geo = {}
        for b in L.blocks:
            f = b.filters
            Ho = (H - 1) // b.stride + 1
            Hq = self._out_dim(L.blocks.index(b), Ho)
            a = {"y1": torch.empty(B, Ho, Ho, f, **bf), "y2": torch.empty(B, Ho, Ho, f, **bf),
                 "out": torch.empty(B, Hq, Hq, 4 * f, **bf)}
            if b.proj and not self.fuse_proj:
                a["sc"] = torch.empty(B, Ho, Ho, 4 * f, **bf)
            self.acts[b.name] = a
            if self.bitmask:
                self.bits[b.name] = {"y1": torch.empty(B, Ho, Ho, f // 8, **u8),
                                     "y2": torch.empty(B, Ho, Ho, f // 8, **u8),
                                     "out": torch.empty(B, Hq, Hq, f // 2, **u8)}
            self.geo[b.name] = (H, Ho)
            inner = max(inner, B * Ho * Ho * f)
            outer = max(outer, B * H * H * b.cin, B * Ho * Ho * 4 * f)
            H = Ho
        self.H5 = H
        # (set before _alloc_acts runs; the subclasses' engines keep one stream)
        ring0 = self._grad_ring or (self.GRAD_RING_SMALL if B <= 64 else self.GRAD_RING)
        ring = opt(E, "grad_ring", ring0) if self._two_stream_wanted(B) else 1
        # deferred side graphs read a segment's data gradients while the next segment runs: no
        # gradient buffer is reused within a step (one per block, + head and stem)
        deep = self.defer_side and self._two_stream_wanted(B)
        if deep:
            ring = len(L.blocks) + 2
        self.gbuf = [torch.empty(outer, **bf) for _ in range(max(2, ring))]
        self.g1bufs = [torch.empty(inner, **bf) for _ in range(ring)]
        self.g2bufs = [torch.empty(inner, **bf) for _ in range(ring)]
        self.g1buf, self.g2buf = self.g1bufs[0], self.g2bufs[0]
        # compact (stride-2 grid) copies of the output gradient / conv2-output gradient of every
        # block feeding a downsampling block (see _s2_fed)
        gc, g2c = 1, 1
        for bi in self._s2_fed():
            b = L.blocks[bi]
            Hc = self.geo[b.name][1] // 2 + self.geo[b.name][1] % 2
            gc = max(gc, B * Hc * Hc * 4 * b.filters)
            g2c = max(g2c, B * Hc * Hc * b.filters)
        self.gcbuf = torch.empty(gc, **bf)
        self.gcbufs = {bi: torch.empty(gc, **bf) for bi in self._s2_fed()} if deep else None
        # full-resolution output gradient of those blocks, zeroed ONCE: the downsampling block's
        # dgrad writes only the stride-2 grid positions (up2 = 2), the off-grid zeros persist
        self.s2full = {}
        for bi in self._s2_fed():
            b = L.blocks[bi]
            Hb = self.geo[b.name][1]
            self.s2full[bi] = torch.zeros(B * Hb * Hb * 4 * b.filters, **bf)
        self.s2g2full = {bi: torch.zeros(B * self.geo[L.blocks[bi].name][1] ** 2 * L.blocks[bi].filters, **bf)
                         for bi in self._s2_fed()}   # (same for their conv2-output gradient)
        self.g2cbuf = torch.empty(g2c, **bf)
        self.g2cbufs = {bi: torch.empty(g2c, **bf) for bi in self._s2_fed()} if deep else None
        self.pooled = torch.empty(B, 2048, **bf)
        self.logits = torch.empty(B, self.num_classes, dtype=torch.float32, device=dev)
        self.dlogits = torch.zeros(B, self.ncls_pad, **bf)
        self.dpooled = torch.empty(B, 2048, **bf)
        self.labels_dev = torch.zeros(B, dtype=torch.int64, device=dev)
        self.cap = B
        self._cred = {}
        self.colpart = torch.empty(self._colred(B)[2], dtype=torch.float32, device=dev)

    def _out_dim(self, bi, Ho) -> int:
        """Spatial size of block bi's stored output: its stride-2 grid when it feeds a
        downsampling block and the compact form is on (see s2c), else Ho."""
        return (Ho + 1) // 2 if self.s2c and bi in self._s2_fed() else Ho

    def _x_geom(self, bi, H, stride):
        """(stored size, stride to apply) of block bi's input: the previous block's output is
        already the stride-2 grid when it was stored compact."""
        if bi > 0 and self.s2c and bi - 1 in self._s2_fed():
            return (H + 1) // 2, 1
        return H, stride

    def _s2_fed(self):
        """Blocks whose output feeds a stride-2 projection block (ResNet v1 downsamples in the
        first 1x1 conv and the shortcut, both reading only the even rows / columns): their output
        gradient is zero off the stride-2 grid, so their conv3 weight / data gradients and conv2
        weight gradient run on the compact quarter (conv2_block3, conv3_block4, conv4_block6)."""
        bl = self.L.blocks
        return {bi for bi in range(len(bl) - 1) if bl[bi + 1].proj and bl[bi + 1].stride == 2}

    def _colred(self, B):
        """Partial column-sum regions of every fused producer for batch B:
        (offsets by consumer layer, device reduce table, total floats)."""
        if B in self._cred:
            return self._cred[B]
        N, L = self.N, self.L
        offs, rows, off = {}, [], 0

        def add(layer, nrows, C):
            nonlocal off
            offs[layer] = off
            rows.append(struct.pack(_CRED_FMT, off, nrows, C, self.ch[layer], 0))
            off += nrows * C
        blocks = L.blocks
        s2 = self._s2_fed()
        add(blocks[-1].convs["3"].name, B, 2048)                              # gap_bwd
        for bi in range(len(blocks) - 1, -1, -1):
            b = blocks[bi]
            H, Ho = self.geo[b.name]
            M = B * Ho * Ho
            f = b.filters
            Mc = M
            if bi in s2:       # c3 dgrad runs on the compact stride-2 grid
                Hc = Ho // 2 + Ho % 2
                Mc = B * Hc * Hc
            if self._bwd_fused(bi, b, s2) or self._bwd_fused_s2(bi, b, s2):     # fused c3 backward -> g2
                add(b.convs["2"].name, N.bwd1x1_partial_rows(Mc, 4 * f, f), f)
            else:
                add(b.convs["2"].name, N.igemm_partial_rows(Mc, f, 4 * f), f)     # c3 dgrad -> g2
            if self._use_c64(f, M, Ho, self.bitmask):                           # c2 dgrad -> g1
                add(b.convs["1"].name, N.conv3x3c64_partial_rows(M), f)
            else:
                add(b.convs["1"].name, N.igemm_partial_rows(M, f, 9 * f), f)
            if bi > 0:                                                           # c1 dgrad -> g_out(prev)
                if self._pre_fused(bi, s2):   # (computed inside block bi-1's fused conv3 backward)
                    add(blocks[bi - 1].convs["3"].name, N.bwd1x1_partial_rows(M, 256, 64), b.cin)
                else:
                    add(blocks[bi - 1].convs["3"].name, N.igemm_partial_rows(M, b.cin, 5 * f if b.proj else f), b.cin)
        if self.fuse_stem:   # (fused pool backward + conv1 weight gradient: one partial row per workgroup)
            add(L.stem.name, N.stem_pool_bwd_partial_rows(B, self.H2), 64)
        else:
            add(L.stem.name, N.maxpool_bwd_partial_rows(B, self.H1, self.H1, 64), 64)
        res = (offs, self._dev_table(rows), off, len(rows))
        self._cred[B] = res
        return res

    # ------------------------------------------------------------------ params
    def init(self, seed=0):
        self.L.init_params(self.params, seed)
        self.after_update()

    def after_update(self):
        """Refresh bf16 forward / dgrad weights and folded BN affine from the fp32 master.  With a
        side stream (eager steps), the dgrad weights are prepared there, under the next forward;
        the backward waits for them before its first data gradient (b32: 43 us off the step)."""
        side = self.side
        if side is None or self._defer is not None or torch.cuda.is_current_stream_capturing():
            self.N.prep(self.params, self._prep_tab, self._prep_n, self._prep_max, self.wbf, self.scale, self.shift,
                        BN_EPS)
        else:
            self.N.prep(self.params, self._prep_tab, self._prep_n, self._prep_max, self.wbf, self.scale, self.shift,
                        BN_EPS, parts=1)
            if self._prep_evs is None:
                self._prep_evs = (torch.cuda.Event(), torch.cuda.Event())
            fork, done = self._prep_evs
            fork.record(torch.cuda.current_stream(self.device))
            side.wait_event(fork)
            with torch.cuda.stream(side):
                self.N.prep(self.params, self._prep_tab, self._prep_n, self._prep_max, self.wbf, self.scale,
                            self.shift, BN_EPS, parts=2)
            done.record(side)
            self._dgrad_ready = done
        if self.fuse_proj and self._fuse_n:
            self.N.prep_fuse(self.params, self._fuse_tab, self._fuse_n, self._fuse_max, self.wbf, self.scale,
                             self.shift, BN_EPS)

    def _wf(self, name, rows, k):
        o = self.wf[name]
        return self.wbf[o:o + rows * k].view(rows, k)

    def _bwd_fused_s2(self, bi, b, s2):   # the stride-2-grid form (block feeding a downsampling block)
        return self.fuse_bwd and self._fuse_bwd_s2 and bi in s2 and (b.filters == 64 or (b.filters == 128 and self._fuse_bwd3))

    def _pre_fused(self, bi, s2) -> bool:
        """Block bi's conv1 data gradient runs inside block bi-1's fused conv3 backward (bwd1x1 pre
        form): both stage-2 (64-channel), block bi not a projection block, block bi-1 on the
        stride-1 fused conv3 backward."""
        L = self.L
        if not self.c1pre or bi < 1 or not self.bitmask:
            return False
        b, pb = L.blocks[bi], L.blocks[bi - 1]
        return (b.filters == 64 and pb.filters == 64 and not b.proj and b.stride == 1 and bi - 1 not in s2
                and self._bwd_fused(bi - 1, pb, s2))

    def _bwd_fused(self, bi, b, s2):
        # stage 2 (256 <- 64 channels) and stage 3 (512 <- 128); PDDL_ENGINE fuse_bwd=2: stage 2 only
        return self.fuse_bwd and bi not in s2 and (b.filters == 64 or (b.filters == 128 and self._fuse_bwd3))

    def _use_c64(self, f, M, W, bits=True) -> bool:
        return self.c64 and f == 64 and W + 2 <= 64 and M >= self.c64_min_m and bits

    def _c3c1_ok(self, b, nb) -> bool:
        """Fuse block b's conv3 with block nb's conv1 (c3c1.hip): 64-channel stride-1 boundaries out of
        a plain block (stage 2: conv2_block2 -> 3), not into a projection block.  (Out of the fused
        projection block conv2_block1, K = 128, it measured no gain: 2.77 ms fused vs 1.87 + 0.90 ms
        separate at b2560, profiles/r4_c3c1.txt.)"""
        return (bool(self.c3c1) and nb is not None and b.filters == 64 and nb.filters == 64 and not b.proj
                and not nb.proj and nb.stride == 1)

    def _c2_wgrad(self, W, y1, g2, c2n, f, B, Ho, g2_n):
        """Weight gradient of a bottleneck's stride-1 3x3 conv (on the side stream when two-stream)."""
        if self.c64w and self._use_c64(f, B * Ho * Ho, Ho) and Ho + 2 <= 64:
            W(self.N.conv3x3c64_wgrad, y1, g2, self._gview(c2n, f, 9 * f), reads=(g2_n,))
        else:
            W(self.N.wgrad, y1, Ho, Ho, 3, 3, 1, 1, Ho, Ho, g2, None, 0, self._gview(c2n, f, 9 * f), 9 * f, 0,
              reads=(g2_n,))

    def _wdv(self, name, cin, k):
        o = self.wd[name]
        return self.wbf[o:o + cin * k].view(cin, k)

    def _gview(self, name, rows, k):
        o = self.L.off(name, "kernel")
        return self.grads[o:o + rows * k].view(rows, k)

    # ------------------------------------------------------------------ forward
    def _stem_mode(self, training, crop_offset):
        if self.crop == self.image_size:
            return 0, 0, 0
        if self.crop > self.image_size or not training:
            return 1, 0, 0
        return 2, crop_offset[0], crop_offset[1]

    def _forward(self, images, B, training, flip, crop_offset):
        self.N.splitk_use(self.splitk_ws)   # this engine's split-K workspace, for this thread's launches
        N, L = self.N, self.L
        mode, oy, ox = self._stem_mode(training, crop_offset)
        x2 = self.stem_x2[:B]
        crop_dev = None
        if mode == 2 and isinstance(crop_offset, torch.Tensor):   # device offsets (graph capture)
            crop_dev, oy, ox = crop_offset, 0, 0
        N.stem_s2d(images, flip if training else None, mode, self.crop, self.crop, oy, ox, x2, crop_dev)
        H1, H2, Hs = self.H1, self.H2, self.Hs
        s = L.stem
        pool = self.pool[:B]
        use_bits = training and self.bitmask
        chs = self.ch[s.name]
        if self.fuse_stem:
            N.stem_pool_fwd(x2, self._wf(s.name, 64, STEM_K), self.scale[chs:chs + 64], self.shift[chs:chs + 64],
                            pool, self.pidx[:B], self.pool_bits[:B] if use_bits else None)
        else:
            c1 = self.c1[:B]
            N.igemm(x2, None, Hs, Hs, 4, 4, 1, 0, H1, H1, self._wf(s.name, 64, STEM_K), 0,
                    self.scale[chs:], self.shift[chs:], None, None, None, c1, 1,
                    None, 0, 0, 0, 0, 0, None, None)
            N.maxpool_fwd(c1, pool, self.pidx[:B], self.pool_bits[:B] if use_bits else None)
        x = pool
        c1_done = False   # this block's conv1 already ran inside the previous block's c3c1 launch
        for bi, b in enumerate(L.blocks):
            a = self.acts[b.name]
            bt = {k: v[:B] for k, v in self.bits[b.name].items()} if use_bits else {}
            H, Ho = self.geo[b.name]
            f, cin = b.filters, b.cin
            y1, y2, out = a["y1"][:B], a["y2"][:B], a["out"][:B]
            c1n = b.convs["1"].name
            ch1 = self.ch[c1n]
            Hx, sx = self._x_geom(bi, H, b.stride)
            if c1_done:
                res = x
            elif b.proj and self.fuse_proj:
                # conv1 alone; the shortcut conv runs inside conv3's GEMM (second A source = the block
                # input at the block's stride, K = f + cin, both BN scales folded into the weights), so
                # the shortcut activation is never written and re-read as a residual
                N.igemm(x, None, Hx, Hx, 1, 1, sx, 0, Ho, Ho, self._wf(c1n, f, cin), 0,
                        self.scale[ch1:], self.shift[ch1:], None, None, None, y1, 1, None, 0, 0, 0, 0, 0, None,
                        bt.get("y1"))
                res = None
            elif b.proj:
                N.igemm(x, None, Hx, Hx, 1, 1, sx, 0, Ho, Ho, self._wf(c1n, 5 * f, cin), 0,
                        self.scale[ch1:], self.shift[ch1:], None, None, None, y1, 1, a["sc"][:B], 0, f, 0, 0, 0,
                        None, bt.get("y1"))
                res = a["sc"][:B]
            else:
                N.igemm(x, None, H, H, 1, 1, 1, 0, Ho, Ho, self._wf(c1n, f, cin), 0,
                        self.scale[ch1:], self.shift[ch1:], None, None, None, y1, 1, None, 0, 0, 0, 0, 0, None,
                        bt.get("y1"))
                res = x
            c2 = b.convs["2"].name
            if self._use_c64(f, B * Ho * Ho, Ho):
                N.conv3x3c64(y1, self._wf(c2, f, 9 * f), 0, y2, scale=self.scale[self.ch[c2]:],
                             shift=self.shift[self.ch[c2]:], bits=bt.get("y2"))
            else:
                N.igemm(y1, None, Ho, Ho, 3, 3, 1, 1, Ho, Ho, self._wf(c2, f, 9 * f), 0,
                        self.scale[self.ch[c2]:], self.shift[self.ch[c2]:], None, None, None, y2, 1, None, 0, 0, 0,
                        0, 0, None, bt.get("y2"))
            c3 = b.convs["3"].name
            nb = L.blocks[bi + 1] if bi + 1 < len(L.blocks) else None
            c1_done = False
            if self._c3c1_ok(b, nb):
                # conv3 of this block + conv1 of the next in one launch: the next conv1 reads this
                # block's output from LDS (c3c1.hip)
                an = self.acts[nb.name]
                btn = {k: v[:B] for k, v in self.bits[nb.name].items()} if use_bits else {}
                c1x = nb.convs["1"].name
                k3 = self.ch[c3]
                N.c3c1(y2, self._wf(c3, 4 * f, f), self.scale[k3:], self.shift[k3:], res, out, bt.get("out"),
                       self._wf(c1x, nb.filters, nb.cin), self.scale[self.ch[c1x]:], self.shift[self.ch[c1x]:],
                       an["y1"][:B], btn.get("y1"))
                c1_done = True
            elif b.proj and self.fuse_proj:
                fz = "fuse:" + b.name
                N.igemm(y2, x, Ho, Ho, 1, 1, 1, 0, Ho, Ho, self._wf(fz, 4 * f, f + cin), 0,
                        self.scale[self.ch[fz]:], self.shift[self.ch[fz]:], None, None, None, out, 1, None, 0, 0, 0,
                        0, 0, None, bt.get("out"))
            elif self._out_dim(bi, Ho) != Ho:
                # feeds a downsampling block: conv3 on the stride-2 grid only (1x1 stride-2 gather
                # of y2, residual read at the grid positions of the full-resolution block input)
                Hq = self._out_dim(bi, Ho)
                N.igemm(y2, None, Ho, Ho, 1, 1, 2, 0, Hq, Hq, self._wf(c3, 4 * f, f), 0,
                        self.scale[self.ch[c3]:], self.shift[self.ch[c3]:], res, None, None, out, 1, None, 0, 0, 1,
                        Ho, Ho, None, bt.get("out"))
            else:
                N.igemm(y2, None, Ho, Ho, 1, 1, 1, 0, Ho, Ho, self._wf(c3, 4 * f, f), 0,
                        self.scale[self.ch[c3]:], self.shift[self.ch[c3]:], res, None, None, out, 1, None, 0, 0, 0,
                        0, 0, None, bt.get("out"))
            x = out
        pooled = self.pooled[:B]
        N.gap_fwd(x, pooled)
        logits = self.logits[:B]
        chd = self.ch["dense"]
        N.igemm(pooled.view(B, 1, 1, 2048), None, 1, 1, 1, 1, 1, 0, 1, 1, self._wf("dense", self.num_classes, 2048), 2,
                self.scale[chd:], self.shift[chd:], None, None, None, logits, 0, None, 0, 0, 0, 0, 0, None, None)
        return x

    def _labels(self, labels, B):
        lab = self.labels_dev[:B]
        if labels.data_ptr() != lab.data_ptr():   # (a graphed step loads straight into labels_dev)
            lab.copy_(labels, non_blocking=True)
        return lab

    # ------------------------------------------------------------------ two-stream backward
    def _two_stream_wanted(self, batch) -> bool:
        ts = opt(E, "two_stream", "auto")
        if ts != "auto":
            return self.TWO_STREAM_OK and ts == "1"
        return self.TWO_STREAM_OK and batch <= self.TWO_STREAM_MAX_BATCH and (not self.graphed or self.defer_side)

    def _event(self):
        """The next fork/join event of this step, from a pool the engine owns for its whole
        life: the i-th record of every step reuses the i-th event (a wait binds to the record
        made before it, so reuse after the wait is safe), so a step -- eager or captured --
        creates and destroys no HIP events."""
        i = self._evi
        self._evi += 1
        if i == len(self._evpool):
            self._evpool.append(torch.cuda.Event())
        return self._evpool[i]

    def _side_run(self, fn, *args, reads=()):
        """Launch a weight-gradient kernel on the side stream, ordered after everything enqueued
        on the compute stream so far; `reads` names the gradient buffers it reads, which the
        compute stream must not overwrite before it is done (see _before_write).

        Deferred (a segmented capture, begin_defer): the call is queued instead, and the capture
        records the queue of each segment as a single-stream side graph that the replay runs
        after that segment's main graph, concurrently with the next segment.  No fork / join
        events inside any graph (the runtime launches single-stream graphs from pre-built packets;
        its multi-branch launch path faults: train/graph.py replay_stream), and no buffer hazards:
        the deferred engine's gradient buffers are never reused within a step (_alloc_acts)."""
        if self._defer is not None:
            self._defer.append((fn, args))
            return
        if self.side is None:
            fn(*args)
            return
        main = torch.cuda.current_stream(self.device)
        ev = self._event()
        ev.record(main)
        self.side.wait_event(ev)
        with torch.cuda.stream(self.side):
            fn(*args)
        done = self._event()
        done.record(self.side)
        for r in reads:
            self._pending[r] = done
        self._last_side = done

    def _before_write(self, *bufs):
        """The compute stream is about to overwrite these gradient buffers: wait for the side
        stream's last reader of each."""
        if self.side is None or self._defer is not None:
            return
        main = torch.cuda.current_stream(self.device)
        for b in bufs:
            ev = self._pending.pop(b, None)
            if ev is not None:
                main.wait_event(ev)

    def _bucket_ready(self, cb, i):
        """Report bucket i complete.  Two streams: its gradients come from both streams, so the
        side stream first waits for the compute stream and the callback runs with the SIDE stream
        current -- whatever it enqueues or records (an all-reduce, an optimizer update) is
        ordered after both, and the compute stream never blocks on the side stream."""
        if self.side is None or self._defer is not None:
            cb(i)
            return
        if getattr(cb, "needs_join", False):   # (e.g. a graph capture cut at the bucket boundary)
            self._join_side()
            cb(i)
            return
        ev = self._event()
        ev.record(torch.cuda.current_stream(self.device))
        self.side.wait_event(ev)
        with torch.cuda.stream(self.side):
            cb(i)
        done = self._event()
        done.record(self.side)
        self._last_side = done

    def begin_defer(self):
        """Queue side-stream work from now on (segmented capture; take_deferred drains it)."""
        assert self.side is not None and self.defer_side
        self._defer = []

    def take_deferred(self):
        q, self._defer = self._defer, []
        return q

    def end_defer(self):
        left, self._defer = self._defer, None
        assert not left, "deferred side work left uncaptured"

    def _join_side(self):
        if self.side is None or self._last_side is None:
            return
        torch.cuda.current_stream(self.device).wait_event(self._last_side)
        self._pending.clear()
        self._last_side = None

    # ------------------------------------------------------------------ train step
    def forward_backward(self, images, labels, gscale, flip=None, crop_offset=(0, 0),
                         bucket_cb: Optional[Callable[[int], None]] = None, buckets=None):
        N, L = self.N, self.L
        B = images.shape[0]
        assert B <= self.cap, "batch larger than the engine's buffers"
        self._pending, self._last_side = {}, None
        self._evi = 0
        # (clearing the workspace on the side stream under the forward measured no gain at b32:
        # 3.604-3.624 vs 3.602-3.606 ms, round 6)
        self.ws.zero_()
        lab = self._labels(labels, B)
        prof.push("step/forward")
        x5 = self._forward(images, B, True, flip, crop_offset)
        prof.pop()
        prof.push("step/backward")
        logits = self.logits[:B]
        dl = self.dlogits[:B]
        N.softmax_xent(logits, lab, self.num_classes, float(gscale), dl, self.stats[0:1], self.stats[1:2])
        if self._dgrad_ready is not None:   # the dgrad weights after_update prepared on the side stream
            if not torch.cuda.is_current_stream_capturing():   # (a capture starts synchronized)
                torch.cuda.current_stream(self.device).wait_event(self._dgrad_ready)
            self._dgrad_ready = None

        # bucket readiness tracking (kernels region is filled in layout order)
        bks = buckets if buckets is not None else []
        nb = [0]
        W = self._side_run

        def done_upto(off):
            while bucket_cb is not None and nb[0] < len(bks) - 1 and bks[nb[0]][1] <= off:
                self._bucket_ready(bucket_cb, nb[0])
                nb[0] += 1

        # ---- head
        pooled = self.pooled[:B]
        chd = self.ch["dense"]
        W(N.wgrad, pooled.view(B, 1, 1, 2048), 1, 1, 1, 1, 1, 0, 1, 1, dl, None, 0,
          self._gview("dense", self.num_classes, 2048), 2048, 0)
        N.colsum(dl, self.num_classes, self.colsum[chd:])
        dpooled = self.dpooled[:B]
        N.igemm(dl.view(B, 1, 1, self.ncls_pad), None, 1, 1, 1, 1, 1, 0, 1, 1,
                self._wdv("dense", 2048, self.ncls_pad), 1, None, None, None, None, None, dpooled, 0,
                None, 0, 0, 0, 0, 0, None, None)
        e = L.entry("dense", "kernel")
        done_upto(e.offset + e.size)
        cur = 0
        H5 = self.H5
        blocks = L.blocks
        gout = self.gbuf[cur][: B * H5 * H5 * 2048].view(B, H5, H5, 2048)
        coffs, ctab, _, cn = self._colred(B)
        cp = self.colpart

        def part(layer):
            return cp[coffs[layer]:]
        self._before_write("gbuf0")
        N.gap_bwd(dpooled, x5, gout, part(blocks[-1].convs["3"].name))
        s2 = self._s2_fed()
        pre = None   # the previous (deeper) block's deferred conv1 data gradient (bwd1x1 pre form)
        # ---- blocks (column sums of every produced gradient are fused into its producer)
        for bi in range(len(blocks) - 1, -1, -1):
            b = blocks[bi]
            a = self.acts[b.name]
            H, Ho = self.geo[b.name]
            f, cin = b.filters, b.cin
            x_in = self.acts[blocks[bi - 1].name]["out"][:B] if bi > 0 else self.pool[:B]
            # conv2_block1's input is the max-pool output y: the stem's ReLU mask at every argmax
            # position equals (y > 0), so it is applied here instead of re-reading conv1's output
            mask_in = x_in
            y1m, y2m = a["y1"][:B], a["y2"][:B]
            if self.bitmask:
                mask_in = self.bits[blocks[bi - 1].name]["out"][:B] if bi > 0 else self.pool_bits[:B]
                y1m, y2m = self.bits[b.name]["y1"][:B], self.bits[b.name]["y2"][:B]
            cs_in = part(blocks[bi - 1].convs["3"].name) if bi > 0 else None
            y1, y2 = a["y1"][:B], a["y2"][:B]
            gout = (self.s2full[bi] if bi in s2 else self.gbuf[cur])[: B * Ho * Ho * 4 * f].view(B, Ho, Ho, 4 * f)
            gout_n = f"s2f{bi}" if bi in s2 else f"gbuf{cur}"
            c1n, c2n, c3n = b.convs["1"].name, b.convs["2"].name, b.convs["3"].name
            rk = bi % len(self.g2bufs)
            g2 = (self.s2g2full[bi] if bi in s2 else self.g2bufs[rk])[: B * Ho * Ho * f].view(B, Ho, Ho, f)
            g2_n = f"s2g2f{bi}" if bi in s2 else f"g2_{rk}"
            assert pre is None or self._bwd_fused(bi, b, s2)
            pre_next = None
            if bi in s2:
                # gout is zero off the stride-2 grid (the next block reads only even rows /
                # columns); its compact copy `gc` came from that block's dgrad epilogue
                Hc = Ho // 2 + Ho % 2
                gc = (self.gcbufs[bi] if self.gcbufs else self.gcbuf)[: B * Hc * Hc * 4 * f].view(B, Hc, Hc, 4 * f)
                g2c = (self.g2cbufs[bi] if self.g2cbufs else self.g2cbuf)[: B * Hc * Hc * f].view(B, Hc, Hc, f)
                if self._bwd_fused_s2(bi, b, s2):   # one read of gc: data + weight gradient
                    self._before_write(g2_n, "g2c")
                    N.bwd1x1(gc, y2, self._wdv(c3n, f, 4 * f), y2m, g2, part(c2n), self._gview(c3n, 4 * f, f), g2c)
                else:
                    W(N.wgrad, y2, Ho, Ho, 1, 1, 2, 0, Hc, Hc, gc, None, 0, self._gview(c3n, 4 * f, f), f, 0,
                      reads=("gc",))
                    self._before_write(g2_n, "g2c")
                    N.igemm(gc, None, Hc, Hc, 1, 1, 1, 0, Hc, Hc, self._wdv(c3n, f, 4 * f), 1, None, None, None, y2m,
                            None, g2, 0, g2c, 0, 0, 2, Ho, Ho, part(c2n), None)
                W(N.wgrad, y1, Ho, Ho, 3, 3, 2, 1, Hc, Hc, g2c, None, 0, self._gview(c2n, f, 9 * f), 9 * f, 0,
                  reads=("g2c",))
            elif self._bwd_fused(bi, b, s2):
                # conv3: data and weight gradient from one read of gout
                self._before_write(g2_n)
                if pre is not None:
                    # gout itself is computed per tile from the next block's conv1 gradient
                    # (pre form): this block's output gradient is written once, never re-read
                    N.bwd1x1(pre["add"], y2, self._wdv(c3n, f, 4 * f), y2m, g2, part(c2n), self._gview(c3n, 4 * f, f),
                             g1=pre["g1"], w1d=pre["w1d"], gmask=pre["gmask"], gx=gout, colsum_gx=pre["cs"])
                else:
                    N.bwd1x1(gout, y2, self._wdv(c3n, f, 4 * f), y2m, g2, part(c2n), self._gview(c3n, 4 * f, f))
                self._c2_wgrad(W, y1, g2, c2n, f, B, Ho, g2_n)
            else:
                # conv3
                W(N.wgrad, y2, Ho, Ho, 1, 1, 1, 0, Ho, Ho, gout, None, 0, self._gview(c3n, 4 * f, f), f, 0,
                  reads=(gout_n,))
                self._before_write(g2_n)
                N.igemm(gout, None, Ho, Ho, 1, 1, 1, 0, Ho, Ho, self._wdv(c3n, f, 4 * f), 1, None, None, None, y2m,
                        None, g2, 0, None, 0, 0, 0, 0, 0, part(c2n), None)
                # conv2 (3x3)
                self._c2_wgrad(W, y1, g2, c2n, f, B, Ho, g2_n)
            g1 = self.g1bufs[rk][: B * Ho * Ho * f].view(B, Ho, Ho, f)
            self._before_write(f"g1_{rk}")
            if self._use_c64(f, B * Ho * Ho, Ho, self.bitmask):
                N.conv3x3c64(g2, self._wdv(c2n, f, 9 * f), 1, g1, bits=y1m, colsum=part(c1n))
            else:
                N.igemm(g2, None, Ho, Ho, 3, 3, 1, 1, Ho, Ho, self._wdv(c2n, f, 9 * f), 1, None, None, None, y1m,
                        None, g1, 0, None, 0, 0, 0, 0, 0, part(c1n), None)
            # conv1 (+ conv0)
            nxt = (cur + 1) % len(self.gbuf)
            gx = self.gbuf[nxt][: B * H * H * cin].view(B, H, H, cin)
            gx_n = [f"gbuf{nxt}"]
            if b.proj:
                Hx, sx = self._x_geom(bi, H, b.stride)
                W(N.wgrad, x_in, Hx, Hx, 1, 1, sx, 0, Ho, Ho, g1, gout, f, self._gview(c1n, 5 * f, cin), cin, 0,
                  reads=(f"g1_{rk}", gout_n))
                W(N.wgrad_finalize, self.params, self.grads, self._fin_tabs[b.name], 4, self.scale, self.dgr,
                  self._fin_rows_n[b.name])
                gxc, up2 = None, 1 if b.stride == 2 else 0
                if bi - 1 in s2:   # compact copy for the previous block's stride-2-grid passes
                    gxc = (self.gcbufs[bi - 1] if self.gcbufs else self.gcbuf)[: B * Ho * Ho * cin].view(B, Ho, Ho, cin)
                    # grid positions only, into the pre-zeroed full-resolution buffer (saves the
                    # 3/4 zero-fill writes: conv3_block1 c1 dgrad 942 -> 681 us at b1024)
                    gx = self.s2full[bi - 1][: B * H * H * cin].view(B, H, H, cin)
                    gx_n = [f"s2f{bi - 1}", "gc"]
                    up2 = 3 if Hx != H else 2   # (3: the stored block input and its mask are compact)
                self._before_write(*gx_n)
                N.igemm(g1, gout, Ho, Ho, 1, 1, 1, 0, Ho, Ho, self._wdv(c1n, cin, 5 * f), 1, None, None, None,
                        mask_in, None, gx, 0, gxc, 0, 0, up2, H, H, cs_in, None)
                last = L.entry(b.convs["0"].name, "kernel")
            else:
                W(N.wgrad, x_in, H, H, 1, 1, 1, 0, Ho, Ho, g1, None, 0, self._gview(c1n, f, cin), cin, 0,
                  reads=(f"g1_{rk}",))
                W(N.wgrad_finalize, self.params, self.grads, self._fin_tabs[b.name], 3, self.scale, self.dgr,
                  self._fin_rows_n[b.name])
                self._before_write(*gx_n)
                if self._pre_fused(bi, s2):   # deferred into block bi-1's fused conv3 backward
                    pre_next = {"add": gout, "g1": g1, "w1d": self._wdv(c1n, cin, f), "gmask": mask_in, "cs": cs_in}
                else:
                    N.igemm(g1, None, Ho, Ho, 1, 1, 1, 0, Ho, Ho, self._wdv(c1n, cin, f), 1, None, None, None,
                            mask_in, gout, gx, 0, None, 0, 0, 0, 0, 0, cs_in, None)
                last = L.entry(c1n, "kernel")
            done_upto(last.offset + last.size)
            cur = nxt
            pre, pre_next = pre_next, None
        # ---- stem (space-to-depth wgrad, folded back to 7x7x3)
        H1, H2, Hs = self.H1, self.H2, self.Hs
        gpool = self.gbuf[cur][: B * H2 * H2 * 64].view(B, H2, H2, 64)
        s = L.stem
        if self.fuse_stem:
            # pool backward + conv1 weight gradient in one launch: conv1's gradient stays in LDS
            N.stem_pool_bwd(self.stem_x2[:B], gpool, self.pidx[:B], self.stem_dw2, part(s.name))
            W(N.stem_wgrad_fold, self.stem_dw2, self._gview(s.name, 64, 147), 64)
        else:
            gcn = (cur + 1) % len(self.gbuf)
            gc1 = self.gbuf[gcn][: B * H1 * H1 * 64].view(B, H1, H1, 64)
            self._before_write(f"gbuf{gcn}")
            N.maxpool_bwd(gpool, self.pidx[:B], None, gc1, part(s.name))
            W(N.wgrad, self.stem_x2[:B], Hs, Hs, 4, 4, 1, 0, H1, H1, gc1, None, 0, self.stem_dw2, STEM_K, 0)
            W(N.stem_wgrad_fold, self.stem_dw2, self._gview(s.name, 64, 147), 64)
        W(N.wgrad_finalize, self.params, self.grads, self._fin_tabs["stem"], 1, self.scale, self.dgr,
          self._fin_rows_n["stem"])
        # (the column-sum fold reads only what the compute stream wrote: it runs under the side
        # stream's last weight gradients, before the join)
        N.colsum_reduce(cp, ctab, cn, self.colsum)
        self._join_side()
        done_upto(L.kernels_end)
        # (deferred: after the finalizes that wrote dgr, in the last side graph, which waits for
        # the main graph holding colsum_reduce)
        (W if self._defer is not None else (lambda f, *a: f(*a)))(
            N.bn_grad, self.params, self.grads, self._bng_tab, self._bng_n, self.colsum, self.dgr, self.scale, BN_EPS)
        prof.pop()
        if bucket_cb is not None:
            while nb[0] < len(bks):
                self._bucket_ready(bucket_cb, nb[0])
                nb[0] += 1
        return self.stats

    @torch.no_grad()
    def evaluate(self, images, labels):
        B = images.shape[0]
        assert B <= self.cap
        self.stats.zero_()
        lab = self._labels(labels, B)
        self._forward(images, B, False, None, (0, 0))
        N = self.N
        N.softmax_xent(self.logits[:B], lab, self.num_classes, 0.0, self.dlogits[:B], self.stats[0:1],
                       self.stats[1:2])
        return self.stats


def make_hip_engine(layout: ParamLayout, batch: int, bn_mode: str = "frozen", **kw) -> HipEngine:
    """HIP engine for the BN mode: frozen (reference `training=False`, folded) or train."""
    if bn_mode == "train":
        from .engine_bn import HipEngineBNTrain
        return HipEngineBNTrain(layout, batch, bn_mode="train", **kw)
    return HipEngine(layout, batch, bn_mode=bn_mode, **kw)
