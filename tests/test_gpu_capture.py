"""Whole-engine HIP-graph capture at the reference's per-replica batch (32, imagenet-resnet50.py:46,
imagenet-resnet50-mirror.py:54) and the engine under the headline (b2560) kernel plan.

The kernel-level capture test (test_gpu_kernels.py) captures single kernels; these capture the
full training step the way the entry scripts do -- GraphedTrainStep (single strategy) and
SegmentedStepGraphs (a Mirrored / MWMS replica: segments cut at the gradient buckets, with the
two-stream backward forked across them, plus the optimizer graph) -- and compare the replayed
trajectory with eager steps of an identically initialised engine."""
import pytest

from pddl.utils.envopts import with_opt
import torch

pytestmark = pytest.mark.gpu


def _inputs(steps, B, hw, seed=21):
    g = torch.Generator().manual_seed(seed)
    img = torch.randint(0, 256, (steps, B, hw, hw, 3), dtype=torch.uint8, generator=g).cuda()
    lab = torch.randint(0, 1000, (steps, B), generator=g).cuda()
    flip = torch.randint(0, 2, (steps, B), dtype=torch.uint8, generator=g).cuda()
    return img, lab, flip


def _engine(crop, B, graphed=False):
    from pddl.models.engine import HipEngine
    from pddl.models.resnet50 import ParamLayout
    from pddl.train.optim import make_optimizer
    eng = HipEngine(ParamLayout(), B, crop=crop, image_size=224, graphed=graphed)
    eng.init(seed=13)
    return eng, make_optimizer("adam", eng, lr=1e-3)


def _eager(crop, B, img, lab, flip):
    eng, opt = _engine(crop, B)
    losses = []
    for i in range(img.shape[0]):
        s = eng.forward_backward(img[i], lab[i], 1.0 / B, flip=flip[i])
        losses.append(s[0].item() / B)
        opt.step()
        eng.after_update()
    torch.cuda.synchronize()
    return losses, eng.params.clone(), eng


def _close(l_ref, p_ref, losses, params):
    assert all(abs(a - b) <= 1e-3 * abs(a) for a, b in zip(l_ref, losses)), (l_ref, losses)
    # (weight gradients are summed with fp32 atomics in no fixed order; Adam amplifies the
    # near-zero-gradient noise, so replays are compared like two eager runs)
    r = ((p_ref - params).norm() / p_ref.norm()).item()
    assert r < 2e-3, r


@pytest.mark.parametrize("crop,c64", [(224, False), (244, False), (224, True)])
def test_whole_engine_graph_capture_at_reference_batch(monkeypatch, crop, c64):
    """B = 32 at crops 224 and 244 (the Q1 up-size), and 224 with the stage-2 64-channel 3x3
    kernels forced on (their full-grid launches are what b >= 84 selects; a zero-byte memset
    node in their data gradient once made capture fail with invalid argument): 4 steps as
    (1) eager, (2) GraphedTrainStep = 1 eager + capture + 3 replays, (3) SegmentedStepGraphs
    replayed segment by segment + the optimizer graph, each from the same initial weights."""
    from pddl.train.graph import GraphedTrainStep, SegmentedStepGraphs
    if c64:
        monkeypatch.setenv("PDDL_ENGINE", with_opt("PDDL_ENGINE", "c64_min_m", "1"))
    B, steps = 32, 4
    img, lab, flip = _inputs(steps, B, 224)
    l_ref, p_ref, eng_ref = _eager(crop, B, img, lab, flip)
    assert eng_ref.side is not None          # b32: the two-stream backward is what runs
    if c64:
        assert eng_ref._use_c64(64, B * 56 * 56, 56, eng_ref.bitmask)

    # (2) the single strategy's whole-step graph
    eng, opt = _engine(crop, B)
    gs = GraphedTrainStep(eng, opt, B, (224, 224), 1.0 / B)
    losses = [gs(img[i], lab[i], flip[i], (0, 0))[0].item() / B for i in range(steps)]
    torch.cuda.synchronize()
    assert gs.graph is not None and opt.iterations == steps
    _close(l_ref, p_ref, losses, eng.params)

    # (3) a Mirrored replica's segmented graphs (what _LocalReplicas replays between all-reduces)
    eng, opt = _engine(crop, B)
    bks = eng.L.buckets(25.0)
    s = eng.forward_backward(img[0], lab[0], 1.0 / B, flip=flip[0], buckets=bks)   # eager first step
    losses = [s[0].item() / B]
    opt.step()
    eng.after_update()
    sg = SegmentedStepGraphs(eng, opt, B, (224, 224), 1.0 / B, bks)
    sg.capture()
    assert sg.captured and len(sg.segments) == len(bks) >= 2 and eng.side is not None
    for i in range(1, steps):
        sg.load(img[i], lab[i], flip[i], (0, 0))
        for k in range(len(bks)):
            sg.replay_segment(k)
        sg.replay_optimizer()
        losses.append(sg.stats[0].item() / B)
    torch.cuda.synchronize()
    assert opt.iterations == steps
    _close(l_ref, p_ref, losses, eng.params)


def test_segmented_single_stream_matches_two_stream():
    """The segmented replica graphs with the side stream forked inside each segment, with the
    single-stream schedule (two_stream=False) and with the weight gradients deferred into one
    single-stream side graph per segment (the Mirrored replicas' default, HipEngine
    graphed="segmented") replay the same gradient -- incl. the BN / bias gradients the last side
    graph's bn_grad writes."""
    from pddl.train.graph import SegmentedStepGraphs
    B = 32
    img, lab, flip = _inputs(1, B, 224, seed=4)
    out = []
    for mode in ("forked", "one", "deferred"):
        eng, opt = _engine(224, B, graphed="segmented" if mode == "deferred" else False)
        bks = eng.L.buckets(25.0)
        eng.forward_backward(img[0], lab[0], 1.0 / B, flip=flip[0], buckets=bks)
        sg = SegmentedStepGraphs(eng, opt, B, (224, 224), 1.0 / B, bks, two_stream=False if mode == "one" else None)
        sg.capture()
        assert (eng.side is not None) == (mode != "one")
        assert sg.deferred == (mode == "deferred")
        if sg.deferred:
            assert len(sg.side_segments) == len(bks) and any(x is not None for x in sg.side_segments)
            assert eng._defer is None
        sg.load(img[0], lab[0], flip[0], (0, 0))
        for k in range(len(bks)):
            sg.replay_segment(k)
        torch.cuda.synchronize()
        out.append(eng.grads.clone())
    for o in out[:2]:
        r = ((o - out[1]).norm() / out[1].norm()).item()
        assert r < 1e-4, r
    r = ((out[2] - out[1]).norm() / out[1].norm()).item()
    assert r < 1e-4, r


def test_engine_headline_kernel_plan_within_noise_floor(monkeypatch):
    """The engine at a small batch forced onto the b2560 plan: single-stream backward, split-K
    off (so the short-K 1x1 layers take the persistent full-grid ring kernel), 64-channel
    full-grid 3x3 kernels -- bounded by the fp32 reference's own
    bf16-point noise floor like the default small-batch plan
    (test_gpu_engine.test_engine_matches_bf16_point_reference_within_its_noise_floor)."""
    from pddl.ops.native import require_native
    from test_gpu_engine import test_engine_matches_bf16_point_reference_within_its_noise_floor as parity
    N = require_native()
    monkeypatch.setenv("PDDL_ENGINE", with_opt("PDDL_ENGINE", "two_stream", "0"))
    monkeypatch.setenv("PDDL_ENGINE", with_opt("PDDL_ENGINE", "c64_min_m", "1"))
    N.set_variant("igemm_splitk", 0)
    try:
        # (the 8-phase 256x256 tiles need more than one round of tiles on the chip, which no
        # small batch has: test_gpu_kernels covers them kernel by kernel)
        assert N.igemm_plan(4 * 49, 512, 4608)[2] == 1 and N.igemm_plan(4 * 196, 256, 2304)[2] == 1
        parity(224, 224)
    finally:
        N.set_variant("igemm_splitk", 1)
