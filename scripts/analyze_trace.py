"""Per-layer breakdown of one training step from a rocprofv3 kernel trace.

    python scripts/analyze_trace.py gpurun_out/prof/run_kernel_trace.csv [batch=1024] [crop=224] [knobs]

Pairs the last complete step's dispatches with the engine's fixed launch schedule and
prints time, TFLOP/s and effective GB/s per launch.
"""
import csv
import os
import sys

sys.path.insert(0, ".")
import pddl  # noqa
from pddl.models.resnet50 import ParamLayout
from pddl.utils.envopts import opt

E = "PDDL_ENGINE"   # the run's engine switches (the schedule follows them)


def schedule(B, crop, fuse=True, fuse_bwd=True, fuse_bwd3=True, fuse_s2=True, fuse_stem=True):
    L = ParamLayout()
    H1 = (crop + 6 - 7) // 2 + 1
    H2 = (H1 + 2 - 3) // 2 + 1
    ev = []
    ev.append(("stem_s2d", "stem", 0, B * H1 * H1 * 4 * 32))
    if fuse_stem:   # conv1 + max-pool in one launch (stem.hip)
        ev.append(("stem_pool", "conv1+pool fwd", 2 * B * H1 * H1 * 256 * 64,
                   B * (H1 + 3) ** 2 * 32 + B * H2 * H2 * 64 * 3, None))
    else:
        ev.append(("igemm", "conv1 fwd", 2 * B * H1 * H1 * 256 * 64, B * H1 * H1 * 64 * 2, (B * H1 * H1, 64, 256)))
        ev.append(("maxpool_fwd", "pool", 0, B * (H1 * H1 + H2 * H2) * 64 * 2))
    H = H2
    geo = []
    c3c1_on = opt(E, "c3c1", 1)
    s2c = opt(E, "s2c", True)
    blocks = list(L.blocks)

    def c3c1(b, nb):   # engine._c3c1_ok
        return bool(c3c1_on) and nb is not None and b.filters == 64 and nb.filters == 64 and not b.proj \
            and not nb.proj and nb.stride == 1
    c1_done = False
    c64_min = opt(E, "c64_min_m", 262144)
    for bi, b in enumerate(blocks):
        f, cin = b.filters, b.cin
        Ho = (H - 1) // b.stride + 1
        M = B * Ho * Ho
        n1 = 5 * f if b.proj and not fuse else f
        nb = blocks[bi + 1] if bi + 1 < len(blocks) else None
        if not c1_done:
            ev.append(("igemm", f"{b.name} c1{'+c0' if n1 > f else ''} fwd", 2 * M * cin * n1,
                       (B * H * H * cin + M * n1) * 2, (M, n1, cin)))
        c64 = f == 64 and M >= c64_min and Ho + 2 <= 64 and opt(E, "c64", True)
        ev.append(("conv3x3c64" if c64 else "igemm", f"{b.name} c2 fwd", 2 * M * 9 * f * f, (M * f * 2) * 2,
                   (M, f, 9 * f)))
        c1_done = c3c1(b, nb)
        if c1_done:   # conv3 (+ shortcut) and the next block's conv1 in one launch
            k3 = f + cin if b.proj else f
            ev.append(("c3c1", f"{b.name} c3 + {nb.name} c1 fwd", 2 * M * k3 * 4 * f + 2 * M * 4 * f * f,
                       (M * k3 + (0 if b.proj else M * 4 * f) + M * 4 * f + M * f) * 2))
        elif b.proj and fuse:   # conv3 + the shortcut conv as one dual-source GEMM (K = f + cin)
            ev.append(("igemm", f"{b.name} c3+c0 fwd", 2 * M * (f + cin) * 4 * f, (M * f + M * cin + M * 4 * f) * 2,
                       (M, 4 * f, f + cin), "dual"))
        elif s2c and nb is not None and nb.proj and nb.stride == 2:   # engine s2c: conv3 on the stride-2 grid
            Mq = B * ((Ho + 1) // 2) ** 2
            ev.append(("igemm", f"{b.name} c3 fwd (s2 grid)", 2 * Mq * f * 4 * f, (Mq * f + 2 * Mq * 4 * f) * 2,
                       (Mq, 4 * f, f)))
        else:
            ev.append(("igemm", f"{b.name} c3 fwd", 2 * M * f * 4 * f, (M * f + 2 * M * 4 * f) * 2, (M, 4 * f, f)))
        geo.append((b, H, Ho))
        H = Ho
    ev.append(("gap_fwd", "gap", 0, B * H * H * 2048 * 2))
    ev.append(("igemm", "dense fwd", 2 * B * 2048 * 1000, 0, (B, 1000, 2048)))
    ev.append(("softmax", "xent", 0, 0))
    ev.append(("wgrad", "dense wgrad", 2 * B * 2048 * 1000, 0))
    ev.append(("colsum", "dense", 0, 0))
    ev.append(("igemm", "dense dgrad", 2 * B * 2048 * 1000, 0, (B, 2048, 1024)))
    ev.append(("gap_bwd", "gap", 0, 0))
    blocks = L.blocks
    s2 = {i for i in range(len(blocks) - 1) if blocks[i + 1].proj and blocks[i + 1].stride == 2}
    c1pre_on = opt(E, "c1pre", True) and c3c1_on != 0

    def fused_c3(i):
        fi = blocks[i].filters
        return fuse_bwd and (fi == 64 or (fi == 128 and fuse_bwd3)) and i not in s2

    def pre_fused(i):   # engine._pre_fused: block i's conv1 dgrad inside block i-1's fused conv3 backward
        return (c1pre_on and i >= 1 and blocks[i].filters == 64 and blocks[i - 1].filters == 64 and not blocks[i].proj
                and blocks[i].stride == 1 and fused_c3(i - 1))
    for bi in range(len(geo) - 1, -1, -1):
        b, H, Ho = geo[bi]
        f, cin = b.filters, b.cin
        M = B * Ho * Ho
        # blocks feeding a stride-2 block: conv3 wgrad/dgrad and conv2 wgrad on the compact quarter
        Mc = B * (Ho // 2 + Ho % 2) ** 2 if bi in s2 else M
        if bi + 1 < len(geo) and pre_fused(bi + 1):
            ev.append(("bwd1x1", f"{blocks[bi + 1].name} c1 dgrad + {b.name} c3 dgrad+wgrad",
                       4 * Mc * f * 4 * f + 2 * M * 4 * f * f, (M * f + 3 * M * 4 * f + 2 * Mc * f) * 2))
        elif fuse_bwd and (f == 64 or (f == 128 and fuse_bwd3)) and (bi not in s2 or fuse_s2):   # bwd1x1: one read of g
            ev.append(("bwd1x1", f"{b.name} c3 dgrad+wgrad", 4 * Mc * f * 4 * f, (Mc * 4 * f + 2 * Mc * f) * 2))
        else:
            ev.append(("wgrad", f"{b.name} c3 wgrad", 2 * Mc * f * 4 * f, (Mc * f + Mc * 4 * f) * 2))
            ev.append(("igemm", f"{b.name} c3 dgrad", 2 * Mc * f * 4 * f, (Mc * 4 * f + Mc * f + M * f) * 2,
                       (Mc, f, 4 * f)))
        c64w = f == 64 and M >= c64_min and Ho + 2 <= 64 and Mc == M and opt(E, "c64", True) and opt(E, "c64w", True)
        ev.append(("conv3x3c64" if c64w else "wgrad", f"{b.name} c2 wgrad", 2 * Mc * 9 * f * f, (Mc + M) * f * 2))
        c64 = f == 64 and M >= c64_min and Ho + 2 <= 64 and opt(E, "c64", True)
        ev.append(("conv3x3c64" if c64 else "igemm", f"{b.name} c2 dgrad", 2 * M * 9 * f * f, 3 * M * f * 2,
                   (M, f, 9 * f)))
        n1 = 5 * f if b.proj else f
        if b.proj:   # conv1 and the shortcut conv: one wgrad launch per gradient source
            ev.append(("wgrad", f"{b.name} c1 wgrad", 2 * M * cin * f, (M * f + B * H * H * cin) * 2))
            ev.append(("wgrad", f"{b.name} c0 wgrad", 2 * M * cin * 4 * f, (M * 4 * f + B * H * H * cin) * 2))
        else:
            ev.append(("wgrad", f"{b.name} c1 wgrad", 2 * M * cin * n1, (M * n1 + B * H * H * cin) * 2))
        ev.append(("wgrad_finalize", b.name, 0, 0))
        if pre_fused(bi):
            continue
        ev.append(("igemm", f"{b.name} c1 dgrad", 2 * M * cin * n1, (M * n1 + 3 * B * H * H * cin) * 2, (M, cin, n1),
                   "dual" if b.proj else ""))
    if fuse_stem:   # pool backward + conv1 weight gradient in one launch (stem.hip)
        ev.append(("stem_pool", "pool bwd + conv1 wgrad", 2 * B * H1 * H1 * 256 * 64, 0))
    else:
        ev.append(("maxpool_bwd", "pool", 0, 0))
        ev.append(("wgrad", "conv1 wgrad", 2 * B * H1 * H1 * 256 * 64, 0))
    ev.append(("stem_wgrad_fold", "fold", 0, 0))
    ev.append(("wgrad_finalize", "stem", 0, 0))
    ev.append(("colsum_reduce", "cred", 0, 0))
    ev.append(("bn_grad", "bn", 0, 0))
    ev.append(("opt_hparams", "hparams", 0, 0))
    if os.environ.get("NO_ADAM") is None:
        ev.append(("adam", "adam", 0, 0))
    ev.append(("prep", "prep", 0, 0))
    return ev


def segment(path, B=1024, crop=224, knobs=""):
    """The last complete training step of a rocprofv3 CSV (kernel trace or one-counter
    collection), paired with the engine's launch schedule: [(event, [csv rows])]."""
    rows = [r for r in csv.DictReader(open(path))]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "pddl::" in r["Kernel_Name"]]
    rows = [r for r in rows if "comm_proxy" not in r["Kernel_Name"]]   # bench --comm-proxy stand-ins
    fb = opt(E, "fuse_bwd", 1)
    ev = schedule(B, crop, opt(E, "fuse_proj", True), fb != 0, fb != 2, opt(E, "fuse_bwd_s2", True),
                  opt(E, "fuse_stem", True))
    # a split launch (8-phase kernel for full rounds + 128x128 tail) is two dispatches of one layer
    try:
        from pddl.ops.native import require_native
        for knob in filter(None, knobs.split(",")):
            k, v = knob.split("=")
            require_native().set_variant(k, int(v))
        plan = require_native().igemm_plan
    except Exception:   # no native module: unsplit schedule
        plan = None

    # ... and a split-K launch is the slices + the combine (igemm_splitk_reduce_kernel); the
    # projection blocks' dual-source c1 dgrad is never split
    pk_dual = 2   # (igemm_pk_dual knob: dual-source forwards with K / 64 <= this run as one ring launch)
    for knob in filter(None, knobs.split(",")):
        if knob.startswith("igemm_pk_dual="):
            pk_dual = int(knob.split("=")[1])

    def ndisp(e):
        if e[0] != "igemm" or plan is None:
            return 1
        if len(e) > 5 and e[5] == "dual" and "fwd" in e[1] and e[4][2] // 64 <= pk_dual:
            return 1
        cfg, split, ks = plan(*e[4])
        dual = len(e) > 5 and e[5] == "dual"
        return 2 if split < e[4][0] or (ks > 1 and not dual) else 1
    nd = [ndisp(e) for e in ev]
    need = sum(nd)
    starts = [i for i, r in enumerate(rows) if "stem_s2d" in r["Kernel_Name"]]
    st = None
    for s in reversed(starts):
        if s + need <= len(rows):
            st = s
            break
    seg = rows[st:st + need]
    out, k = [], 0
    for e, n in zip(ev, nd):
        rs = seg[k:k + n]
        k += n
        kn = kernel_names(rs)
        assert e[0].split("_")[0] in kn, (e[0], kn)
        out.append((e, rs))
    return out


def kernel_names(rs):
    return " + ".join(r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
                      .replace("pddl::", "")[:22] for r in rs)


def main():
    path = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    crop = int(sys.argv[3]) if len(sys.argv) > 3 else 224
    knobs = sys.argv[4] if len(sys.argv) > 4 else ""   # the run's PDDL_KNOBS (changes the launch plan)
    segs = segment(path, B, crop, knobs)
    tot = 0
    agg = {}
    for e, rs in segs:
        kind, name, flops, byts = e[:4]
        kn = kernel_names(rs)
        t = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 for r in rs)
        tot += t
        k2 = kind + (" fwd" if "fwd" in name and kind == "igemm" else " dgrad" if "dgrad" in name else "")
        agg[k2] = agg.get(k2, 0) + t
        tf = flops / t / 1e12 if flops else 0
        gb = byts / t / 1e9 if byts else 0   # MODELLED logical bytes (see scripts/roofline.py for measured)
        grid = "+".join(r.get("Grid_Size_X") or r.get("Grid_Size", "?") for r in rs)
        meas = ""
        if "Counter_Value" in rs[0]:
            # rocprofv3 counter collection: WRITE_SIZE / FETCH_SIZE in KiB (FETCH_SIZE reads half the
            # bytes on gfx950: calibrated against a streaming read of known size, profiles/r3_hbm_bytes)
            cn = rs[0]["Counter_Name"]
            mb = sum(float(r["Counter_Value"]) for r in rs) * 1024 * (2 if cn == "FETCH_SIZE" else 1) / 1e6
            meas = f"  {cn[:5]} {mb:8.1f} MB ({mb * 1e6 / t / 1e9:6.0f} GB/s)"
        print(f"{t*1e6:9.1f} us  {tf:7.1f} TF/s  {gb:7.0f} GB/s(model)  grid={grid:>16}  {kn[:40]:40s} {name}{meas}")
    print(f"step total {tot*1e3:.2f} ms")
    seg0, seg1 = segs[0][1][0], segs[-1][1][-1]
    t_first, t_last = int(seg0["Start_Timestamp"]), int(seg1["End_Timestamp"])
    print(f"step span (first start -> last end) {(t_last - t_first) * 1e-6:.2f} ms")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1]):
        print(f"  {k:24s} {v*1e3:8.3f} ms")


if __name__ == "__main__":
    main()
