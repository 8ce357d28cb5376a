"""Measured-bytes roofline of one training step.

    python scripts/roofline.py TRACE.csv FETCH.csv WRITE.csv [batch=2560] [crop=224]

TRACE.csv is a rocprofv3 --kernel-trace of bench.py; FETCH.csv / WRITE.csv are rocprofv3
--pmc FETCH_SIZE / --pmc WRITE_SIZE counter collections of the same command (one counter
per pass: FETCH_SIZE alone takes 3 of the 4 TCC counters).  Every launch of the last complete
step is paired with the engine schedule (scripts/analyze_trace.py) and gets

    time (kernel trace), FLOP (schedule), measured read / write bytes (counters),
    bound = max(FLOP / 2.5 PF, bytes / HBM)   and   %bound = bound / time.

FETCH_SIZE reports HALF the bytes of a wide streaming read on gfx950 (MI355X_MICROARCH.md
§HBM; our own calibration profiles/r3_hbm_bytes_per_layer.txt), so read bytes = 2 x FETCH_SIZE;
WRITE_SIZE is exact for 16-byte stores.  Both count Infinity-Cache hits as fabric traffic, so
a kernel whose operand stays in the 256 MiB MALL reads as bandwidth-heavier than it is.
HBM = 6.29 TB/s (the guide's measured float4 copy; our store_pattern copy: 4.81 TB/s).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import analyze_trace as at  # noqa: E402

PEAK_BF16 = 2.5e15
HBM = 6.29e12


def main():
    tr, fe, wr = sys.argv[1:4]
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 2560
    crop = int(sys.argv[5]) if len(sys.argv) > 5 else 224
    knobs = os.environ.get("PDDL_KNOBS", "")   # the run's kernel knobs (they change the launch plan)
    st = at.segment(tr, B, crop, knobs)
    sf = at.segment(fe, B, crop, knobs)
    sw = at.segment(wr, B, crop, knobs)
    assert len(st) == len(sf) == len(sw)

    def kib(rs):
        return sum(float(r["Counter_Value"]) for r in rs) * 1024

    print(f"# batch {B}, crop {crop}; bound = max(FLOP / {PEAK_BF16/1e15:.1f} PF, (read + write) / {HBM/1e12:.2f} TB/s)")
    print(f"{'time us':>9} {'TF/s':>7} {'read MB':>9} {'write MB':>9} {'TB/s':>6} {'bound us':>9} {'%bound':>6} "
          f"{'limit':>5}  layer")
    tot_t = tot_b = tot_r = tot_w = 0.0
    stages = {}
    rows = []
    for (e, rt), (_, rf), (_, rw) in zip(st, sf, sw):
        kind, name, flops = e[0], e[1], e[2]
        t = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 for r in rt)
        rd, wb = 2 * kib(rf), kib(rw)
        tc, tm = flops / PEAK_BF16, (rd + wb) / HBM
        bound = max(tc, tm)
        lim = "mfma" if tc >= tm else "hbm"
        tot_t += t
        tot_b += bound
        tot_r += rd
        tot_w += wb
        stg = name.split("_")[0] if name.startswith("conv") else "other"
        s = stages.setdefault(stg, [0.0, 0.0])
        s[0] += t
        s[1] += bound
        rows.append((t, bound, name))
        print(f"{t*1e6:9.1f} {flops/t/1e12 if flops else 0:7.1f} {rd/1e6:9.1f} {wb/1e6:9.1f} {(rd+wb)/t/1e12:6.2f} "
              f"{bound*1e6:9.1f} {100*bound/t:5.0f}% {lim:>5}  {name}  [{at.kernel_names(rt)[:34]}]")
    print(f"\nstep: {tot_t*1e3:.2f} ms of kernels, sum of per-launch bounds {tot_b*1e3:.2f} ms "
          f"({100*tot_b/tot_t:.0f}%), measured traffic read {tot_r/1e9:.1f} GB + write {tot_w/1e9:.1f} GB")
    for k, (t, b) in sorted(stages.items()):
        print(f"  {k:8s} {t*1e3:7.2f} ms  bound {b*1e3:7.2f} ms  ({100*b/t:.0f}%)")
    print("\nlargest gaps (time - bound):")
    for t, b, n in sorted(rows, key=lambda r: -(r[0] - r[1]))[:15]:
        print(f"  {(t-b)*1e6:8.1f} us  {n}")


if __name__ == "__main__":
    main()
