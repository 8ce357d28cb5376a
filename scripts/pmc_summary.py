"""Summarize rocprofv3 PMC counters per pddl kernel (mean over dispatches).

    python scripts/pmc_summary.py gpurun_out/pmc
"""
import collections
import csv
import glob
import sys


def main(root):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{root}/pmc_*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "pddl::" not in name:
                continue
            key = name.split("(")[0].replace("void ", "").replace("pddl::", "") + f" grid={r['Grid_Size']}"
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(agg):
        c = {n: sum(v) / len(v) for n, v in agg[k].items()}
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        busy = c.get("SQ_BUSY_CYCLES", 0) or 1
        line = [k[:70]]
        if "SQ_WAIT_ANY" in c:
            line.append(f"wait_any {c['SQ_WAIT_ANY'] / wc:5.2f} wait_inst {c['SQ_WAIT_INST_ANY'] / wc:5.2f} "
                        f"active {c['SQ_ACTIVE_INST_ANY'] / wc:5.2f} mfma_busy/busy {c['SQ_VALU_MFMA_BUSY_CYCLES'] / busy:6.2f}")
        if "SQ_LDS_BANK_CONFLICT" in c:
            line.append(f"lds_conf/active {c['SQ_LDS_BANK_CONFLICT'] / max(1, c['SQ_LDS_IDX_ACTIVE']):5.3f} "
                        f"valu/mfma {c['SQ_INSTS_VALU'] / max(1, c['SQ_INSTS_MFMA']):5.1f}")
        if "TCC_HIT_sum" in c:
            line.append(f"L2 hit {c['TCC_HIT_sum'] / max(1, c['TCC_HIT_sum'] + c['TCC_MISS_sum']):5.2f} "
                        f"unaligned {c.get('SQ_LDS_UNALIGNED_STALL', 0):.0f}")
        print(" | ".join(line))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
