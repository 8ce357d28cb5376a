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
            key = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("pddl::", "") + f" grid={r['Grid_Size']}"
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(agg):
        c = {n: sum(v) / len(v) for n, v in agg[k].items()}

        def ratio(a, b):
            return c[a] / c[b] if a in c and b in c and c[b] else None
        derived = {
            "lds_active/cu_busy": ratio("SQ_LDS_IDX_ACTIVE", "SQ_BUSY_CU_CYCLES"),
            "mfma_busy/cu_busy": ratio("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CU_CYCLES"),
            "lds_data_fifo_full/cu_busy": ratio("SQ_LDS_DATA_FIFO_FULL", "SQ_BUSY_CU_CYCLES"),
            "wait_any/wave": ratio("SQ_WAIT_ANY", "SQ_WAVE_CYCLES"),
            "wait_inst/wave": ratio("SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES"),
            "wait_inst_lds/wave": ratio("SQ_WAIT_INST_LDS", "SQ_WAVE_CYCLES"),
            "active/wave": ratio("SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES"),
            "valu/mfma": ratio("SQ_INSTS_VALU", "SQ_INSTS_MFMA"),
            "salu/mfma": ratio("SQ_INSTS_SALU", "SQ_INSTS_MFMA"),
            "lds_insts/mfma": ratio("SQ_INSTS_LDS", "SQ_INSTS_MFMA"),
            "lds_bank_conf/lds_active": ratio("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"),
            "L2_hit": (c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
                       if "TCC_HIT_sum" in c and (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]) else None),
        }
        print(k[:80] + " | " + " ".join(f"{n} {v:.3f}" for n, v in derived.items() if v is not None))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
