"""Summarise rocprofv3 --pmc counter CSVs per kernel (sum over dispatches) + derived ratios.

usage: python tools/pmc_summary.py gpurun_out/pmc_<tag> [kernel-substring ...]
"""
import collections
import csv
import glob
import os
import sqlite3
import sys


def short(name: str) -> str:
    if "gemm_mfma_kernel" in name:
        return "pz_gemm<" + name.split("gemm_mfma_kernel<", 1)[1].split(">(", 1)[0] + ">"
    if "gemm_sk_kernel" in name:
        return "pz_sk<" + name.split("gemm_sk_kernel<", 1)[1].split(">(", 1)[0] + ">"
    if name.startswith("Cijk_"):
        return name[:60]
    return name.split("(", 1)[0][:60]


def main():
    root = sys.argv[1]
    keep = sys.argv[2:] or ["gemm_mfma", "gemm_sk", "Cijk_"]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))

    def add(kernel, counter, value):
        if any(s in kernel for s in keep):
            agg[short(kernel)][counter] += float(value)

    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                add(r["Kernel_Name"], r["Counter_Name"], r["Counter_Value"])
    for path in glob.glob(os.path.join(root, "**", "*results.db"), recursive=True):  # rocpd SQLite output
        con = sqlite3.connect(path)
        for k, n, v in con.execute("select kernel_name, counter_name, value from counters_collection"):
            add(k, n, v)
        con.close()
    for k, c in sorted(agg.items()):
        print(f"== {k}")
        for n, v in sorted(c.items()):
            print(f"   {n:36s} {v:16.0f}")
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA"):
                if n in c:
                    print(f"   {n + ' / WAVE_CYCLES':36s} {c[n] / wc:16.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
            # MFMA busy is summed over SIMDs (256 CUs x 4); GUI_ACTIVE is per-GPU cycles
            print(f"   {'MFMA util (busy/(gui*1024))':36s} "
                  f"{c['SQ_VALU_MFMA_BUSY_CYCLES'] / (c['GRBM_GUI_ACTIVE'] * 1024):16.3f}")
        if "TCC_HIT_sum" in c:
            print(f"   {'L2 hit rate':36s} {c['TCC_HIT_sum'] / max(1.0, c['TCC_HIT_sum'] + c['TCC_MISS_sum']):16.3f}")


if __name__ == "__main__":
    main()
