"""Per-kernel MFMA utilisation of the training step from tools/pmc_step_mfma.sh.

util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 256 CUs * 4 SIMDs); counter passes
serialise kernels, so every row is that kernel running alone (no optimizer overlap).
"""
import csv
import glob
import sys
from collections import defaultdict


def main(root: str) -> None:
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"].split("(pz::")[0].replace("void pz::(anonymous namespace)::", "")[:80], r["Grid_Size"])
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    rows = []
    for k, c in acc.items():
        gui = c["GRBM_GUI_ACTIVE"]
        if gui <= 0:
            continue
        wc = max(c["SQ_WAVE_CYCLES"], 1.0)
        rows.append((c["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui / 8 * 1024), k, len(disp[k]), gui / 8 / len(disp[k]),
                     c["SQ_WAIT_ANY"] / wc, c["SQ_WAIT_INST_ANY"] / wc, c["SQ_ACTIVE_INST_ANY"] / wc))
    print(f"{'kernel':80} {'grid':>8} {'n':>3} {'cyc/disp':>9} {'MFMA':>6} {'WAIT_ANY':>8} {'WAIT_INST':>9} {'ACTIVE':>6}")
    for util, (name, grid), n, cyc, wa, wi, ac in sorted(rows, key=lambda r: -r[3] * r[2]):
        print(f"{name:80} {grid:>8} {n:3d} {cyc:9.0f} {util:6.3f} {wa:8.3f} {wi:9.3f} {ac:6.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
