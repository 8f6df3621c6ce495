"""MFMA-pipe utilisation per GEMM kernel from tools/pmc_mfma.sh (rocprofv3 --pmc, CSV).

SQ_VALU_MFMA_BUSY_CYCLES counts matrix-pipe busy cycles summed over every SIMD (16 per
v_mfma_f32_16x16x32_bf16, 32 per 32x32x16: MI355X_MICROARCH cycle constants), and
GRBM_GUI_ACTIVE counts GPU-busy cycles summed over the 8 XCDs. So

    MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 256 CUs * 4 SIMDs)

(the round-1 "busy / (gui * 1024)" was 8x too small). Cross-check printed next to it: the busy
cycles the kernel's FLOPs imply (FLOP / 16384 MFMAs x 16 cycles) against the counter.
"""
import csv
import glob
import os
import sys
from collections import defaultdict

FLOP = {"fwd_L2": 2 * 8192 * 4096 * 4096, "dX_L2": 2 * 8192 * 4096 * 4096, "dW_L2": 2 * 4096 * 4096 * 8192,
        "fwd_L1": 2 * 8192 * 4096 * 1024, "dX_L3": 2 * 8192 * 4096 * 1024}


def main(root: str) -> None:
    print(f"{'case':8} {'kernel':44} {'disp':>5} {'MFMA util':>9} {'busy/FLOP-implied':>17} "
          f"{'clock GHz':>9} {'WAIT_ANY':>8} {'WAIT_INST':>9} {'ACTIVE':>7}")
    for case in sorted(FLOP):
        files = glob.glob(os.path.join(root, case, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            continue
        acc = defaultdict(lambda: defaultdict(float))
        disp = defaultdict(set)
        dur = defaultdict(float)
        for row in csv.DictReader(open(files[0])):
            name = row["Kernel_Name"]
            if "gemm_mfma_kernel" not in name:
                continue
            acc[name][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[name].add(row["Dispatch_Id"])
        trace = glob.glob(os.path.join(root, case, "**", "*kernel_trace.csv"), recursive=True)
        if trace:
            for row in csv.DictReader(open(trace[0])):
                if "gemm_mfma_kernel" in row["Kernel_Name"]:
                    dur[row["Kernel_Name"]] += (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
        for name, c in acc.items():
            n = len(disp[name])
            gui = c["GRBM_GUI_ACTIVE"]
            util = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui / 8 * 1024) if gui else float("nan")
            implied = FLOP[case] / (16 * 16 * 32 * 2) * 16 * n
            clock = gui / 8 / dur[name] / 1e9 if dur.get(name) else float("nan")
            wc = c["SQ_WAVE_CYCLES"] or 1
            var = name.split("unsigned short, ")[-1].split(">")[0] if "unsigned short, " in name else name[-40:]
            short = ("<" + ",".join(name.split("<")[1].split(",")[4:6]) + "," + var + ">")[:44]
            print(f"{case:8} {short:44} {n:5d} {util:9.3f} {c['SQ_VALU_MFMA_BUSY_CYCLES'] / implied:17.3f} "
                  f"{clock:9.2f} {c['SQ_WAIT_ANY'] / wc:8.3f} {c['SQ_WAIT_INST_ANY'] / wc:9.3f} "
                  f"{c['SQ_ACTIVE_INST_ANY'] / wc:7.3f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_mfma")
