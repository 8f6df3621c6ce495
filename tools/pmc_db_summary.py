"""Per-(kernel, grid) counter summary from rocprofv3 --pmc rocpd databases (ROCm 7 SQLite output).

MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs), LDS busy =
SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE / 8 x 256 CUs) (MI355X_MICROARCH rocprofv3
notes: GUI_ACTIVE is summed over the 8 XCDs, MFMA busy over every SIMD); the SQ_WAIT_* / ACTIVE_*
columns are fractions of SQ_WAVE_CYCLES; LDS columns per dispatch. One row per kernel and grid size
(gemm_bench runs each shape's kernels several times; rows group the dispatches of one shape).

    python tools/pmc_db_summary.py gpurun_out/pmc_<tag> [name-substring ...]
"""
import collections
import glob
import os
import sqlite3
import sys


def short(name: str) -> str:
    if "gemm_mfma" in name:
        inner = name.split("<", 1)[1].split(">(", 1)[0].replace("unsigned short", "u16").replace(" ", "")
        return ("pz_pair<" if "pair" in name else "pz_gemm<") + inner + ">"
    return name.split("(", 1)[0][:48]


def main():
    root = sys.argv[1]
    keep = sys.argv[2:] or ["gemm_mfma", "Cijk"]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    passes = collections.defaultdict(lambda: collections.defaultdict(set))
    for db in sorted(glob.glob(os.path.join(root, "**", "*.db"), recursive=True)):
        con = sqlite3.connect(db)
        rows = list(con.execute("select dispatch_id, kernel_name, grid_size, counter_name, value "
                                "from counters_collection order by dispatch_id"))
        con.close()
        # consecutive dispatches of one (kernel, grid) form a run: gemm_bench times each case's
        # fused / plain / hipBLASLt kernels in back-to-back loops, so run k of every counter pass
        # is the same loop and same-template kernels of different cases stay apart
        run, last, seen = -1, None, set()
        for did, kname, grid, cname, val in rows:
            if did not in seen:
                seen.add(did)
                k = (kname, grid)
                if k != last:
                    run, last = run + 1, k
            if not any(s in kname for s in keep):
                continue
            key = (run, short(kname), int(grid))
            acc[key][cname] += float(val)
            disp[key].add((db, did))
            passes[key][cname].add(db)
    hdr = f"{'kernel':60} {'grid':>8} {'disp':>5} {'MFMA':>6} {'WAIT_ANY':>8} {'WAIT_INST':>9} {'WAIT_LDS':>8} " \
          f"{'ACTIVE':>6} {'LDS instr/disp':>14} {'bank confl/disp':>15} {'LDS busy':>8}"
    print(hdr)
    for key in sorted(acc):
        # a counter collected in several passes (GRBM_GUI_ACTIVE rides along in each): per-pass mean
        c = {k: v / len(passes[key][k]) for k, v in acc[key].items()}
        n = len(disp[key]) // max(1, len({d for d, _ in disp[key]}))
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or float("nan")
        gui = c.get("GRBM_GUI_ACTIVE", 0.0)
        util = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui / 8 * 1024) if gui and "SQ_VALU_MFMA_BUSY_CYCLES" in c else float("nan")
        f = lambda k: c[k] / wc if k in c else float("nan")  # noqa: E731
        # LDS-array busy share per CU: SQ_LDS_IDX_ACTIVE (summed over CUs) / (GUI/8 x 256 CUs)
        lds_busy = c["SQ_LDS_IDX_ACTIVE"] / (gui / 8 * 256) if gui and "SQ_LDS_IDX_ACTIVE" in c else float("nan")
        print(f"{key[0]:2d} {key[1][:57]:57} {key[2]:8d} {n:5d} {util:6.3f} {f('SQ_WAIT_ANY'):8.3f} {f('SQ_WAIT_INST_ANY'):9.3f} "
              f"{f('SQ_WAIT_INST_LDS'):8.3f} {f('SQ_ACTIVE_INST_ANY'):6.3f} {c.get('SQ_INSTS_LDS', float('nan')) / n:14.0f} "
              f"{c.get('SQ_LDS_BANK_CONFLICT', float('nan')) / n:15.0f} {lds_busy:8.3f}")


if __name__ == "__main__":
    main()
