"""Summarise a rocprofv3 kernel-trace CSV: per-kernel totals and the last full training step."""
import csv
import sys


def main(path_dir: str, marker: str = "step_finalize_kernel") -> None:
    """``marker``: a kernel launched exactly once per training step (step_finalize ends every step;
    the optimizer runs as several launches per step when its updates overlap the backward)."""
    stats = list(csv.DictReader(open(f"{path_dir}/run_kernel_stats.csv")))
    print("== kernel totals ==")
    for r in stats[:30]:
        print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms  calls={r['Calls']:>5}  avg={float(r['AverageNs'])/1e3:9.1f} us  "
              f"{r['Percentage'][:5]:>5}%  {r['Name'][:110]}")
    rows = sorted(csv.DictReader(open(f"{path_dir}/run_kernel_trace.csv")), key=lambda r: int(r['Start_Timestamp']))
    idx = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
    if len(idx) >= 2:
        a, b = idx[-2], idx[-1]
        t0 = int(rows[a]['End_Timestamp'])
        print(f"== last step timeline (us since the previous {marker} ended) ==")
        for r in rows[a + 1:b + 1]:
            s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
            print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:9.1f}us vgpr={r['VGPR_Count']:>4} agpr={r['Accum_VGPR_Count']:>4} "
                  f"lds={r['LDS_Block_Size']:>6} grid={r['Grid_Size_X']:>7} {r['Kernel_Name'][:100]}")
        print(f"step span: {(int(rows[b]['End_Timestamp']) - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main(*sys.argv[1:])
