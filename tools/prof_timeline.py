"""Per-kernel timeline (both streams) of the last complete step of a rocprofv3 kernel trace.

usage: python tools/prof_timeline.py gpurun_out/prof_<tag> [--steps-back 2]
Times are microseconds relative to the end of the step_finalize launch that closed the step
before; q = the HIP queue (compute stream / optimizer side stream).
"""
import argparse
import csv
import glob
import os


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps-back", type=int, default=2)
    a = ap.parse_args()
    path = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    fin = [i for i, r in enumerate(rows) if "step_finalize" in r["Kernel_Name"]]
    lo, hi = fin[-1 - a.steps_back], fin[-a.steps_back]
    t0 = int(rows[lo]["End_Timestamp"])
    for r in rows[lo - 3:hi + 1]:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        name = r["Kernel_Name"].replace("void pz::(anonymous namespace)::", "").replace("pz::(anonymous namespace)::", "")
        print(f"{s:9.1f} {e:9.1f} {e - s:8.1f}  q{r.get('Stream_Id', r.get('Queue_Id', '?'))}  "
              f"grid={r.get('Grid_Size_X', r.get('Grid_Size', '?')):>8}  {name[:90]}")
    print(f"step: {(int(rows[hi]['End_Timestamp']) - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
