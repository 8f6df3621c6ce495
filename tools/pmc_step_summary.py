"""Per-kernel HBM traffic of a training step from two rocprofv3 --pmc passes over bench.py.

usage: python tools/pmc_step_summary.py gpurun_out/pmc_step   (expects f/ = FETCH_SIZE, w/ = WRITE_SIZE)

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. Counter runs serialise kernels, so the durations
here are un-overlapped single-kernel times and the rates are what each kernel achieves alone.
"""
import csv
import sys
from collections import defaultdict


def load(path, counter):
    rows = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            key = (r["Kernel_Name"].split("(pz::")[0][:90], int(r["Grid_Size"]))
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            rows[key].append((float(r["Counter_Value"]), dur))
    return rows


def main(root):
    fetch = load(f"{root}/f/run_counter_collection.csv", "FETCH_SIZE")
    write = load(f"{root}/w/run_counter_collection.csv", "WRITE_SIZE")
    print(f"{'kernel':90s} {'grid':>8s} {'n':>3s} {'rd MB':>8s} {'wr MB':>8s} {'us':>8s} {'GB/s':>7s}")
    out = []
    for key, fv in fetch.items():
        wv = write.get(key, [])
        n = len(fv)
        rd = sum(v for v, _ in fv) / n / 1024
        wr = (sum(v for v, _ in wv) / len(wv) / 1024) if wv else 0.0
        us = sum(d for _, d in fv) / n * 1e6
        out.append((key, n, rd, wr, us, (rd + wr) * 1e6 / 1e3 / max(us, 1e-9)))
    for key, n, rd, wr, us, bw in sorted(out, key=lambda t: -t[4]):
        if us < 2:
            continue
        print(f"{key[0]:90s} {key[1]:8d} {n:3d} {rd:8.1f} {wr:8.1f} {us:8.1f} {bw:7.0f}")


if __name__ == "__main__":
    main(sys.argv[1])
