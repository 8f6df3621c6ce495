#!/bin/bash
# r4: L2 / TA counters of pz vs hipBLASLt on dX_L2 and fwd_L2 (pmc_gemm.sh mem set: three passes)
PMC_SET=mem bash tools/pmc_gemm.sh mem2 dX_L2 fwd_L2 || exit 2
python tools/pmc_db_summary.py gpurun_out/pmc_mem2 > gpurun_out/pmc_mem2/summary.txt 2>&1 || true
python - <<'PY'
import sqlite3, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for db in sorted(glob.glob("gpurun_out/pmc_mem2/**/*.db", recursive=True)):
    con = sqlite3.connect(db)
    for did, k, c, v in con.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection"):
        key = ("pz " if "gemm_mfma" in k else "hipblaslt " if "Cijk" in k else "other ") + k.split("(")[0][-60:]
        acc[key][c] += v
for k, c in acc.items():
    if k.startswith("other"): continue
    hit, miss = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
    print(k[:80], {kk: round(vv) for kk, vv in c.items()}, "L2 hit %.3f" % (hit / max(1, hit + miss)))
PY
