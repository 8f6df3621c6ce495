#!/bin/bash
# One rocprofv3 --pmc pass (kernel trace only) over tools/gemm_w4_lab; per-kernel counter sums.
set -e
repo=$(pwd)
out=$repo/gpurun_out/pmc_w4
mkdir -p "$out"
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --kernel-trace \
    --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
          SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
    -d "$out" -o run --output-format csv -- "$repo/tools/gemm_w4_lab") > "$out.log" 2>&1
python3 - "$out" <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]; k = ("lib_var30" if "gemm_mfma" in k else k.split("::")[1].split("(")[0] if k.startswith("void w4::") else None)
        if k is None: continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
for k, c in sorted(acc.items()):
    gui = c["GRBM_GUI_ACTIVE"]; wc = c["SQ_WAVE_CYCLES"]
    print(f"{k:10} disp {len(n[k]):3} MFMA util {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (gui / 8 * 1024):.3f} "
          f"WAIT_ANY {c['SQ_WAIT_ANY'] / wc:.3f} WAIT_INST {c['SQ_WAIT_INST_ANY'] / wc:.3f} "
          f"ACTIVE {c['SQ_ACTIVE_INST_ANY'] / wc:.3f} WAIT_LDS {c['SQ_WAIT_INST_LDS'] / wc:.3f} "
          f"LDS_BANK_CONFL/disp {c['SQ_LDS_BANK_CONFLICT'] / len(n[k]):.0f}")
PY
