set -e
mkdir -p gpurun_out
ROUNDS=1 ARGS="--steps 40 --warmup 10" bash tools/ab_bench.sh "nat_hi=PZ_FORCE_COMM=1,PZ_COMM=native" "nat_lo=PZ_FORCE_COMM=1,PZ_COMM=native,PZ_COMM_PRIO=0" "torch=PZ_FORCE_COMM=1,PZ_COMM=torch" > gpurun_out/s10_ab.txt 2>&1 || { cat gpurun_out/s10_ab.txt; exit 1; }
cat gpurun_out/s10_ab.txt
cd /tmp && export TMPDIR=/tmp
PZ_FORCE_COMM=1 PZ_COMM=native timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_cmem -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_cmem.log 2>&1
cd $GRAFT_REPO_ROOT
ls gpurun_out/prof_cmem
python - <<'PY'
import csv, glob
for f in glob.glob('gpurun_out/prof_cmem/**/*memory_copy*.csv', recursive=True):
    rows = list(csv.DictReader(open(f)))
    print(f, len(rows))
    for r in rows[-12:]:
        print({k: r[k] for k in r if k in ('Direction','Bytes','Start_Timestamp','End_Timestamp','Src_Agent_Id','Dst_Agent_Id')})
PY
