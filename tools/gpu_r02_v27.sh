#!/bin/bash
# r02 v27: rocprofv3 kernel trace of C5 steady-state steps (does the 32-bps pipeline overlap?)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02_v27}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c5 -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --config c5 --no-cpu --no-e2e --no-pmc --steps 4 --warmup 2 > $OUT/c5.log 2>&1 || { echo TRACE_FAILED; tail -20 $OUT/c5.log; exit 1; }
python - <<'PY'
import csv, glob, os
f = glob.glob(os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r02_v27/c5/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
big = [i for i, r in enumerate(rows) if "k_analyze" in r["Kernel_Name"] and dur(r) > 50]
t0 = int(rows[big[2]]["Start_Timestamp"])
for r in rows[big[2] - 8: big[4] + 1]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e6; e = (int(r["End_Timestamp"]) - t0) / 1e6
    if e - s > 0.05: print(f"{s:9.2f} {e:9.2f} {e-s:8.2f} q{r['Queue_Id']:>3} {r['Kernel_Name'][:50]}")
PY
echo ALLOK
