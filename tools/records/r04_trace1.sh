#!/bin/bash
# kernel trace of one A/B child (the group kernels' grids and durations)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04tr1}; mkdir -p $OUT
export SLAT_LIB_PATH=$GRAFT_REPO_ROOT/tools/var/libslat_k4.so SLAT_GROUP=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/ab.py --child --steps 20 --chain > $OUT/child.json 2> $OUT/child.err || { tail -20 $OUT/child.err; exit 1; }
cat $OUT/child.json
python3 - $OUT <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/trace/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
agg = collections.defaultdict(list)
for r in rows:
    k = r["Kernel_Name"].split("(")[0][:70]
    agg[(k, r.get("Grid_Size_X", r.get("Grid_Size")), r.get("Workgroup_Size_X", r.get("Workgroup_Size")), r.get("LDS_Block_Size"), r.get("VGPR_Count"), r.get("SGPR_Count"))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
print(list(rows[0].keys()))
for k, v in sorted(agg.items(), key=lambda x: -sum(x[1]))[:25]:
    print(len(v), round(sum(v) / len(v) / 1000, 1), "us", k)
PY
