#!/bin/bash
# WaveNet layer kernels vs batch size (rocprofv3 kernel stats), layer mode $1 (default 1)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${2:-r02_wnscan}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for B in ${BATCHES:-2 4 8 16}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/b$B -o run --output-format csv -- \
    python3 -u $GRAFT_REPO_ROOT/tools/bench_wn.py --layer ${1:-1} --batch $B > $O/b$B.log 2>&1 || { tail -20 $O/b$B.log; exit 1; }
  python3 - $O/b$B $B <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wn_" in r["Name"]:
            print(f'B={sys.argv[2]:3s} {r["Name"][:60]:60s} calls {r["Calls"]:>5s} avg {float(r["AverageNs"])/1e3:8.2f} us')
PY
done
