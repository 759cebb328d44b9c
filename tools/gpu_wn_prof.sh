#!/bin/bash
# rocprofv3 kernel stats of the WaveNet forward, fused layer (0) vs two-kernel layer (1)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02_wnprof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for L in 0 1; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/l$L -o run --output-format csv -- \
    python3 -u $GRAFT_REPO_ROOT/tools/bench_wn.py --layer $L > $O/l$L.log 2>&1 || { tail -20 $O/l$L.log; exit 1; }
  tail -1 $O/l$L.log
  python3 - $O/l$L <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wn_" in r["Name"]:
            print(f'{r["Name"][:70]:70s} calls {r["Calls"]:>5s} avg {float(r["AverageNs"])/1e3:8.2f} us')
PY
done
