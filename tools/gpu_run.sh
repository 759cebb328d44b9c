#!/bin/bash
# The one GPU-box measurement script: runs the named parts in order, each GPU step under its
# own time limit; the first failure ends the script (set -e).  Output under gpurun_out/<tag>/.
#
# usage (GPU box): tools/gpu_run.sh <tag> <part> [<part> ...]
#   tests[=<pytest -k expr>]  every -m gpu test (or the selected ones)       -> gpu_tests.log
#   bench=<cfg>[,<cfg>...]    one bench.py line per config (C3 C2 C4 C5 C5DS) -> bench_<cfg>.json
#   trace=<cfg>               rocprofv3 --kernel-trace --stats of that bench -> trace_<cfg>/
#   (trace / traffic / sq run one job at a time, --overlap 1: the bench line's roofline launch times
#   come from its isolated pass, bench.py)
#   traffic=<cfg>             FETCH_SIZE / WRITE_SIZE passes on the hot kernels -> <cfg>_traffic.json
#   sq=<cfg>                  SQ-counter passes (tools/pmc_sq.sh) + summary  -> <cfg>_sq.json
#   ab=<lib|->:<args>;...     same-box A/B bench lines (tools/gpu_ab_libs.sh), ';'-separated specs
# e.g. tools/gpu_run.sh r05_a tests bench=C3,C5 trace=C3 traffic=C3
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
export TMPDIR=/tmp

bench_args() {   # config -> bench.py arguments
  case $1 in
    C5DS) echo "--config C5 --lengths ds" ;;
    C4) echo "--config C4 --cpu-frames 0" ;;
    *) echo "--config $1" ;;
  esac
}
regex() {        # config -> kernels the PMC passes cover
  case $1 in
    C5*) echo "nsf_pair_kernel|nsf_wconv|nsf_ups_kernel|wn_stack_bf16" ;;
    PITCH) echo "wn_stack_bf16|wn_xa|matvec" ;;
    *) echo "lvc_block_bf16_kernel|lvc_ps_kernel|kp_kernel_bf16|wn_stack_bf16|kp_hidden_bf16|dblock_bf16" ;;
  esac
}

for part in "$@"; do
  key=${part%%=*}; val=${part#*=}; [ "$val" = "$part" ] && val=""
  case $key in
    tests)
      K=(); [ -n "$val" ] && K=(-k "$val")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" \
        > $O/gpu_tests.log 2>&1
      tail -2 $O/gpu_tests.log ;;
    bench)
      for c in ${val//,/ }; do
        timeout -k 10 300 python -u bench.py $(bench_args $c) > $O/bench_$c.json 2> $O/bench_$c.err
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); \
print(sys.argv[2], d['ms_per_step'], 'ms/step', d['value'], d['roofline']['kernel'], d['roofline']['frac'])" \
          $O/bench_$c.json $c
      done ;;
    trace)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$val -o run --output-format csv -- \
        python -u $R/bench.py $(bench_args $val) --overlap 1 --cpu-frames 0 --no-kernel-timing > $O/trace_$val.log 2>&1) ;;
    traffic)
      for pmc in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc $pmc --kernel-include-regex "$(regex $val)" \
          -d $O/pmc_$val/pmc_$pmc -o run --output-format csv -- \
          python -u $R/bench.py $(bench_args $val) --overlap 1 --steps 2 --warmup 1 --cpu-frames 0 --no-kernel-timing \
          > $O/pmc_${val}_$pmc.log 2>&1)
      done
      case $val in C4) b=32 ;; *) b=8 ;; esac   # (PITCH: 8 x 861 too)
      python tools/pmc_traffic.py $O/pmc_$val $O/${val}_traffic.json $TAG ${val%DS} $b 861 ;;
    sq)
      timeout -k 10 500 tools/pmc_sq.sh $TAG/sq_$val "$(regex $val)|enc_|dblock_bf16" $(bench_args $val) --overlap 1 --steps 1
      python tools/sq_summary.py gpurun_out/$TAG/sq_$val --config ${val%DS} -o $O/${val}_sq.json ;;
    ab)
      IFS=';' read -ra specs <<< "$val"
      tools/gpu_ab_libs.sh $TAG/ab "${specs[@]/:/|}" ;;
    *) echo "unknown part $part"; exit 2 ;;
  esac
done
echo done
