#!/bin/bash
# GPU box: the measurement steps of a session, each under its own time limit,
# stopping at the first failure.  Output under gpurun_out/<tag>/.
#
# usage: tools/gpu_steps.sh <tag> <step> [<step> ...]
#   parity[:files]     pytest -m gpu (all tests, or the comma-separated files)
#   bench:<config>     one driver-flag bench line (--steps 20 --warmup 5)
#   events:<config>    bench lines with --events 2 / 1 / 0 (what events cost)
#   kstats:<config>    rocprofv3 --kernel-trace --stats of a bench run, and the
#                      gaps between the last launches (tools/gaps.py)
#   conn:<lib,...>     connection batches at 12 and 64 local ACLs per build
#                      (default = vpp_amd/libcontivcls.so, else variants/lib_<x>.so),
#                      with rocprofv3 kernel stats
#   connn:<n>          connection batches of n connections, 12 local ACLs, kernel stats
#   gp16:<lib,...>     gen-policy ingress lists, 16-byte layout, 10 % IPv6
#   gp:<layout>        gen-policy 20-block list: 64 / 256 Mi packets, TCP/UDP only
#   gpmix:<layout>     the 20-block list without protocol 47, without ICMP
#   gpb:<bytes>:<layout>:<blocks>  a gen-policy ingress list compiled with an
#                      LDS budget of <bytes> (option lds_budget: counter tiers)
#   ab:<config>:<lib>  one-process A/B of the classify kernel against a variant
#   sq:<config>        SQ counter passes of the classify kernel (tools/sq_profile.sh)
#   sqgp:<layout>:<blocks>  the same for a gen-policy ingress list
#   sqconn:<locals>    the same for the connection batch's kernels
#   pmc:<config>       HBM traffic PMC passes (tools/gpu_pmc.sh)
#   fetchgp:<layout>:<blocks>  FETCH_SIZE of the classify kernel on a gen-policy
#                      ingress list against its algorithmic bytes
set -e -o pipefail
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export TMPDIR=/tmp
lib() { [ "$1" = default ] && echo $R/vpp_amd/libcontivcls.so || echo $R/vpp_amd/variants/lib_$1.so; }
B="--steps 20 --warmup 5 --cpu-sample 0"
for step in "$@"; do
  kind=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=
  echo "== $step"
  case $kind in
  parity)
    files=tests; [ -n "$arg" ] && files=$(echo $arg | tr , ' ')
    timeout -k 10 900 python -u -m pytest $files -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
    tail -2 $O/pytest.log ;;
  bench)
    timeout -k 10 300 python bench.py --config $arg $B > $O/bench_c$arg.json 2> $O/bench_c$arg.err
    python3 tools/jl.py $O/bench_c$arg.json value ms_per_step step_ms_median roofline.kernel_ms_median roofline.stream_floor_ms roofline.frac ;;
  benchk)
    # benchk:<config>[:<tag>[:key=value...]]: the bench line under rocprofv3 kernel stats (no stream floor)
    c=${arg%%:*}; rest=${arg#*:}; t=""; opts=""
    if [ "$rest" != "$arg" ]; then t=_${rest%%:*}; [ "$rest" != "${rest%%:*}" ] && for o in $(echo ${rest#*:} | tr : ' '); do opts="$opts --opt $o"; done; fi
    k=benchk_c$c$t
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$k -o run --output-format csv -- python3 $R/bench.py --config $c $B --no-stream-floor $opts > $O/$k.json 2> $O/$k.err)
    echo "-- config $c$t:$opts"; python3 tools/jl.py $O/$k.json value ms_per_step step_ms_median roofline.kernel_ms_median
    python3 tools/kstats.py $O/$k/run_kernel_stats.csv | grep -E "classify|finish|fold" ;;
  events)
    for ev in 2 1 0; do
      timeout -k 10 200 python bench.py --config $arg $B --events $ev > $O/ev_c${arg}_$ev.json 2> /dev/null
      python3 tools/jl.py $O/ev_c${arg}_$ev.json value ms_per_step step_ms_median host_submit_ms_per_step roofline.kernel_ms_median
    done ;;
  kstats)
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_c$arg -o run --output-format csv -- python3 $R/bench.py --config $arg $B > $O/kt_c$arg.log 2>&1)
    python3 tools/kstats.py $O/kt_c$arg/run_kernel_stats.csv
    python3 tools/gaps.py $O/kt_c$arg/run_kernel_trace.csv --last 120 ;;
  conn)
    for v in $(echo $arg | tr , ' '); do
      for loc in 12 64; do
        (cd /tmp && CONTIVCLS_LIB=$(lib $v) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/conn_${v}_$loc -o run --output-format csv -- python3 $R/tools/conn_bench.py --locals $loc --cpu-sample $([ $v = default ] && echo 20000 || echo "0 --no-check") > $O/conn_${v}_$loc.json 2> $O/conn_${v}_$loc.err)
        echo "-- $v, $loc local ACLs"
        python3 tools/jl.py $O/conn_${v}_$loc.json hbm_resident hbm_resident_counted
        python3 tools/kstats.py $O/conn_${v}_$loc/run_kernel_stats.csv | grep -E "connect|pair"
      done
    done ;;
  connx)
    # connx:<locals>:<tag>[:key=value...]: a connection bench under library options, kernel stats
    loc=${arg%%:*}; rest=${arg#*:}; t=${rest%%:*}; opts=""; [ "$rest" != "$t" ] && for o in $(echo ${rest#*:} | tr : ' '); do opts="$opts --opt $o"; done
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/connx_${t}_$loc -o run --output-format csv -- python3 $R/tools/conn_bench.py --locals $loc --cpu-sample 0 --cpu-fast-sample 0 --opt debug_conn=1 $opts > $O/connx_${t}_$loc.json 2> $O/connx_${t}_$loc.err)
    echo "-- $t, $loc local ACLs:$opts"; awk '/connect: n 4194304/ && !/bitmaps 0 / && !seen[$0]++ && c++ < 4' $O/connx_${t}_$loc.err
    python3 tools/jl.py $O/connx_${t}_$loc.json hbm_resident hbm_resident_counted
    python3 tools/kstats.py $O/connx_${t}_$loc/run_kernel_stats.csv | grep -E "connect|pair|rows" ;;
  connn)
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/connn_$arg -o run --output-format csv -- python3 $R/tools/conn_bench.py --locals 12 --n $arg --cpu-sample 0 > $O/connn_$arg.json 2> $O/connn_$arg.err)
    python3 tools/jl.py $O/connn_$arg.json hbm_resident hbm_resident_counted
    python3 tools/kstats.py $O/connn_$arg/run_kernel_stats.csv | grep -E "connect|pair|stream_conn" ;;
  gp16)
    for v in $(echo $arg | tr , ' '); do
      CONTIVCLS_LIB=$(lib $v) timeout -k 10 300 python tools/genpolicy_bench.py --layout 16 --v6 0.1 --blocks 20 200 1000 --match ingress --packets 67108864 --iters 5 > $O/gp16_$v.jsonl 2> $O/gp16_$v.err
      echo "-- $v"; python3 tools/jl.py $O/gp16_$v.jsonl rules list_mode kernel_ms Gpps_kernel Gpps_wall
    done ;;
  gp)
    for n in 67108864 268435456; do
      timeout -k 10 300 python tools/genpolicy_bench.py --layout $arg --blocks 20 --match ingress --packets $n --iters 5 > $O/gp${arg}_$n.jsonl 2> $O/gp${arg}_$n.err
      echo "-- $n packets"; python3 tools/jl.py $O/gp${arg}_$n.jsonl kernel_ms Gpps_kernel hbm_frac_kernel
    done
    timeout -k 10 300 python tools/genpolicy_bench.py --layout $arg --blocks 20 --match ingress --packets 67108864 --iters 5 --mix 0.5 0.5 0 0 > $O/gp${arg}_tcpudp.jsonl 2> $O/gp${arg}_tcpudp.err
    echo "-- TCP/UDP only"; python3 tools/jl.py $O/gp${arg}_tcpudp.jsonl kernel_ms Gpps_kernel hbm_frac_kernel ;;
  gpmix)
    for mix in "0.445 0.445 0.11 0" "0.495 0.495 0 0.01"; do
      timeout -k 10 300 python tools/genpolicy_bench.py --layout $arg --blocks 20 --match ingress --packets 67108864 --iters 5 --mix $mix > $O/gpmix$arg.jsonl 2> $O/gpmix$arg.err
      echo "-- mix $mix"; python3 tools/jl.py $O/gpmix$arg.jsonl kernel_ms Gpps_kernel hbm_frac_kernel
    done ;;
  gpb)
    bud=${arg%%:*}; rest=${arg#*:}; lay=${rest%%:*}; nb=${rest#*:}
    timeout -k 10 300 python tools/genpolicy_bench.py --opt lds_budget=$bud --layout $lay --v6 0.1 --blocks $nb --match ingress --packets 67108864 --iters 5 > $O/gpb_${bud}_${lay}_$nb.jsonl 2> $O/gpb_${bud}_${lay}_$nb.err
    python3 tools/jl.py $O/gpb_${bud}_${lay}_$nb.jsonl rules ctr16 lds_slots slots kernel_ms Gpps_kernel ;;
  ab)
    cfg=${arg%%:*}; v=${arg#*:}
    bash tools/gpu_ab.sh $TAG $cfg $(lib $v) ;;
  sq)
    bash tools/sq_profile.sh ${TAG}_c$arg --config $arg > /dev/null 2>&1
    cat gpurun_out/sq_${TAG}_c$arg/summary.txt ;;
  sqgp)
    lay=${arg%%:*}; nb=${arg#*:}
    SQ_CMD="python3 $R/tools/genpolicy_bench.py --layout $lay --v6 0.1 --blocks $nb --match ingress --iters 2 --packets 67108864" bash tools/sq_profile.sh ${TAG}_gp${lay}_$nb > /dev/null 2>&1
    cat gpurun_out/sq_${TAG}_gp${lay}_$nb/summary.txt ;;
  fetchgp)
    lay=${arg%%:*}; nb=${arg#*:}
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_gp${lay}_$nb -o run --output-format csv -- python3 $R/tools/genpolicy_bench.py --layout $lay --v6 0.1 --blocks $nb --match ingress --iters 2 --packets 67108864 > $O/fetch_gp${lay}_$nb.log 2>&1)
    python3 - $O/fetch_gp${lay}_$nb $lay <<'PY'
import csv, glob, sys
vals = [float(r["Counter_Value"]) for f in glob.glob(sys.argv[1] + "/*/run_counter_collection.csv")
        for r in csv.DictReader(open(f)) if "classify" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE"]
alg = (12 if sys.argv[2] == "4" else 36) * 67108864 - 67108864       # reads only (the verdict byte is written)
for v in vals:
    print("FETCH_SIZE %.0f KiB -> %.3f GB read (x2, gfx950), %.3fx the %.3f GB algorithmic reads" % (v, v * 2048 / 1e9, v * 2048 / alg, alg / 1e9))
PY
    ;;
  sqconn)
    SQ_KERNELS=connect_kernel,classify4_pair SQ_CMD="python3 $R/tools/conn_bench.py --locals $arg --count 1 --iters 2 --cpu-sample 0 --cpu-fast-sample 0" bash tools/sq_profile.sh ${TAG}_conn$arg > /dev/null 2>&1
    cat gpurun_out/sq_${TAG}_conn$arg/summary.txt ;;
  pmc)
    bash tools/gpu_pmc.sh ${TAG}_pmc$arg $arg > /dev/null 2>&1
    grep -h "ratio\|source_hash" gpurun_out/${TAG}_pmc$arg/pmc.json ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
