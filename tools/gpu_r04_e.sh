set -e -o pipefail
# connection batches: kernel builds A/B (prefetch variants), 12 and 64 local
# ACLs, batch times and rocprofv3 kernel stats per build
O=gpurun_out/r04h; mkdir -p $O
R=$(pwd)
export TMPDIR=/tmp
for v in base ids_pairpf full_pairpf; do
  L=$R/vpp_amd/variants/lib_v_$v.so
  for loc in 12 64; do
    (cd /tmp && CONTIVCLS_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/${v}_$loc -o run --output-format csv -- python3 $R/tools/conn_bench.py --locals $loc --cpu-sample 0 > $R/$O/${v}_$loc.json 2> $R/$O/${v}_$loc.err)
    echo "== $v locals $loc"
    python3 tools/jl.py $O/${v}_$loc.json hbm_resident hbm_resident_counted
    python3 tools/kstats.py $O/${v}_$loc/run_kernel_stats.csv | grep -E "connect|pair"
  done
done
