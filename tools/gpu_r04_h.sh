set -e -o pipefail
# default build (dense connection calls in place, 16-byte OTHER reps only
# for packets classified in place) against lib_pf0 (the committed kernels
# before both): parity, connection batches, gen-policy lists; then the
# 20-block list's batch-size and protocol-mix sweeps in both layouts
O=gpurun_out/r04k; mkdir -p $O
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_connect_scale.py tests/test_gpu_policy_chain.py tests/test_gpu_v16.py tests/test_gpu_configurator.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
export TMPDIR=/tmp
for v in default pf0; do
  L=$R/vpp_amd/libcontivcls.so; [ $v = default ] || L=$R/vpp_amd/variants/lib_$v.so
  CONTIVCLS_LIB=$L timeout -k 10 300 python tools/genpolicy_bench.py --layout 16 --v6 0.1 --blocks 20 200 1000 --match ingress --packets 67108864 --iters 5 > $O/gp16_$v.jsonl 2> $O/gp16_$v.err
  echo "== gen-policy 16-byte $v"; python3 tools/jl.py $O/gp16_$v.jsonl rules kernel_ms Gpps_kernel Gpps_wall
  for loc in 12 64; do
    (cd /tmp && CONTIVCLS_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/${v}_$loc -o run --output-format csv -- python3 $R/tools/conn_bench.py --locals $loc --cpu-sample 0 > $R/$O/${v}_$loc.json 2> $R/$O/${v}_$loc.err)
    echo "== $v locals $loc"
    python3 tools/jl.py $O/${v}_$loc.json hbm_resident hbm_resident_counted
    python3 tools/kstats.py $O/${v}_$loc/run_kernel_stats.csv | grep -E "connect|pair"
  done
done
for lay in 4 16; do
  for n in 67108864 268435456; do
    timeout -k 10 300 python tools/genpolicy_bench.py --layout $lay --blocks 20 --match ingress --packets $n --iters 5 > $O/gp${lay}_$n.jsonl 2> $O/gp${lay}_$n.err
    echo "== layout $lay packets $n"; python3 tools/jl.py $O/gp${lay}_$n.jsonl kernel_ms Gpps_kernel hbm_frac_kernel
  done
  timeout -k 10 300 python tools/genpolicy_bench.py --layout $lay --blocks 20 --match ingress --packets 67108864 --iters 5 --mix 0.5 0.5 0 0 > $O/gp${lay}_tcpudp.jsonl 2> $O/gp${lay}_tcpudp.err
  echo "== layout $lay TCP/UDP only"; python3 tools/jl.py $O/gp${lay}_tcpudp.jsonl kernel_ms Gpps_kernel hbm_frac_kernel
done
