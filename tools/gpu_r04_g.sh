set -e -o pipefail
# 16-byte classify: ordered prefetch (default build) against four-at-a-time
# without prefetch (lib_pf0): parity, gen-policy lists, config 5 A/B
O=gpurun_out/r04j; mkdir -p $O
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_v16.py tests/test_gpu_configurator.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for lib in default pf0; do
  L=$R/vpp_amd/libcontivcls.so; [ $lib = default ] || L=$R/vpp_amd/variants/lib_$lib.so
  CONTIVCLS_LIB=$L timeout -k 10 300 python tools/genpolicy_bench.py --layout 16 --v6 0.1 --blocks 20 200 1000 --match ingress --packets 67108864 > $O/gp16_$lib.jsonl 2> $O/gp16_$lib.err
  echo "== $lib"
  python3 tools/jl.py $O/gp16_$lib.jsonl rules list_mode kernel_ms Gpps_kernel Gpps_wall
done
bash tools/gpu_ab.sh r04j 5 vpp_amd/variants/lib_pf0.so
