set -e -o pipefail
# gen-policy lists in the 16-byte layout: the default build (four packets
# classified together) against the two-at-a-time build; IPv6 share 0 / 0.1 /
# 0.5; then the SQ counter passes of the 20- and 200-block ingress lists
O=gpurun_out/r04g; mkdir -p $O
R=$(pwd)
for lib in default v_full_pairpf; do
  L=$R/vpp_amd/libcontivcls.so; [ $lib = default ] || L=$R/vpp_amd/variants/lib_$lib.so
  for v in 0 0.1 0.5; do
    CONTIVCLS_LIB=$L timeout -k 10 300 python tools/genpolicy_bench.py --layout 16 --v6 $v --blocks 20 200 1000 --match ingress --packets 67108864 > $O/gp16_${lib}_v$v.jsonl 2> $O/gp16_${lib}_v$v.err
    echo "== $lib v6 $v"
    python3 tools/jl.py $O/gp16_${lib}_v$v.jsonl rules list_mode kernel_ms Gpps_kernel Gpps_wall
    [ $lib = default ] || break
  done
done
for b in 20 200; do
SQ_CMD="python3 $R/tools/genpolicy_bench.py --layout 16 --v6 0.1 --blocks $b --match ingress --iters 2 --packets 67108864" bash tools/sq_profile.sh gp16_$b > /dev/null 2>&1
cat gpurun_out/sq_gp16_$b/summary.txt
done
