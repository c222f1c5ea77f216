set -e -o pipefail
O=gpurun_out/r02s4_gp; mkdir -p $O
timeout -k 10 300 python tools/ab_inproc.py --rounds 8 vpp_amd/variants/lib_pf0.so vpp_amd/variants/lib_pf2.so vpp_amd/libcontivcls.so > $O/ab.log 2>&1
grep median $O/ab.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_configurator.py -m gpu -v -k gen_policy --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
tail -6 $O/pytest.log
timeout -k 10 300 python tools/genpolicy_bench.py --blocks 20 60 200 > $O/gp.jsonl 2> $O/gp.err
cat $O/gp.jsonl
timeout -k 10 300 python tools/genpolicy_bench.py --blocks 1000 --packets 16777216 --iters 3 > $O/gp1000.jsonl 2> $O/gp1000.err
cat $O/gp1000.jsonl
