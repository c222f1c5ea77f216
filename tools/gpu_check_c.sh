set -e -o pipefail
O=gpurun_out/r02s4_c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "beyond_one_launch or config3_full" --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
tail -4 $O/pytest.log
timeout -k 10 300 python tools/genpolicy_bench.py --blocks 20 60 200 > $O/gp.jsonl 2> $O/gp.err
python3 tools/jl.py $O/gp.jsonl rules Gpps_wall kernel_ms Gpps_kernel lds_slots slots
timeout -k 10 500 python tools/commit_bench.py --pods 1000 --engine gpu > $O/commit.json 2> $O/commit.err
cat $O/commit.json
