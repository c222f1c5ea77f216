set -e -o pipefail
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu_ab.sh r04e 3 vpp_amd/variants/lib_r03.so
bash tools/gpu_ab.sh r04e 5 vpp_amd/variants/lib_r03.so
timeout -k 10 500 python tools/genpolicy_bench.py --layout 16 --v6 0.1 --blocks 20 200 1000 --packets 67108864 > $O/gp16.jsonl 2> $O/gp16.err
python3 tools/jl.py $O/gp16.jsonl workload rules list_mode lds_resident kernel_ms Gpps_kernel Gpps_wall
for c in 3 2; do for ev in 2 1 0; do
timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --cpu-sample 0 --events $ev > $O/ev_c${c}_$ev.json 2>/dev/null
python3 tools/jl.py $O/ev_c${c}_$ev.json value ms_per_step host_submit_ms_per_step roofline.kernel_ms_median
done; done
