set -e -o pipefail
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_connect_scale.py tests/test_gpu_policy_chain.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_a.log 2>&1 || { tail -40 $O/pytest_a.log; exit 1; }
tail -2 $O/pytest_a.log
bash tools/gpu_conn_prof.sh r04f_conn
for c in 3 2; do for ev in 2 1 0; do
timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --cpu-sample 0 --events $ev > $O/ev_c${c}_$ev.json 2>/dev/null
python3 tools/jl.py $O/ev_c${c}_$ev.json value ms_per_step step_ms_median host_submit_ms_per_step roofline.kernel_ms_median roofline.stream_floor_ms
done; done
timeout -k 10 500 python tools/genpolicy_bench.py --layout 16 --v6 0.1 --blocks 20 200 1000 --packets 67108864 > $O/gp16.jsonl 2> $O/gp16.err
python3 tools/jl.py $O/gp16.jsonl workload rules list_mode lds_resident kernel_ms Gpps_kernel Gpps_wall
