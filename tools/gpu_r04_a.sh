set -e -o pipefail
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_connect_scale.py tests/test_gpu_policy_chain.py tests/test_gpu_parity.py tests/test_gpu_v16.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_a.log 2>&1 || { tail -40 $O/pytest_a.log; exit 1; }
tail -2 $O/pytest_a.log
bash tools/gpu_conn_prof.sh r04d_conn
timeout -k 10 120 ./tools/stream_loader.bin > $O/stream_loader.txt 2>&1; cat $O/stream_loader.txt
bash tools/gpu_cfg2.sh r04d_cfg2
timeout -k 10 600 python -u -m pytest tests/test_gpu_configurator.py -m gpu -x -q -k "v16 or default_scale" --timeout 900 --timeout-method thread > $O/pytest_gp16.log 2>&1 || { tail -40 $O/pytest_gp16.log; exit 1; }
tail -2 $O/pytest_gp16.log
