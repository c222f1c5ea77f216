set -e -o pipefail
O=gpurun_out/r04i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_v16.py tests/test_gpu_configurator.py tests/test_gpu_connect_scale.py tests/test_gpu_policy_chain.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu_r04_e.sh
bash tools/gpu_r04_d.sh
