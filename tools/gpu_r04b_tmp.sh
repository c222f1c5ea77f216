set -e -o pipefail
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_connect_scale.py tests/test_gpu_policy_chain.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_conn.log 2>&1 || { tail -40 $O/pytest_conn.log; exit 1; }
tail -2 $O/pytest_conn.log
bash tools/gpu_conn_prof.sh r04c_conn
timeout -k 10 120 ./tools/stream_loader.bin > $O/stream_loader.txt 2>&1; cat $O/stream_loader.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu_ab.sh r04c 3 vpp_amd/variants/lib_r03.so
bash tools/gpu_ab.sh r04c 5 vpp_amd/variants/lib_r03.so
