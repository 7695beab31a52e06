set -o pipefail
O=gpurun_out/r6s20; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_graph_memset_gpu.py tests/test_graph_gpu.py tests/test_graph_cifar_o2_gpu.py tests/test_graph_dp_gpu.py > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -40
exit $rc
