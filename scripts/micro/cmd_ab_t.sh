# parity tests of the tiled kernel, then the lab A/B (SMFV_LAB=1: HEAD's kernel)
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_ab.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-ab} bash scripts/micro/cmd_ab.sh
