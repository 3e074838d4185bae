timeout -k 10 400 python -u -m pytest -x -q -s --timeout 380 --timeout-method thread tests/test_gpu_fullsize.py -k c2 > gpurun_out/c2t.log 2>&1; echo c2 rc=$?; grep -E "C2 @1024|passed|failed" gpurun_out/c2t.log | cut -c1-3000
SKIP_TESTS=1 bash tools/gpu_full.sh
