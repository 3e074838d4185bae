mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_layers.py -q -x -k attention --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_attn.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/pytest_attn.log | head -20; exit $rc; }
ATTN_VARIANTS=${ATTN_VARIANTS:-0,22,44} timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn_bench.txt 2>&1; rc=$?
cat gpurun_out/attn_bench.txt
exit $rc
