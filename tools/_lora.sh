mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_layers.py > gpurun_out/pytest_k.log 2>&1 || { tail -30 gpurun_out/pytest_k.log; exit 1; }
tail -1 gpurun_out/pytest_k.log
for v in 0 1 2 3; do
  echo "== skinny variant $v"; PSO_SKINNY_VARIANT=$v TN_ONLY_AUTO=1 timeout -k 10 120 python -u tools/tn_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done > gpurun_out/tn_bench.txt
cat gpurun_out/tn_bench.txt
timeout -k 10 120 python -u tools/attn_bench.py > gpurun_out/attn_bench.txt 2>&1 || exit 1
cat gpurun_out/attn_bench.txt
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
cut -c1-200 gpurun_out/bench.json
