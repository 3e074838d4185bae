timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; echo rc=$?; tail -3 gpurun_out/bench.err
