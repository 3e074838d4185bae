#!/bin/bash
# C3 full-UNet step under rocprofv3 (kernel trace): per-stream busy time and the main stream's idle gaps
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
rm -rf gpurun_out/c3p
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3p -o run -- \
  python3 bench.py --full-unet --mode dmd --num-steps 4 --pairs 1 --gas 1 --steps 3 --warmup 2 --no-cpu-baseline \
  --no-roofline --epochs 0 --no-extra > gpurun_out/c3p.json 2> gpurun_out/c3p.err || exit 1
