#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 500 python tools/probe_torch_conv.py 16 > gpurun_out/probe_conv.txt 2>&1
