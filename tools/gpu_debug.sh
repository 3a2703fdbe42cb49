#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/debug_alexnet.py > gpurun_out/debug.txt 2>&1
