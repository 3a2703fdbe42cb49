#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r4c
timeout -k 10 60 tools/probes/smfmac_probe gpurun_out/r4c > gpurun_out/r4c/probe.txt 2>&1 || exit 1
grep -E "rate|throughput" gpurun_out/r4c/probe.txt
