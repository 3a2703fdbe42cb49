#!/bin/bash
# round 4, call a: smfmac / LDS probe, headline bench (1 GPU, both launch shapes of --gpus 1)
set -o pipefail
mkdir -p gpurun_out/r4a
timeout -k 10 60 tools/probes/smfmac_probe gpurun_out/r4a > gpurun_out/r4a/probe.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r4a/bench.json 2> gpurun_out/r4a/bench.err || exit 1
timeout -k 10 120 python bench.py --gpus 2 --steps 1 --warmup 1 > gpurun_out/r4a/bench_g2_refuse.txt 2>&1; echo "g2 rc=$?" >> gpurun_out/r4a/bench_g2_refuse.txt
cat gpurun_out/r4a/probe.txt gpurun_out/r4a/bench.json gpurun_out/r4a/bench_g2_refuse.txt
