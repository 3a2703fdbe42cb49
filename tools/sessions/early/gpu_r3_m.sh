#!/bin/bash
# ResNet-18-GN engine analysis: per-layer kernel bench at SubAvg (G=10) and DisPFL (G=100) client counts, and a
# kernel timeline of one DisPFL round
set -o pipefail
mkdir -p gpurun_out/r3m
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for g in 10 100; do
  timeout -k 10 300 python -u tools/kbench_resnet.py $g 10 > gpurun_out/r3m/kbench_resnet_g$g.txt 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/r3m/kbench_resnet_g$g.txt
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/dprof -o run -- python3 -u tools/bench_cifar.py \
  --algorithm dispfl --rounds 1 --warmup 1 > gpurun_out/r3m/prof_dispfl.txt 2>&1 || exit 1
db=$(find /tmp/dprof -name "*.db" | head -1)
s=$(python3 -c "import json; print([json.loads(l) for l in open('gpurun_out/r3m/prof_dispfl.txt') if l.startswith('{')][0]['s_per_round'])")
ms=$(python3 -c "print(int(float('$s') * 1000))")
python3 tools/prof_summary.py "$db" gpurun_out/r3m/round_kernels_dispfl.txt --window-ms $ms --top 30 > /dev/null
head -34 gpurun_out/r3m/round_kernels_dispfl.txt
