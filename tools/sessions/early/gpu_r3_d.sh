#!/bin/bash
# ResNet-18-GN engine after round-3 changes (fused augmented input, 2-launch packing, sub-pixel dgrad):
# CLI tests incl. Tiny-ImageNet, the reference's timed CIFAR configs (SubAvg / DisPFL) with and without augmentation,
# Tiny SubAvg, and a kernel timeline of one SubAvg round
set -o pipefail
mkdir -p gpurun_out/r3d
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_cli.py -x -v --timeout 300 --timeout-method thread \
  -k "resnet18" > gpurun_out/r3d/pytest_cli.txt 2>&1
rc=$?; tail -3 gpurun_out/r3d/pytest_cli.txt; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
for spec in "subavg 2 " "dispfl 1 " "subavg 2 --no-augment" ; do
  set -- $spec
  timeout -k 10 600 python -u tools/bench_cifar.py --algorithm $1 --rounds $2 --warmup 1 $3 > gpurun_out/r3d/cifar_$1$3.txt 2>&1 || exit 1
  grep '^{' gpurun_out/r3d/cifar_$1$3.txt | cut -c1-330
done
timeout -k 10 600 python -u tools/bench_cifar.py --algorithm subavg --dataset tiny --batch 128 --rounds 1 --warmup 1 \
  > gpurun_out/r3d/tiny_subavg.txt 2>&1 || exit 1
grep '^{' gpurun_out/r3d/tiny_subavg.txt | cut -c1-330
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/cprof -o run -- python3 -u tools/bench_cifar.py \
  --algorithm subavg --rounds 1 --warmup 1 > gpurun_out/r3d/prof_subavg.txt 2>&1 || exit 1
db=$(find /tmp/cprof -name "*.db" | head -1)
s=$(python3 -c "import json; print([json.loads(l) for l in open('gpurun_out/r3d/prof_subavg.txt') if l.startswith('{')][0]['s_per_round'])")
ms=$(python3 -c "print(int(float('$s') * 1000))")
python3 tools/prof_summary.py "$db" gpurun_out/r3d/round_kernels_subavg.txt --window-ms $ms --top 30 > /dev/null
head -34 gpurun_out/r3d/round_kernels_subavg.txt
