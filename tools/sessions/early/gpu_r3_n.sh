#!/bin/bash
# bf16 residual-gradient stream (3D + 2D ResNet engines): GPU tests of both engines, config 5 round with a kernel
# timeline, the CIFAR SubAvg / DisPFL benches
set -o pipefail
mkdir -p gpurun_out/r3n
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_resnet3d.py tests/test_gpu_resnet2d.py -v --timeout 300 \
  --timeout-method thread > gpurun_out/r3n/pytest.txt 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r3n/pytest.txt | tail -3; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/c5profn -o run -- python3 -u tools/config5_resnet3d.py \
  --clients 256 --train-per-client 36 --test-per-client 9 --batch 4 --group 32 --rounds 1 \
  > gpurun_out/r3n/config5.txt 2>&1 || { tail -30 gpurun_out/r3n/config5.txt; exit 1; }
grep '^{' gpurun_out/r3n/config5.txt | cut -c1-400
db=$(find /tmp/c5profn -name "*.db" | head -1)
[ -n "$db" ] && python3 tools/prof_summary.py "$db" gpurun_out/r3n/config5_kernels.txt --top 40 > /dev/null 2>&1
head -25 gpurun_out/r3n/config5_kernels.txt
for spec in "subavg 2" "dispfl 1"; do
  set -- $spec
  timeout -k 10 600 python -u tools/bench_cifar.py --algorithm $1 --rounds $2 --warmup 1 > gpurun_out/r3n/cifar_$1.txt 2>&1 || exit 1
  grep '^{' gpurun_out/r3n/cifar_$1.txt | cut -c1-250
done
