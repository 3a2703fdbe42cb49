#!/bin/bash
# magic-number divisions in the forward prologue: numerics, then interleaved A/B against the previous build
# (NIDT_EXT_DIR = tools/ab_so) on CIFAR SubAvg, AlexNet at 8 clients and the 64-client kbench step
set -o pipefail
mkdir -p gpurun_out/r3as /tmp/oldext
cp tools/ab_so/_nidt_hip_old.so /tmp/oldext/_nidt_hip.cpython-310-x86_64-linux-gnu.so
export PYTHONUNBUFFERED=1 KBENCH_EVAL=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_resnet2d.py tests/test_gpu_resnet3d.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r3as/pytest.txt 2>&1
rc=$?; tail -1 gpurun_out/r3as/pytest.txt; if [ $rc -ne 0 ]; then tail -30 gpurun_out/r3as/pytest.txt; exit $rc; fi
for arm in new old new old; do
  if [ $arm = old ]; then export NIDT_EXT_DIR=/tmp/oldext; else unset NIDT_EXT_DIR; fi
  timeout -k 10 200 python -u tools/bench_cifar.py --algorithm subavg --rounds 2 --warmup 1 > gpurun_out/r3as/subavg_$arm.txt 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --clients 8 --steps 15 --warmup 3 > gpurun_out/r3as/b8_$arm.txt 2>&1 || exit 1
  timeout -k 10 300 python -u tools/kbench.py 64 6 > gpurun_out/r3as/kb_$arm.txt 2>&1 || exit 1
  echo "$arm: subavg $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3as/subavg_$arm.txt) | 8 clients $(grep -o '"value": [0-9.]*' gpurun_out/r3as/b8_$arm.txt) | $(grep 'full train step' gpurun_out/r3as/kb_$arm.txt)"
done
