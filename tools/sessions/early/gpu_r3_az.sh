#!/bin/bash
# padded-bucket evaluation of ragged test splits (NIDT_EVAL_PAD): runner / personalized / ResNet GPU tests, then
# interleaved A/B on CIFAR SubAvg / DisPFL and the AlexNet size-skew bench, plus a no-eval CIFAR round for reference
set -o pipefail
mkdir -p gpurun_out/r3az
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_resnet2d.py tests/test_gpu_resnet3d.py -x -v -s \
  --timeout 300 --timeout-method thread > gpurun_out/r3az/pytest.txt 2>&1
rc=$?; tail -1 gpurun_out/r3az/pytest.txt; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAIL" gpurun_out/r3az/pytest.txt | head -30; exit $rc; fi
for arm in 1 0 1 0; do
  export NIDT_EVAL_PAD=$arm
  timeout -k 10 200 python -u tools/bench_cifar.py --algorithm subavg --rounds 2 --warmup 1 > gpurun_out/r3az/subavg_$arm.txt 2>&1 || exit 1
  echo "pad=$arm: subavg $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3az/subavg_$arm.txt)"
done
timeout -k 10 200 python -u tools/bench_cifar.py --algorithm subavg --rounds 2 --warmup 1 --no-eval > gpurun_out/r3az/subavg_noeval.txt 2>&1 || exit 1
echo "no eval: subavg $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3az/subavg_noeval.txt)"
for arm in 1 0; do
  export NIDT_EVAL_PAD=$arm
  timeout -k 10 300 python -u tools/bench_cifar.py --algorithm dispfl --rounds 1 --warmup 1 > gpurun_out/r3az/dispfl_$arm.txt 2>&1 || exit 1
  echo "pad=$arm: dispfl $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3az/dispfl_$arm.txt)"
done
for arm in 1 0; do
  export NIDT_EVAL_PAD=$arm
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --size-skew 1.0 > gpurun_out/r3az/skew_$arm.txt 2>&1 || exit 1
  echo "pad=$arm: alexnet size skew 1.0 $(grep -o '"value": [0-9.]*' gpurun_out/r3az/skew_$arm.txt)"
done
