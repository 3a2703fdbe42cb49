#!/bin/bash
# split-K thresholds for the small-grid client-grouped convs (CIFAR ResNet-18 tails): SubAvg / DisPFL s/round A/B
set -o pipefail
mkdir -p gpurun_out/r3ah
export PYTHONUNBUFFERED=1
run() {  # name slots minks
  export NIDT_FWDG_SLOTS=$2 NIDT_FWDG_MINKS=$3
  timeout -k 10 200 python -u tools/bench_cifar.py --algorithm subavg --rounds 2 --warmup 1 > gpurun_out/r3ah/subavg_$1.txt 2>&1 || exit 1
  echo "subavg $1 (slots $2 minks $3): $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3ah/subavg_$1.txt)"
}
run base 0 0
run s1024 1024 0
run s1024k8 1024 8
run s2048k6 2048 6
run base2 0 0
run s1024k8b 1024 8
