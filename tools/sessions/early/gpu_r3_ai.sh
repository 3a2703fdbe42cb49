#!/bin/bash
# skinny deep-layer convs at few clients: 256-position blocks + wide split-K (NIDT_FWD_SMALLBP / NIDT_FWDG_*) A/B
set -o pipefail
mkdir -p gpurun_out/r3ai
export PYTHONUNBUFFERED=1
run() {  # name smallbp slots minks kmax
  export NIDT_FWD_SMALLBP=$2 NIDT_FWDG_SLOTS=$3 NIDT_FWDG_MINKS=$4 NIDT_FWDG_KMAX=$5
  timeout -k 10 200 python -u tools/bench_cifar.py --algorithm subavg --rounds 2 --warmup 1 > gpurun_out/r3ai/subavg_$1.txt 2>&1 || exit 1
  echo "subavg $1 ($2 $3 $4 $5): $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3ai/subavg_$1.txt)"
}
run base 0 0 0 0
run bp1k_k16 1024 512 4 16
run bp1k_k8 1024 0 0 0
run bp4k_k16 4096 512 4 16
run base2 0 0 0 0
run bp1k_k32 1024 1024 2 32
