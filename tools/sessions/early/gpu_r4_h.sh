#!/bin/bash
# G=8 (per-GPU load of the 8-GPU headline) A/B of the conv1 forward row split and the conv2 wgrad split-K, the Tiny /
# CIFAR round-time diagnosis of round 3 (tools/sessions/early/gpu_r3_bc.sh), and the headline bench
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r4h
kb() {  # name, env..., -- G
  local name=$1; shift; local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python tools/kbench.py "$@" 10 > gpurun_out/r4h/kb_$name.txt 2>&1 || { tail -5 gpurun_out/r4h/kb_$name.txt; exit 1; }
  echo "$name: $(grep 'full train' gpurun_out/r4h/kb_$name.txt | head -1) | $(grep -E '^conv1_fwd|^conv2_wgrad' gpurun_out/r4h/kb_$name.txt | tr -s ' ' | tr '\n' ';')"
}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "conv1 or alexnet" > gpurun_out/r4h/pytest_conv1.txt 2>&1 || { tail -30 gpurun_out/r4h/pytest_conv1.txt; exit 1; }
tail -2 gpurun_out/r4h/pytest_conv1.txt
kb g64_tapord0 NIDT_C1_TAPORD=0 -- 64
kb g64_tapord1 X=1 -- 64
kb g64_tapord0b NIDT_C1_TAPORD=0 -- 64
kb g64_tapord1b X=1 -- 64
kb g8_base X=1 -- 8
kb g8_nq2 NIDT_C1_NQ=2 -- 8
kb g8_nq3 NIDT_C1_NQ=3 -- 8
kb g8_ns8 NIDT_WG_TRI_NS=8 -- 8
kb g8_ns16 NIDT_WG_TRI_NS=16 -- 8
kb g8_ns24 NIDT_WG_TRI_NS=24 -- 8
kb g8_base2 X=1 -- 8
kb g64_nq2 NIDT_C1_NQ=2 -- 64
timeout -k 10 300 python bench.py --clients 8 --steps 10 --warmup 3 > gpurun_out/r4h/bench_c8.json 2>&1 || exit 1
echo "bench 8 clients: $(grep -o '"value": [0-9.]*' gpurun_out/r4h/bench_c8.json)"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r4h/bench.json 2>&1 || exit 1
echo "bench 64 clients: $(grep -o '"value": [0-9.]*' gpurun_out/r4h/bench.json)"
bash tools/sessions/early/gpu_r3_bc.sh 2>&1 | tee gpurun_out/r4h/r3bc.txt
cp -r gpurun_out/r3bc gpurun_out/r4h/ 2>/dev/null
