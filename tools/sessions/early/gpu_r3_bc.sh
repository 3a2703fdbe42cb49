#!/bin/bash
# diagnosis of the Tiny (batch 128) / SubAvg round-time spread: session-3 switches one at a time, interleaved
set -o pipefail
mkdir -p gpurun_out/r3bc
export PYTHONUNBUFFERED=1
run() {  # name, env assignments..., then bench args after --
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u tools/bench_cifar.py "$@" > gpurun_out/r3bc/$name.txt 2>&1 || { tail -5 gpurun_out/r3bc/$name.txt; exit 1; }
  echo "$name: $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3bc/$name.txt) warmup $(grep -o '"warmup_round_s": [^]]*' gpurun_out/r3bc/$name.txt)"
}
T="--algorithm subavg --dataset tiny --batch 128 --rounds 1 --warmup 1"
S="--algorithm subavg --rounds 2 --warmup 1"
run tiny_default X=1 -- $T
run tiny_evalpad0 NIDT_EVAL_PAD=0 -- $T
run tiny_slab0 NIDT_2D_SLAB=0 -- $T
run tiny_head0 NIDT_CLS_HEAD=0 -- $T
run tiny_graphs0 NIDT_HIP_GRAPHS=0 -- $T
run tiny_default2 X=1 -- $T
run subavg_default X=1 -- $S
run subavg_evalpad0 NIDT_EVAL_PAD=0 -- $S
run subavg_graphs0 NIDT_HIP_GRAPHS=0 -- $S
run subavg_default2 X=1 -- $S
