#!/bin/bash
# final-tree numbers of the secondary configs: config 5 steady state, CIFAR SubAvg / DisPFL
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4aj; mkdir -p $OUT
timeout -k 10 400 python3 -u tools/config5_resnet3d.py --clients 256 --train-per-client 36 \
  --test-per-client 9 --batch 4 --group 32 --rounds 3 --warmup 1 > $OUT/config5.txt 2>&1 \
  || { tail -30 $OUT/config5.txt; exit 1; }
echo "config5: $(grep '^{' $OUT/config5.txt | grep -o '"steady_s_per_round": [0-9.]*\|"s_round_each": [^]]*]\|"peak_gib_each_round": [^]]*]' | tr '\n' ' ')"
timeout -k 10 300 python tools/bench_cifar.py --rounds 2 > $OUT/cifar_subavg.txt 2>&1 || exit 1
echo "cifar subavg: $(grep -o '"value": [0-9.]*\|"s_round_each": [^]]*]' $OUT/cifar_subavg.txt | tr '\n' ' ')"
timeout -k 10 300 python tools/bench_cifar.py --algorithm dispfl --rounds 1 > $OUT/cifar_dispfl.txt 2>&1 || exit 1
echo "cifar dispfl: $(grep -o '"value": [0-9.]*\|"s_round_each": [^]]*]' $OUT/cifar_dispfl.txt | tr '\n' ' ')"
