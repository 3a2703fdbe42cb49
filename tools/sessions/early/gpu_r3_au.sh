#!/bin/bash
# Verification after the 2-D slab convs: full GPU suite, smoke, headline bench (driver shape), CIFAR / Tiny benches
set -o pipefail
mkdir -p gpurun_out/r3au
export PYTHONUNBUFFERED=1
O=gpurun_out/r3au
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -2 $O/pytest_gpu.txt; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $O/pytest_gpu.txt | head -20; exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
echo "smoke ok"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.txt 2>&1 || { tail -20 $O/bench.txt; exit 1; }
tail -1 $O/bench.txt
for a in subavg dispfl; do
  timeout -k 10 300 python -u tools/bench_cifar.py --algorithm $a --rounds 2 --warmup 1 > $O/cifar_$a.txt 2>&1 || exit 1
  echo "cifar $a $(grep -o '"s_per_round": [0-9.]*' $O/cifar_$a.txt)"
done
timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --dataset tiny --rounds 2 --warmup 1 > $O/tiny_subavg.txt 2>&1 || exit 1
echo "tiny subavg $(grep -o '"s_per_round": [0-9.]*' $O/tiny_subavg.txt)"
