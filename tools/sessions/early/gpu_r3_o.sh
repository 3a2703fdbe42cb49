#!/bin/bash
# r3_n (bf16 residual gradient: tests, config 5 timeline, CIFAR benches), then conv1 fwd occupancy A/B, then the
# chaos-control cosines of the HIP-vs-fp32 runner comparison
bash tools/sessions/early/gpu_r3_n.sh; rc=$?
echo "r3_n rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
mkdir -p gpurun_out/r3o
for o in 2 3 2 3; do
  export NIDT_C1_OCC=$o
  timeout -k 10 300 python -u tools/kbench.py 64 10 > gpurun_out/r3o/kbench_occ$o.txt 2>&1 || exit 1
  echo "== occ $o"; grep -E "full train step|conv1_fwd|eval" gpurun_out/r3o/kbench_occ$o.txt
done
unset NIDT_C1_OCC
timeout -k 10 500 python -u tools/chaos_cosine.py fedavg salientgrads local > gpurun_out/r3o/chaos.txt 2>&1
rc=$?; grep '^{' gpurun_out/r3o/chaos.txt; exit $rc
