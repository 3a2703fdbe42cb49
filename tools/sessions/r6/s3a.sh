#!/bin/bash
# one steady training step, dispatch by dispatch: CIFAR SubAvg (G=10, B=16) and the 8-client AlexNet3D step
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s3a; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/cfa -o run -- python3 -u tools/bench_cifar.py --algorithm subavg --rounds 1 --warmup 1 > $OUT/subavg_prof.txt 2>&1 || { tail -20 $OUT/subavg_prof.txt; exit 1; }
db=$(find /tmp/cfa -name "*.db" | head -1)
python3 tools/step_timeline.py "$db" $OUT/subavg_step.txt && tail -3 $OUT/subavg_step.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/c8 -o run -- python3 -u bench.py --clients 8 --steps 2 --warmup 1 > $OUT/c8_prof.txt 2>&1 || { tail -20 $OUT/c8_prof.txt; exit 1; }
db=$(find /tmp/c8 -name "*.db" | head -1)
python3 tools/step_timeline.py "$db" $OUT/c8_step.txt --marker k_conv1_fwd --must k_local_step && tail -3 $OUT/c8_step.txt
