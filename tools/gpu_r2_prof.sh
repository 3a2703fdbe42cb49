#!/bin/bash
# rocprofv3 kernel timelines of one personalized-algorithm round each + the skewed headline round
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for spec in "dispfl 0.1 0" "subavg 0.1 0" "fedfomo 0.1 0" "dpsgd 0.1 0" "salientgrads 1.0 1.0"; do
  set -- $spec
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$1 -o run -- python3 bench.py --steps 2 --warmup 1 --algorithm $1 --frac $2 --size-skew $3 > gpurun_out/prof_$1.txt 2>&1
  rc=$?; echo "prof $1 rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
