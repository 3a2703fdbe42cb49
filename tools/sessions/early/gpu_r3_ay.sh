#!/bin/bash
# rocprofv3 kernel timelines of one measured CIFAR SubAvg / DisPFL round with the session-3 ResNet engine (summaries only)
set -o pipefail
mkdir -p gpurun_out/r3ay
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for alg in subavg dispfl; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_c$alg -o run -- python3 tools/bench_cifar.py --algorithm $alg --rounds 1 --warmup 1 > gpurun_out/r3ay/prof_cifar_$alg.txt 2>&1
  rc=$?; echo "prof $alg rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/r3ay/prof_cifar_$alg.txt; exit $rc; fi
  db=$(find /tmp/prof_c$alg -name "*.db" | head -1)
  ms=$(python3 -c "import json; print([json.loads(l) for l in open('gpurun_out/r3ay/prof_cifar_$alg.txt') if l.startswith('{')][0]['s_per_round']*1000)")
  python3 tools/prof_summary.py "$db" gpurun_out/r3ay/prof_cifar_${alg}_summary.txt --window-ms $ms --top 45 > /dev/null
  rm -rf /tmp/prof_c$alg
done
