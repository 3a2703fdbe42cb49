#!/bin/bash
# rocprofv3 kernel timelines of one round of each personalized algorithm + the skewed headline round; only the
# summaries come back (the rocpd databases are deleted on the box)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for spec in "dispfl 0.1 0" "subavg 0.1 0" "fedfomo 0.1 0" "dpsgd 0.1 0" "salientgrads 1.0 1.0"; do
  set -- $spec
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$1 -o run -- python3 bench.py --steps 1 --warmup 1 --algorithm $1 --frac $2 --size-skew $3 > gpurun_out/prof_$1.txt 2>&1
  rc=$?; echo "prof $1 rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  db=$(find /tmp/prof_$1 -name "*.db" | head -1)
  ms=$(python3 -c "import json,sys; print([json.loads(l) for l in open('gpurun_out/prof_$1.txt') if l.startswith('{')][0]['ms_per_step'])")
  python3 tools/prof_summary.py "$db" gpurun_out/prof_$1_summary.txt --window-ms $ms --top 25 > /dev/null
  rm -rf /tmp/prof_$1
done
