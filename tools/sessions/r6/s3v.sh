#!/bin/bash
# [GN-EPI] kernel times on vs off (CIFAR DisPFL steady round)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s3v; mkdir -p $OUT
for f in 1 0; do
  NIDT_GN_EPI=$f timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/ge_$f -o run -- python3 -u tools/bench_cifar.py --algorithm dispfl --rounds 1 --warmup 1 > $OUT/prof_$f.txt 2>&1 || { tail -20 $OUT/prof_$f.txt; exit 1; }
  db=$(find /tmp/ge_$f -name "*.db" | head -1)
  steady=$(python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/prof_$f.txt') if l.startswith('{')][-1]
print(int(1000*sum(d['s_round_each'])))")
  python3 tools/prof_summary.py "$db" $OUT/k_$f.txt --top 60 --window-ms "$steady" > /dev/null 2>&1
  echo "== gn_epi=$f"; grep -E "gn_fwd|gn_apply|conv_fwd_slab<64, 1, 4, 384|conv_fwd_slab<128, 2, 4, 384|TIMELINE" $OUT/k_$f.txt | cut -c1-150
done
