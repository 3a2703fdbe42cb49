#!/bin/bash
# CIFAR DisPFL (100 clients, G = 100): env sweep of the kernel-choice switches on the end-of-round build, one box,
# arms back to back
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s4h; mkdir -p $OUT
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 -u tools/bench_cifar.py --algorithm dispfl --rounds 2 --warmup 1 > $OUT/$n.txt 2>&1 || { tail -20 $OUT/$n.txt; exit 1; }
  printf "== %-30s %s\n" "$n" "$(tail -1 $OUT/$n.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["s_round_each"])')"
}
run X=0 X=0
run WG_DIRECT=2 NIDT_WG_DIRECT=2
run FWD_KSPLIT=1 NIDT_FWD_KSPLIT=1
run WG_TRI=0 NIDT_WG_TRI=0
run WG_TRI_MINPOS=1e9 NIDT_WG_TRI_MINPOS=1000000000
run WG_NSPLIT_LEGACY=1 NIDT_WG_NSPLIT_LEGACY=1
run 2D_SLAB_BD=0 NIDT_2D_SLAB_BD=0
run GN_HOLD=0 NIDT_GN_HOLD=0
run PACK_WT=1 NIDT_PACK_WT=1
run GN_EPI=1 NIDT_GN_EPI=1
run FORK_GROUP=0 NIDT_FORK_GROUP=0
run X=1 X=1
