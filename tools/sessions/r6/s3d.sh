#!/bin/bash
# CIFAR SubAvg upper-bound probes: what removing a kernel family from the step would gain (invalid runs, A/B only)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s3d; mkdir -p $OUT
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 -u tools/debug/cifar_skip_ab.py --algorithm subavg --rounds 3 --warmup 1 > $OUT/$n.txt 2>&1 || { tail -20 $OUT/$n.txt; exit 1; }
  echo "== $n $(tail -1 $OUT/$n.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["s_round_each"], d["phase_s_total"])')"
}
run base X=0
run no_gnpg NIDT_SKIP=gn_param_grads
run no_resgrad NIDT_SKIP=res_grad,res_grad_s2
run no_gnbwd NIDT_SKIP=gn_bwd,gn_param_grads
run no_gnfwd NIDT_SKIP=gn_fwd
run base2 X=1
