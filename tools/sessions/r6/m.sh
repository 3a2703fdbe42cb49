#!/bin/bash
# AlexNet pack fusion: bit-identity tests, graph-vs-eager tests, bench A/B (64 and 8 clients); sharded-row parity
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6m; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_personalized.py -k "pack_fuse or graphs_bit_identical" tests/test_gpu_kernels.py::test_hip_graph_local_steps_match_eager > $OUT/t.txt 2>&1 || { tail -30 $OUT/t.txt; exit 1; }
tail -1 $OUT/t.txt
for F in 1 0; do
  NIDT_AX_PACK_FUSE=$F timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $OUT/b64_f$F.txt 2>&1 || { tail -20 $OUT/b64_f$F.txt; exit 1; }
  echo "== PACK_FUSE=$F 64"; tail -1 $OUT/b64_f$F.txt | cut -c1-170
  NIDT_AX_PACK_FUSE=$F timeout -k 10 200 python -u bench.py --clients 8 --steps 40 --warmup 5 > $OUT/b8_f$F.txt 2>&1 || { tail -20 $OUT/b8_f$F.txt; exit 1; }
  echo "== PACK_FUSE=$F 8"; tail -1 $OUT/b8_f$F.txt | cut -c1-170
done
bash tools/sessions/r6/l.sh
