#!/bin/bash
# Config 5 steady state: 256 clients, 3 rounds under a kernel trace (summary of the last two rounds = the
# steady window, plus the whole-run table), then PMC passes over the three hottest 3D kernels on a 32-client round.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4l; mkdir -p $OUT
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/c5prof -o run -- python3 -u tools/config5_resnet3d.py \
  --clients 256 --train-per-client 36 --test-per-client 9 --batch 4 --group 32 --rounds 3 --warmup 1 \
  > $OUT/config5.txt 2>&1 || { tail -30 $OUT/config5.txt; exit 1; }
grep '^{' $OUT/config5.txt | cut -c1-600
db=$(find /tmp/c5prof -name "*.db" | head -1)
steady=$(python3 - "$OUT/config5.txt" <<'EOF'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d = json.loads(ln)
print(int(1000 * 2 * d.get("steady_s_per_round", 16.0)))
EOF
)
echo "steady window ms: $steady"
python3 tools/prof_summary.py "$db" $OUT/config5_kernels.txt --top 40 > /dev/null 2>&1
python3 tools/prof_summary.py "$db" $OUT/config5_steady_kernels.txt --top 40 --window-ms "$steady" > /dev/null 2>&1
tail -12 $OUT/config5_steady_kernels.txt
RE='k_conv_fwd_dma|k_conv_wgrad_dma|k_bnr_bwd_apply'
i=0
for C in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
         "FETCH_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex "$RE" --output-format csv \
      -d /tmp/pmc/p$i -o run -- python3 -u tools/config5_resnet3d.py --clients 32 --train-per-client 4 \
      --test-per-client 1 --batch 4 --group 32 --rounds 1 --warmup 0 > $OUT/pmc$i.log 2>&1 \
      || { tail -5 $OUT/pmc$i.log; exit 1; }
done
python3 tools/pmc_summary.py /tmp/pmc $OUT/pmc_summary.txt > /dev/null 2>&1 || true
cat $OUT/pmc_summary.txt
