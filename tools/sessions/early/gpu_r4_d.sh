#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r4d
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "smfmac or conv1_fused" > gpurun_out/r4d/pytest.txt 2>&1 || { tail -40 gpurun_out/r4d/pytest.txt; exit 1; }
tail -3 gpurun_out/r4d/pytest.txt
for mode in 0 1; do
  NIDT_C1WG_SMF=$mode timeout -k 10 200 python tools/kbench.py 64 10 > gpurun_out/r4d/kbench_g64_smf$mode.txt 2>&1 || exit 1
  echo "smf=$mode"; grep -E "full train|conv1_wgrad" gpurun_out/r4d/kbench_g64_smf$mode.txt
done
cd /tmp && export TMPDIR=/tmp
NIDT_C1WG_SMF=1 timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-include-regex "wgrad_smf" -d $GRAFT_REPO_ROOT/gpurun_out/r4d/pmc1 -o pmc -- python $GRAFT_REPO_ROOT/tools/kbench.py 64 2 > $GRAFT_REPO_ROOT/gpurun_out/r4d/pmc1.log 2>&1 || exit 1
NIDT_C1WG_SMF=1 timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE --kernel-include-regex "wgrad_smf" -d $GRAFT_REPO_ROOT/gpurun_out/r4d/pmc2 -o pmc -- python $GRAFT_REPO_ROOT/tools/kbench.py 64 2 > $GRAFT_REPO_ROOT/gpurun_out/r4d/pmc2.log 2>&1 || exit 1
ls -R $GRAFT_REPO_ROOT/gpurun_out/r4d | head
