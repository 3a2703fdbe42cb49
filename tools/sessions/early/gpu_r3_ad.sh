#!/bin/bash
# slab forward with the kappa-keyed union swizzle (NIDT_SLAB_KAP=1) vs row-index swizzle: numerics, kbench, LDS PMC
set -o pipefail
mkdir -p gpurun_out/r3ad
export PYTHONUNBUFFERED=1 KBENCH_EVAL=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "slab or fwd_stats or alexnet" > gpurun_out/r3ad/pytest.txt 2>&1
rc=$?; tail -1 gpurun_out/r3ad/pytest.txt; if [ $rc -ne 0 ]; then exit $rc; fi
for arm in 1 0 1 0; do
  export NIDT_SLAB_KAP=$arm
  timeout -k 10 300 python -u tools/kbench.py 64 10 > gpurun_out/r3ad/kbench_$arm.txt 2>&1 || exit 1
  echo "arm $arm: $(grep -E 'full train step|conv2_fwd|conv2_dgrad' gpurun_out/r3ad/kbench_$arm.txt | tr -s ' ' | tr '\n' '|')"
done
for arm in 1 0; do
  export NIDT_SLAB_KAP=$arm
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA \
    --kernel-include-regex "k_conv_fwd_slab" --output-format csv -d gpurun_out/r3ad/pmc$arm -o run -- python3 tools/kbench.py 64 3 \
    > gpurun_out/r3ad/pmc$arm.log 2>&1 || exit 1
  python3 tools/pmc_summary.py gpurun_out/r3ad/pmc$arm gpurun_out/r3ad/pmc_summary_$arm.txt > /dev/null 2>&1
  echo "pmc arm $arm:"; grep -E "^==|derived" gpurun_out/r3ad/pmc_summary_$arm.txt
done
