#!/bin/bash
# bf16-vs-fp32 convergence ablation (tools/convergence_ablation.py): HIP engine, fp32 reference, fp32 with 1e-6
# perturbed init (chaos control), bf16 autocast on MIOpen
set -o pipefail
mkdir -p gpurun_out/r3e
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u tools/convergence_ablation.py hip fp32 fp32_pert amp_bf16 > gpurun_out/r3e/ablation.txt 2>&1
rc=$?; grep '^{' gpurun_out/r3e/ablation.txt; exit $rc
