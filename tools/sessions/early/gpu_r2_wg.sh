#!/bin/bash
# wgrad 128-channel blocks: numerics tests, then kbench A/B (64-channel blocks forced vs default) at G=64 and G=8
set -o pipefail
mkdir -p gpurun_out/wg
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad or train_step" \
  > gpurun_out/wg/pytest.txt 2>&1 || { tail -30 gpurun_out/wg/pytest.txt; exit 1; }
tail -2 gpurun_out/wg/pytest.txt
timeout -k 10 200 python -u tools/kbench.py 64 10 > gpurun_out/wg/kb64_new.txt 2>&1 || exit 1
NIDT_WG_NCH=1 timeout -k 10 200 python -u tools/kbench.py 64 10 > gpurun_out/wg/kb64_old.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/kbench.py 8 20 > gpurun_out/wg/kb8_new.txt 2>&1 || exit 1
NIDT_WG_NCH=1 timeout -k 10 200 python -u tools/kbench.py 8 20 > gpurun_out/wg/kb8_old.txt 2>&1 || exit 1
for f in kb64_old kb64_new kb8_old kb8_new; do echo "== $f"; grep -E "step|wgrad" gpurun_out/wg/$f.txt; done
