#!/bin/bash
# LDS bank conflicts of the slab conv and the three-tap wgrad with the union-position vs output-space swizzles:
# PMC (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, MFMA busy) per arm, numerics, kbench A/B of the wgrad swizzle
set -o pipefail
export PYTHONUNBUFFERED=1 KBENCH_EVAL=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4p; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "wgrad or slab" > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
RE='k_conv_fwd_slab|k_conv_wgrad_tri'
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES"
for arm in "old NIDT_SLAB_LSWZ=0 NIDT_WGTRI_LSWZ=0" "new NIDT_SLAB_LSWZ=1 NIDT_WGTRI_LSWZ=1"; do
  set -- $arm; name=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex "$RE" --output-format csv \
      -d /tmp/pmc_$name -o run -- python3 tools/kbench.py 64 2 > $OUT/pmc_$name.log 2>&1 || { tail -5 $OUT/pmc_$name.log; exit 1; }
  python3 tools/pmc_summary.py /tmp/pmc_$name $OUT/pmc_$name.txt > /dev/null 2>&1 || true
  echo "== $name"; grep -E "^==|derived" $OUT/pmc_$name.txt
done
kb() {  # name, env..., -- G
  local name=$1; shift; local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python tools/kbench.py "$@" 10 > $OUT/kb_$name.txt 2>&1 || { tail -5 $OUT/kb_$name.txt; exit 1; }
  echo "$name: $(grep 'full train' $OUT/kb_$name.txt | head -1) | $(grep -E '_wgrad' $OUT/kb_$name.txt | tr -s ' ' | tr '\n' ';')"
}
kb g64_w1 NIDT_WGTRI_LSWZ=1 -- 64
kb g64_w0 NIDT_WGTRI_LSWZ=0 -- 64
kb g64_w1b NIDT_WGTRI_LSWZ=1 -- 64
kb g64_w0b NIDT_WGTRI_LSWZ=0 -- 64
kb g8_w1 NIDT_WGTRI_LSWZ=1 -- 8
kb g8_w0 NIDT_WGTRI_LSWZ=0 -- 8
