#!/bin/bash
# stem diagnostics (r3_i), then the conv1 dot-product wgrad A/B with register-prefetched staging (r3_h)
bash tools/sessions/early/gpu_r3_i.sh; rc=$?
echo "r3_i rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/sessions/early/gpu_r3_h.sh
