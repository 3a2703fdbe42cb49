#!/bin/bash
# r3_f (stem parity, chaos cosines) then r3_h (conv1 wgrad dot A/B) — h only if f ended without a crash/timeout
bash tools/sessions/early/gpu_r3_f.sh; rc=$?
echo "r3_f rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/sessions/early/gpu_r3_h.sh
