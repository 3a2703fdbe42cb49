#!/bin/bash
bash tools/sessions/early/gpu_r3_g.sh; rc=$?
echo "r3_g rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/sessions/early/gpu_r3_m.sh
