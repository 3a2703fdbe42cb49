#!/bin/bash
# every algorithm on the client-batched executor with the round-3 kernels (64 AlexNet3D clients), size skew, config 4
set -o pipefail
mkdir -p gpurun_out/r3ao
export PYTHONUNBUFFERED=1
O=gpurun_out/r3ao/algos.jsonl
: > $O
run() {  # label args...
  local lab=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > gpurun_out/r3ao/$lab.txt 2>&1 || { tail -20 gpurun_out/r3ao/$lab.txt; exit 1; }
  echo "{\"run\": \"$lab\", \"args\": \"$*\", \"result\": $(grep '^{' gpurun_out/r3ao/$lab.txt)}" >> $O
  echo "$lab: $(grep -o '"value": [0-9.]*' gpurun_out/r3ao/$lab.txt) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3ao/$lab.txt)"
}
run salientgrads --steps 8 --warmup 2
run fedavg --algorithm fedavg --steps 8 --warmup 2
run local --algorithm local --steps 8 --warmup 2
run dpsgd --algorithm dpsgd --frac 0.1 --steps 8 --warmup 2
run dispfl --algorithm dispfl --frac 0.1 --steps 6 --warmup 2
run fedfomo --algorithm fedfomo --frac 0.1 --steps 6 --warmup 2
run ditto --algorithm ditto --frac 0.1 --steps 10 --warmup 2
run subavg --algorithm subavg --frac 0.1 --steps 10 --warmup 2
run skew1 --size-skew 1.0 --steps 6 --warmup 2
run skew03 --size-skew 0.3 --steps 6 --warmup 2
run krum128 --algorithm fedprox --aggregator krum --clients 128 --steps 4 --warmup 1
run fedavg8 --algorithm fedavg --clients 8 --steps 20 --warmup 3
