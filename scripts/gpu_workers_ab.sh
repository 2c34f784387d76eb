#!/bin/bash
# A/B of host worker count for the batched small-LP sections (C3, C4); no CPU baseline.
set -o pipefail
mkdir -p gpurun_out
for w in ${WS:-8 12 16}; do
  timeout -k 10 200 python bench.py --m 2000 --n 10000 --steps 5 --no-cpu --no-c5 \
    --batch-workers $w --c3-workers $w > gpurun_out/ab_w$w.log 2> gpurun_out/ab_w$w.err || { echo "w=$w failed"; tail -20 gpurun_out/ab_w$w.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_w$w.log')); print($w, 'c3', round(d['c3']['value'],1), 'c4', round(d['batched']['value'],1))"
done
