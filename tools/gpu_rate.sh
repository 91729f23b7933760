#!/bin/bash
# K10 rate-control traces on one MI355X: 600 frames of 1080p60 H.264 CBR at 8 and
# 16 Mbit/s on motion and desktop content, plus CRF for comparison.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-rate}
mkdir -p $OUT
for k in 8000 16000; do
  for c in motion desktop; do
    timeout -k 10 300 python tools/rc_trace.py --backend hip --frames 600 --content $c --mode cbr --kbps $k \
        --json $OUT/cbr_${c}_${k}.json >> $OUT/summary.jsonl 2>> $OUT/err.log || exit 1
  done
done
for c in motion desktop; do
  timeout -k 10 300 python tools/rc_trace.py --backend hip --frames 600 --content $c --mode crf \
      --json $OUT/crf_${c}.json >> $OUT/summary.jsonl 2>> $OUT/err.log || exit 1
done
cat $OUT/summary.jsonl
