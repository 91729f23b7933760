#!/bin/bash
# GPU box: hardware counters for the hot kernels, one pass per counter group (rocprofv3
# cannot multiplex: <= 8 SQ, 4 TCC, 2 GRBM per pass). H.264 driver config, then HEVC 1080p.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-pmc}
mkdir -p gpurun_out/$TAG
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P3="FETCH_SIZE TCC_HIT"
P4="WRITE_SIZE TCC_MISS"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/$TAG/h264_p$i -o run -- python3 bench.py --gpus 1 --steps 10 --warmup 3 --e2e-sessions 0 --extra-4k 0 > gpurun_out/$TAG/h264_p$i.log 2>&1 || { echo "h264 pass $i failed"; tail -5 gpurun_out/$TAG/h264_p$i.log; exit 1; }
  echo "h264 pass $i ok"
done
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/$TAG/hevc_p$i -o run -- python3 bench.py --gpus 1 --encoder hevc --sessions 1 --width 3840 --height 2160 --mode fullframe --steps 4 --warmup 2 --e2e-sessions 0 --extra-4k 0 > gpurun_out/$TAG/hevc_p$i.log 2>&1 || { echo "hevc pass $i failed"; tail -5 gpurun_out/$TAG/hevc_p$i.log; exit 1; }
  echo "hevc pass $i ok"
done
