#!/bin/bash
# One entry point for the GPU-box runs (gpurun -- bash tools/gpu.sh RECIPE TAG [ARGS]).
# Every GPU step has its own time limit; the first failing step ends the script.
#   tests  TAG [PYTEST-ARGS...]  pytest -m gpu on the named tests (default: all)
#   bench  TAG [BENCH-ARGS...]   python bench.py ARGS > gpurun_out/TAG/bench.jsonl
#   prof   TAG [BENCH-ARGS...]   rocprofv3 --kernel-trace --stats of bench.py ARGS + kernel table
#   pmc    TAG [BENCH-ARGS...]   four --pmc passes of bench.py ARGS -> gpurun_out/TAG/pmc.md
#   py     TAG SCRIPT [ARGS...]  python SCRIPT ARGS > gpurun_out/TAG/out.txt
#   profpy TAG SCRIPT [ARGS...]  rocprofv3 --kernel-trace --stats of python SCRIPT ARGS + kernel table
#   rate   TAG [CODECS...]       K10 CBR traces (rc_trace.py) per codec + tools/rate_report.py
#   driver TAG                   the driver's bench command (bench.py --gpus 1 --steps 20 --warmup 5)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd)
RECIPE=$1; TAG=${2:-run}; shift 2
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
case "$RECIPE" in
tests)
    timeout -k 10 1000 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu "${@:-tests/}" \
        > "$OUT/pytest.log" 2>&1
    rc=$?; tail -5 "$OUT/pytest.log"
    [ $rc -ne 0 ] && grep -E "FAILED|Error" "$OUT/pytest.log" | tail -20
    # a hung test (pytest-timeout) or a fatal signal in a test process ends the GPU work
    # of the call like a time limit does (gpu_steps.sh stops at 124)
    grep -qE "^E? *Failed: Timeout|Timeout \(>|Fatal Python error|Segmentation fault|Aborted" "$OUT/pytest.log" && exit 124
    exit $rc ;;
bench)
    timeout -k 10 500 python -u bench.py "$@" > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
    rc=$?; tail -1 "$OUT/bench.jsonl"; [ $rc -ne 0 ] && tail -20 "$OUT/bench.err"
    exit $rc ;;
prof)
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" "$@" \
        > "$OUT/prof.log" 2>&1
    rc=$?; cd "$ROOT"
    DB=$(ls "$OUT"/prof/*/run_results.db "$OUT"/prof/run_results.db 2>/dev/null | head -1)
    [ -n "$DB" ] && python tools/rocprof_summary.py "$DB" > "$OUT/kernels.md" && head -40 "$OUT/kernels.md"
    tail -1 "$OUT/prof.log"
    exit $rc ;;
profpy)
    # rocprofv3 --kernel-trace --stats of a python script: profpy TAG SCRIPT [ARGS...]
    SCRIPT=$1; shift
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 "$ROOT/$SCRIPT" "$@" \
        > "$OUT/out.txt" 2> "$OUT/prof.log"
    rc=$?; cd "$ROOT"
    DB=$(ls "$OUT"/prof/*/run_results.db "$OUT"/prof/run_results.db 2>/dev/null | head -1)
    [ -n "$DB" ] && python tools/rocprof_summary.py "$DB" > "$OUT/kernels.md" && head -14 "$OUT/kernels.md"
    tail -3 "$OUT/out.txt"
    exit $rc ;;
rate)
    # K10 traces: rate TAG [CODECS...] - 600 frames of 1080p60 CBR at 8 / 16 Mbit/s on
    # motion and desktop content per codec (default h264 hevc av1), then the report
    CODECS=${@:-h264 hevc av1}
    for codec in $CODECS; do
      for k in 8000 16000; do
        for c in motion desktop; do
          timeout -k 10 300 python -u tools/rc_trace.py --backend hip --codec $codec --frames 600 --content $c \
              --mode cbr --kbps $k --json "$OUT/${codec}_cbr_${c}_${k}.json" >> "$OUT/summary.jsonl" 2>> "$OUT/err.log"
          rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/err.log"; exit $rc; }
        done
      done
    done
    python tools/rate_report.py "$OUT" > "$OUT/rate.md" && cat "$OUT/rate.md" | head -40
    exit 0 ;;
driver)
    # the driver's round-end command (bench.py --gpus 1 --steps 20 --warmup 5) + its kernel profile
    timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
    rc=$?; tail -1 "$OUT/bench.jsonl" | cut -c1-1500; [ $rc -ne 0 ] && { tail -20 "$OUT/bench.err"; exit $rc; }
    exit 0 ;;
pmcpy)
    # the first two counter passes of `pmc` over a python script: pmcpy TAG SCRIPT [ARGS...]
    SCRIPT=$1; shift
    P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
    P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
    cd /tmp && export TMPDIR=/tmp
    i=0; dirs=""
    for P in "$P1" "$P2"; do
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/$SCRIPT" "$@" \
            > "$OUT/p$i.log" 2>&1
        rc=$?; [ $rc -ne 0 ] && { echo "pmc pass $i failed"; tail -5 "$OUT/p$i.log"; exit $rc; }
        dirs="$dirs $(dirname $(ls "$OUT"/p$i/*counter_collection.csv "$OUT"/p$i/*/*counter_collection.csv 2>/dev/null | head -1))"
    done
    cd "$ROOT"
    python tools/pmc_summary.py $dirs > "$OUT/pmc.md" 2>&1; head -40 "$OUT/pmc.md"
    exit 0 ;;
pmc)
    # four counter passes (rocprofv3 does not multiplex: <= 8 SQ, 4 TCC, 2 GRBM per pass)
    P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
    P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
    P3="FETCH_SIZE TCC_HIT"
    P4="WRITE_SIZE TCC_MISS"
    cd /tmp && export TMPDIR=/tmp
    i=0; dirs=""
    for P in "$P1" "$P2" "$P3" "$P4"; do
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/bench.py" "$@" \
            > "$OUT/p$i.log" 2>&1
        rc=$?; [ $rc -ne 0 ] && { echo "pmc pass $i failed"; tail -5 "$OUT/p$i.log"; exit $rc; }
        dirs="$dirs $(dirname $(ls "$OUT"/p$i/*counter_collection.csv "$OUT"/p$i/*/*counter_collection.csv 2>/dev/null | head -1))"
    done
    cd "$ROOT"
    python tools/pmc_summary.py $dirs > "$OUT/pmc.md" 2>&1; head -40 "$OUT/pmc.md"
    exit 0 ;;
py)
    SCRIPT=$1; shift
    timeout -k 10 500 python -u "$SCRIPT" "$@" > "$OUT/out.txt" 2>&1
    rc=$?; tail -30 "$OUT/out.txt"; exit $rc ;;
*)
    echo "unknown recipe $RECIPE"; exit 2 ;;
esac
