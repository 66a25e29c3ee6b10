#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace / PMC summaries.
# Every GPU step has its own time limit; a crash/abort/timeout (anything but a plain test
# failure) ends the session so nothing else touches a possibly faulted GPU.
# usage: tools/gpu_session.sh <tag> [steps...]   steps: tests smoke bench driver quick prof pmc sq
#        stamp cfgs pmc5 sweep
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
TAG="${1:-r02}"
shift || true
STEPS="${*:-tests smoke bench prof}"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
FAST="--no-cpu --no-e2e --no-check ${BENCH_EXTRA:-}"  # BENCH_EXTRA: e.g. --path 6 for A/B profiles

run() {  # name seconds cmd...
  local name=$1 to=$2
  shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" >"$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 12 "$OUT/$name.log"
  return $rc
}

for s in $STEPS; do
  case $s in
    tests)
      run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread
      rc=$?
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    tests_k)  # one file/selection: TESTK env
      run pytest_k 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread ${TESTK}
      rc=$?
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    ledger)  # every GPU test, with the tolerance ledger (largest error per check) written
      ZFFT_TOL_LEDGER="$OUT/tol_ledger.json" run pytest_ledger 1100 python -u -m pytest tests -m gpu -q \
        -p no:cacheprovider -rf --timeout 300 --timeout-method thread
      rc=$?
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    smoke)
      run smoke 400 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench)
      run bench 900 python bench.py || exit $? ;;
    driver)  # the driver's own bench command line
      run bench_driver 900 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $? ;;
    quick)
      run quick 300 python bench.py --steps 100 --warmup 3 $FAST || exit $? ;;
    cfgs)
      CHK="--no-cpu --no-e2e"
      run bench_cfg3 300 python bench.py --config cfg3 --steps 50 --warmup 2 $CHK || exit $?
      run bench_cfg5 300 python bench.py --config cfg5 --steps 20 --warmup 2 $CHK || exit $?
      run bench_cfg5_f16 300 python bench.py --config cfg5 --in-dtype complex32 --steps 20 --warmup 2 $CHK || exit $?
      run bench_cfg1 300 python bench.py --config cfg1 --steps 50 --warmup 2 $CHK || exit $?
      run bench_cfg4 300 python bench.py --config cfg4 --steps 50 --warmup 2 $CHK || exit $?
      run bench_cfg2_u8 300 python bench.py --in-dtype cu8 --steps 50 --warmup 2 $CHK || exit $?
      run bench_cfg2_f16 300 python bench.py --in-dtype complex32 --steps 50 --warmup 2 $CHK || exit $? ;;
    pmc5)  # cfg5 traffic, complex64 and fp16 (complex32) IQ storage
      for dt in complex64 complex32; do
        run pmc5_fetch_$dt 300 rocprofv3 --pmc FETCH_SIZE --output-format csv \
          -d "$OUT/pmc5_fetch_$dt" -o run -- python3 "$R/bench.py" --config cfg5 --in-dtype $dt --steps 2 --warmup 1 $FAST || exit $?
        run pmc5_write_$dt 300 rocprofv3 --pmc WRITE_SIZE --output-format csv \
          -d "$OUT/pmc5_write_$dt" -o run -- python3 "$R/bench.py" --config cfg5 --in-dtype $dt --steps 2 --warmup 1 $FAST || exit $?
        python3 "$R/tools/pmc_traffic.py" "$OUT/pmc5_fetch_$dt" "$OUT/pmc5_write_$dt" 2048 cfg5 \
          "$OUT/traffic_cfg5_$dt.json" $dt > "$OUT/traffic5_$dt.log" || exit $?
      done ;;
    sweep)
      run sweep 900 python tools/sweep_schedule.py "$OUT/sweep_schedule.json" || exit $? ;;
    prof)
      run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/prof" -o run -- python3 "$R/bench.py" --steps 20 --warmup 2 $FAST || exit $? ;;
    pmc)
      run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv \
        -d "$OUT/pmc_fetch" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 $FAST || exit $?
      run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv \
        -d "$OUT/pmc_write" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 $FAST || exit $?
      python3 "$R/tools/pmc_traffic.py" "$OUT/pmc_fetch" "$OUT/pmc_write" 4096 cfg2 \
        "$OUT/traffic_cfg2.json" complex64 > "$OUT/traffic.log" || exit $? ;;
    sq)
      run pmc_sq 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU \
        SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT \
        GRBM_GUI_ACTIVE --output-format csv \
        -d "$OUT/pmc_sq" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 $FAST || exit $?
      python3 "$R/tools/sq_counters.py" "$OUT/pmc_sq" 4096 cfg2 complex64 "$OUT/sq_cfg2.json" 299008 \
        > "$OUT/sq.log" || exit $? ;;
    stamp)  # this session's PMC/SQ summaries become the ones bench.py reads (same sources)
      cp "$OUT/traffic_cfg2.json" "$OUT/sq_cfg2.json" "$R/profiles/" || exit $? ;;
    *)
      echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== session done"
