#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/abort/timeout (anything but a plain
# test failure) ends the session so nothing else touches a possibly faulted GPU.
# usage: tools/gpu_session.sh <tag> [steps...]   steps: tests smoke bench prof pmc
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
TAG="${1:-r01}"
shift || true
STEPS="${*:-tests smoke bench prof}"
OUT="$R/gpurun_out"
mkdir -p "$OUT"

run() {  # name seconds cmd...
  local name=$1 to=$2
  shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" >"$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "$OUT/$name.log"
  return $rc
}

for s in $STEPS; do
  case $s in
    tests)
      run pytest_gpu 1100 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 120 --timeout-method thread
      rc=$?
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    smoke)
      run smoke 400 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench)
      run bench 600 python bench.py --steps 10 --warmup 2 --cpu-seconds 8 || exit $? ;;
    ab)
      run bench_exact 300 python bench.py --steps 5 --warmup 1 --no-cpu --path 1 || exit $?
      run bench_fused 300 python bench.py --steps 5 --warmup 1 --no-cpu --path 2 || exit $?
      run bench_xt 300 python bench.py --steps 5 --warmup 1 --no-cpu --path 3 || exit $? ;;
    sweep)
      for blk in 512 1024 2048 4096; do
        run sweep_b$blk 300 python bench.py --steps 5 --warmup 1 --no-cpu --block $blk || exit $?
      done ;;
    bench5)
      run bench_cfg5_f32 600 python bench.py --config cfg5 --steps 5 --warmup 1 --no-cpu || exit $?
      run bench_cfg5_f16 600 python bench.py --config cfg5 --steps 5 --warmup 1 --no-cpu --in-dtype complex32 || exit $?
      run bench_cfg2_f16 600 python bench.py --steps 5 --warmup 1 --no-cpu --in-dtype complex32 || exit $?
      run bench_cfg2_u8 600 python bench.py --steps 5 --warmup 1 --no-cpu --in-dtype cu8 || exit $? ;;
    bench3)
      run bench_cfg3 600 python bench.py --config cfg3 --steps 10 --warmup 2 --no-cpu || exit $? ;;
    prof)
      export TMPDIR=/tmp
      run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu || exit $? ;;
    pmc)
      export TMPDIR=/tmp
      run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv \
        -d "$OUT/pmc_fetch_$TAG" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu || exit $?
      run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv \
        -d "$OUT/pmc_write_$TAG" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu || exit $?
      python3 "$R/tools/pmc_traffic.py" "$OUT/pmc_fetch_$TAG" "$OUT/pmc_write_$TAG" 4096 cfg2 \
        "$OUT/traffic_cfg2_$TAG.json" xa > /dev/null || exit $? ;;
    *)
      echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== session done"
