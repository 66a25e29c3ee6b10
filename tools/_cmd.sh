set -u
export TMPDIR=/tmp
O=gpurun_out/r04q; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pc.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pc.log 2>&1; rc=$?
tail -25 $O/pc.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for p in 5 6 7 8 5 6; do
  timeout -k 10 300 python bench.py --path $p --steps 50 --warmup 3 --no-cpu --no-e2e > $O/bench_p$p.log 2>&1 || exit $?
  python - $O/bench_p$p.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith("{")][-1]; d=json.loads(l)
print(sys.argv[1], d["ms_per_step"], {k: round(v,3) for k,v in d.get("kernels",{}).items()}, d.get("parity_checked_frames",{}).get("max_abs_ddb_within_100dB"), d.get("parity_checked_frames",{}).get("pass"))
PY
done
